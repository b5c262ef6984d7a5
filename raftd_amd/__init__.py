"""raftd-amd: MI355X-native batched Raft step engine for raftd's hot path.

The product is the C-ABI library raftd_amd/libraftgpu.so (include/raftgpu.h); raftd_amd.engine
is its Python binding. See DESIGN.md.
"""
from .engine import Engine, RgError, default_config, load_library  # noqa: F401

__all__ = ["Engine", "RgError", "default_config", "load_library"]
