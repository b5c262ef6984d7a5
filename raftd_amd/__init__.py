"""raftd-amd: MI355X-native batched Raft step engine for raftd's hot path.

The product is the C-ABI library raftd_amd/libraftgpu.so (include/raftgpu.h); raftd_amd.engine
is its Python binding. See DESIGN.md.
"""
import os

# Kernel arguments in host memory (HIP_FORCE_DEV_KERNARG=0), set before anything initialises HIP.
# Device-memory kernel arguments are the suspected cause of the intermittent control-kernel
# faults (DESIGN.md §3 "The control-kernel fault"). An explicit setting in the environment wins.
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "0")

from .engine import Engine, RgError, default_config, load_library  # noqa: F401

__all__ = ["Engine", "RgError", "default_config", "load_library"]
