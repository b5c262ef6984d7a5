"""Where the HIP runtime puts kernel arguments in this process ("The
control-kernel fault").
usage: [HIP_FORCE_DEV_KERNARG=0|1] python scripts/kernarg_probe.py (r02: this runtime put them in
device memory either way, so control_kernel takes its parameter block from a device slot)"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raftd_amd.engine import load_library  # noqa: E402

L = load_library()
fn = L.rg_debug_kernarg_placement
fn.argtypes = [C.c_int32, C.POINTER(C.c_uint64), C.POINTER(C.c_int32)]
addr, dev = C.c_uint64(), C.c_int32()
rc = fn(0, C.byref(addr), C.byref(dev))
print(f"HIP_FORCE_DEV_KERNARG={os.environ.get('HIP_FORCE_DEV_KERNARG')} rc={rc} kernarg={addr.value:#x} "
      f"device_memory={dev.value}")
sys.exit(0 if rc == 0 else 1)
