#!/bin/bash
# Build an experimental variant of the engine library (ablations; never the product path).
# usage: bash scripts/build_variant.sh OUT.so -DFLAG ...
set -e
OUT=$1; shift
cd "$(dirname "$0")/../raftd_amd/csrc"
OBJS=""
for f in raftgpu_kernels.hip raftgpu_admin.hip raftgpu_wire.hip raftgpu_apply.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 "$@" -c -x hip $f -o /tmp/var_${f%.*}.o
  OBJS="$OBJS /tmp/var_${f%.*}.o"
done
for f in raftgpu_engine.cpp raftgpu_rccl.cpp raftgpu_sdma.cpp; do  # host-only runtime (raftd_amd/build.py)
  /opt/rocm/bin/hipcc -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -O3 -fPIC -std=c++17 "$@" -c $f -o /tmp/var_${f%.*}.o
  OBJS="$OBJS /tmp/var_${f%.*}.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $OBJS -ldl
