#!/bin/bash
# Build an experimental variant of the engine library (ablations; never the product path).
# usage: bash scripts/build_variant.sh OUT.so -DFLAG ...
set -e
OUT=$1; shift
cd "$(dirname "$0")/../raftd_amd/csrc"
SRCS="raftgpu_kernels.hip raftgpu_admin.hip raftgpu_wire.hip raftgpu_apply.hip raftgpu_engine.cpp"
OBJS=""
for f in $SRCS; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 "$@" -c -x hip $f -o /tmp/var_${f%.*}.o
  OBJS="$OBJS /tmp/var_${f%.*}.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $OBJS
