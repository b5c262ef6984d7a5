#!/bin/bash
# Build an experimental variant of the engine library (ablations; never the product path).
# usage: bash scripts/build_variant.sh OUT.so -DFLAG ...
set -e
cd "$(dirname "$0")/.."
python -m raftd_amd.build --variant "$@"
