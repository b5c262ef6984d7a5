# Head-page rows, the four row words loaded together: the C5 A/B against the page-table build.
set -o pipefail
LIBS="raftd_amd/libraftgpu.so diag/nohp.so" AB_TIMEOUT=300 bash scripts/ab_lib.sh --groups 1048576 --entries 1 --steps 10 --warmup 3 || exit 1
