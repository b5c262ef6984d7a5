set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for a in "4096 256" "4096 0" "65536 256"; do echo "== $a"; timeout -k 10 200 python3 scripts/ctl_profile.py ab/ctlprof.so $a || exit 1; done 2>&1 | tee gpurun_out/r06f_ctl_profile.txt
