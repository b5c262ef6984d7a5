set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python scripts/ctl_profile.py build_variants/ctlprof.so 4096 > gpurun_out/ctlprof_4k.log 2>&1 && \
timeout -k 10 200 python scripts/ctl_profile.py build_variants/ctlprof.so 65536 > gpurun_out/ctlprof_64k.log 2>&1
rc=$?; tail -8 gpurun_out/ctlprof_4k.log gpurun_out/ctlprof_64k.log; exit $rc
