#!/bin/bash
# A/B at full spp (tools/gpu_ab_full.sh), then the GPU tests on the working tree.
#   LIBS="base:tools/bin/base/libzrt.so new:" bash tools/gpu_abt.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-abt}
mkdir -p $out
bash tools/gpu_ab_full.sh ${1:-abt} || exit $?
[ "${SKIP_TESTS:-0}" = 1 ] && exit 0
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > $out/pytest_gpu.log 2>&1
rc=$?; tail -3 $out/pytest_gpu.log; exit $rc
