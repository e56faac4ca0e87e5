#!/bin/bash
# f2 check: device grid build parity + CLI wall clock with both builds
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_grid_build_gpu.py -x -q -s --timeout 120 --timeout-method thread > gpurun_out/pytest_f2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -14 gpurun_out/pytest_f2.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_cli.sh
