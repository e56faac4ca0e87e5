#!/bin/bash
# parity (all GPU tests) then an A/B sweep of the XCD split
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/kbench.py --spp 64 --reps 2 --var "" --var ZRT_XCD=1 --var "" --var ZRT_XCD=1 > gpurun_out/sweep13.log 2>&1
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/sweep13.log
exit $rc
