#!/bin/bash
# parity tests (fast) then a variant sweep
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python tools/kbench.py "$@" > gpurun_out/sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/sweep.log | tail -20
exit $rc
