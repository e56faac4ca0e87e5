#!/bin/bash
# round-1 check: parity (non-park), A/B sweep, then the park tests last
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: rc=$1"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests -m gpu -k "not park" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; ok $rc
timeout -k 10 300 python tools/kbench.py --spp 64 --reps 2 --var "" --var ZRT_BMASK=0 --var ZRT_WF_MINW=7 --var ZRT_MODE=mega > gpurun_out/sweep12.log 2>&1
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/sweep12.log; ok $rc
ZRT_DEBUG=1 timeout -k 10 200 python -u -m pytest tests -m gpu -k "park" -x -q --timeout 60 --timeout-method thread > gpurun_out/pytest_park.log 2>&1
rc=$?; echo "park rc=$rc"; tail -15 gpurun_out/pytest_park.log
exit $rc
