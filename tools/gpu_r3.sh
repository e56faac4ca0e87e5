#!/bin/bash
# Round-3 GPU pass: parity tests -> headline bench (+ wall clock, CPU
# baseline) -> roofline profiles (one-stream bench under rocprofv3) per config.
# Stops at the first failure.   tools/gpu_r3.sh <tag> [configs...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-r03}
shift
cfgs=${*:-cfg3}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
timeout -k 10 900 python3 bench.py > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; cat $out/bench.json
[ $rc -eq 0 ] || exit $rc
fi
for c in $cfgs; do
  bash tools/gpu_roofline.sh $tag $c || exit $?
done
