#!/bin/bash
# Round-4 GPU pass: parity tests -> headline bench -> per-rank tile times
# (N = 1, 2, 4, 8 on one GPU) for the listed configs.  Stops at the first
# failure.   tools/gpu_r4.sh <tag> [rank-time configs...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-r04}
shift
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
for c in "$@"; do
  timeout -k 10 600 python3 -u tools/rank_time.py --config $c > $out/rank_time_$c.log 2>&1
  rc=$?; echo "rank_time $c rc=$rc"; cat $out/rank_time_$c.log
  [ $rc -eq 0 ] || exit $rc
done
