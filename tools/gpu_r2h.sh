#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r02h}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python3 -u tools/park_smoke.py > $out/park_smoke.log 2>&1
rc=$?; echo "park_smoke rc=$rc"; cat $out/park_smoke.log
[ $rc -eq 0 ] || exit $rc
for cfg in "cfg3 64" "cfg5 32" "cfg2 64"; do
  set -- $cfg
  timeout -k 10 300 python3 -u tools/kbench.py --config $1 --spp $2 --reps 3 --var "" --var FLAGS=8 --var FLAGS=2 --var FLAGS=4 > $out/kbench_$1.log 2>&1
  rc=$?; echo "kbench $1 rc=$rc"; cat $out/kbench_$1.log
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log
exit $rc
