#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r02l}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python3 -u tools/park_smoke.py > $out/park_smoke.log 2>&1
rc=$?; echo "park_smoke rc=$rc"; cat $out/park_smoke.log
[ $rc -eq 0 ] || exit $rc
for cfg in "cfg3 64" "cfg5 32" "cfg2 64"; do
  set -- $cfg
  timeout -k 10 300 python3 -u tools/kbench.py --config $1 --spp $2 --reps 3 --var "" --var FLAGS=8 --var FLAGS=2 > $out/kbench_$1.log 2>&1
  rc=$?; echo "kbench $1 rc=$rc"; cat $out/kbench_$1.log
  [ $rc -eq 0 ] || exit $rc
done
ZRT_LIB=tools/bin/sweep/libzrt.so timeout -k 10 300 python3 -u tools/kbench.py --config cfg3 --spp 64 --reps 1 --var ZRT_PARK_PROFILE=1 \
  --var ZRT_PARK_T=8 --var ZRT_PARK_T=16 --var ZRT_PARK_T=20 --var ZRT_PARK_R=12 --var ZRT_PARK_R=20 > $out/prof_cfg3.log 2>&1
rc=$?; echo "prof rc=$rc"; cat $out/prof_cfg3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log
exit $rc
