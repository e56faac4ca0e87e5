#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r02k}
mkdir -p $out
export TMPDIR=/tmp
for cfg in "cfg3 64" "cfg5 32"; do
  set -- $cfg
  ZRT_LIB=tools/bin/sweep/libzrt.so timeout -k 10 300 python3 -u tools/kbench.py --config $1 --spp $2 --reps 2 --var "" \
     --var ZRT_PARK_SKIP=8 --var ZRT_PARK_SKIP=16 --var ZRT_PARK_SKIP=24 --var ZRT_PARK_SKIP=32 --var ZRT_PARK_SKIP=48 \
     --var ZRT_PARK_PROFILE=1,ZRT_PARK_SKIP=24 > $out/skip_$1.log 2>&1
  rc=$?; echo "skip $1 rc=$rc"; cat $out/skip_$1.log
  [ $rc -eq 0 ] || exit $rc
done
