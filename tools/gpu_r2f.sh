#!/bin/bash
# Park-kernel profile (ZRT_SWEEP build: round cycles) and the brick-skip A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r02f}
mkdir -p $out
export TMPDIR=/tmp
SW=tools/bin/sweep/libzrt.so
for cfg in "cfg3 64" "cfg5 32"; do
  set -- $cfg
  ZRT_LIB=$SW timeout -k 10 300 python3 -u tools/kbench.py --config $1 --spp $2 --reps 2 --var "" --var ZRT_PARK_SKIP=1 \
     --var ZRT_PARK_PROFILE=1 --var ZRT_PARK_PROFILE=1,ZRT_PARK_SKIP=1 > $out/kbench_$1.log 2>&1
  rc=$?; echo "kbench $1 rc=$rc"; cat $out/kbench_$1.log
  [ $rc -eq 0 ] || exit $rc
done
