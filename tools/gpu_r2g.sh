#!/bin/bash
# A/B in one process per config (product build) + the sweep build's round profile.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r02g}
mkdir -p $out
export TMPDIR=/tmp
for cfg in "cfg3 64" "cfg5 32" "cfg2 64"; do
  set -- $cfg
  timeout -k 10 300 python3 -u tools/kbench.py --config $1 --spp $2 --reps 3 --var "" --var FLAGS=2 --var FLAGS=4 > $out/kbench_$1.log 2>&1
  rc=$?; echo "kbench $1 rc=$rc"; cat $out/kbench_$1.log
  [ $rc -eq 0 ] || exit $rc
done
ZRT_LIB=tools/bin/sweep/libzrt.so timeout -k 10 300 python3 -u tools/kbench.py --config cfg3 --spp 64 --reps 1 --var ZRT_PARK_PROFILE=1 \
   --var ZRT_PARK_PROFILE=1,ZRT_PARK_T=16,ZRT_PARK_R=16 --var ZRT_PARK_PROFILE=1,ZRT_PARK_T=8,ZRT_PARK_R=24 > $out/prof_cfg3.log 2>&1
rc=$?; echo "profile rc=$rc"; cat $out/prof_cfg3.log
exit $rc
