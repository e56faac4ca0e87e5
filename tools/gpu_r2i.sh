#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r02i}
mkdir -p $out
export TMPDIR=/tmp
V=""
for t in 8 12 16 24; do for r in 4 8 16; do V="$V --var ZRT_PARK_T=$t,ZRT_PARK_R=$r"; done; done
ZRT_LIB=tools/bin/sweep/libzrt.so timeout -k 10 300 python3 -u tools/kbench.py --config cfg3 --spp 64 --reps 2 --var "" $V \
   --var ZRT_PARK_PROFILE=1 > $out/sweep_cfg3.log 2>&1
rc=$?; echo "sweep cfg3 rc=$rc"; cat $out/sweep_cfg3.log
[ $rc -eq 0 ] || exit $rc
ZRT_LIB=tools/bin/sweep/libzrt.so timeout -k 10 300 python3 -u tools/kbench.py --config cfg5 --spp 32 --reps 2 --var "" \
   --var ZRT_PARK_T=16,ZRT_PARK_R=8 --var ZRT_PARK_T=24,ZRT_PARK_R=8 --var ZRT_PARK_T=16,ZRT_PARK_R=4 --var ZRT_PARK_PROFILE=1 > $out/sweep_cfg5.log 2>&1
rc=$?; echo "sweep cfg5 rc=$rc"; cat $out/sweep_cfg5.log
exit $rc
