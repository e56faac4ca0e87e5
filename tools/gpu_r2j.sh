#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r02j}
mkdir -p $out
export TMPDIR=/tmp
ZRT_LIB=tools/bin/sweep/libzrt.so timeout -k 10 300 python3 -u tools/kbench.py --config cfg3 --spp 64 --reps 2 --var "" \
   --var ZRT_PARK_BLOCK=768 --var ZRT_PARK_BLOCK=512 --var ZRT_PARK_BLOCK=256 \
   --var ZRT_PARK_PROFILE=1,ZRT_PARK_BLOCK=512 > $out/occ_cfg3.log 2>&1
rc=$?; echo "occ cfg3 rc=$rc"; cat $out/occ_cfg3.log
exit $rc
