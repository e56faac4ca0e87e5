#!/bin/bash
# Park-kernel round profile (ZRT_SWEEP build, s_memtime per round):
# walk / test / refill cycles and counts, cfg3 64 spp and cfg5 32 spp.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-pp}
mkdir -p $out
for c in "cfg3 64" "cfg5 32"; do
  set -- $c
  ZRT_LIB=${PLIB:-tools/bin/sweep/libzrt.so} ZRT_PARK_PROFILE=1 timeout -k 10 200 python -u tools/kbench.py --config $1 --spp $2 --reps 1 --var "" \
    > $out/pp_$1.log 2>&1 || { tail $out/pp_$1.log; exit 1; }
  grep -h "zrt_park_profile\|zrt_primary_profile\|mrays" $out/pp_$1.log | tail -3
done
