#!/bin/bash
# Park schedule (test_min T x refill_min R) re-swept with two pass sets in
# flight (tools/bin/sets: -DZRT_SETS_ENV reads ZRT_PARK_T / ZRT_PARK_R, no
# stamps), full spp, one process per config, 2 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-tr}
mkdir -p $out
log=$out/tr.log
: > $log
export ZRT_LIB=tools/bin/sets/libzrt.so
for rep in 1 2; do
  for c in cfg3 cfg5 cfg2; do
    timeout -k 10 400 python -u tools/kbench.py --config $c --spp 0 --reps 2 \
        --var ZRT_PARK_T=12,ZRT_PARK_R=16 --var ZRT_PARK_T=8,ZRT_PARK_R=16 --var ZRT_PARK_T=16,ZRT_PARK_R=16 \
        --var ZRT_PARK_T=12,ZRT_PARK_R=12 --var ZRT_PARK_T=12,ZRT_PARK_R=24 2>&1 \
      | grep mrays | sed "s/^/{\"cfg\": \"$c\"} /" >> $log || { cat $log; exit 1; }
  done
done
cat $log
