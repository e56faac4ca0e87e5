#!/bin/bash
# Lead samples with two pass sets: ZRT_LEAD % of a pass moved from the last
# pass to the first (tools/bin/sets: -DZRT_SETS_ENV), full spp, one process
# per config, 2 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-lead}
mkdir -p $out
log=$out/lead.log
: > $log
export ZRT_LIB=tools/bin/sets/libzrt.so
for rep in 1 2; do
  for c in cfg3 cfg5 cfg2; do
    timeout -k 10 400 python -u tools/kbench.py --config $c --spp 0 --reps 2 \
        --var ZRT_LEAD=${LEADS_A:-0} --var ZRT_LEAD=12 --var ZRT_LEAD=16 --var ZRT_LEAD=20 --var ZRT_LEAD=25 --var ZRT_LEAD=30 --var ZRT_LEAD=40 2>&1 \
      | grep mrays | sed "s/^/{\"cfg\": \"$c\"} /" >> $log || { cat $log; exit 1; }
  done
done
cat $log
