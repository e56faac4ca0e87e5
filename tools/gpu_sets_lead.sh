#!/bin/bash
# Pass sets x lead (tools/bin/sets: -DZRT_SETS_ENV reads ZRT_SETS, ZRT_LEAD),
# full spp, one process per config, 2 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-setslead}
mkdir -p $out
log=$out/setslead.log
: > $log
export ZRT_LIB=tools/bin/sets/libzrt.so
for rep in 1 2; do
  for c in cfg3 cfg5 cfg2; do
    timeout -k 10 400 python -u tools/kbench.py --config $c --spp 0 --reps 2 \
        --var ZRT_SETS=2,ZRT_LEAD=20 --var ZRT_SETS=3,ZRT_LEAD=20 --var ZRT_SETS=3,ZRT_LEAD=35 \
        --var ZRT_SETS=3,ZRT_LEAD=50 2>&1 \
      | grep mrays | sed "s/^/{\"cfg\": \"$c\"} /" >> $log || { cat $log; exit 1; }
  done
done
cat $log
