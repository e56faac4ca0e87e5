#!/bin/bash
# Pass sets in flight (streams) 1-4 at the configs' full spp, one process per
# config (tools/bin/sets: render.hip built with -DZRT_SETS_ENV), 2 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-sets}
mkdir -p $out
log=$out/sets.log
: > $log
for rep in 1 2; do
  for c in cfg3 cfg2 cfg5; do
    ZRT_LIB=tools/bin/sets/libzrt.so timeout -k 10 400 python -u tools/kbench.py --config $c --spp 0 --reps 2 \
        --var ZRT_SETS=2 --var ZRT_SETS=1 --var ZRT_SETS=3 --var ZRT_SETS=4 2>&1 \
      | grep mrays | sed "s/^/{\"cfg\": \"$c\"} /" >> $log || { cat $log; exit 1; }
  done
done
cat $log
