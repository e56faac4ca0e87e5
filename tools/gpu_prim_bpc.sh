#!/bin/bash
# Primary launch grid (blocks per CU) with two pass sets and the lead
# full spp, one process per config, 2 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-primbpc}
mkdir -p $out
log=$out/primbpc.log
: > $log
export ZRT_LIB=tools/bin/sets/libzrt.so
for rep in 1 2; do
  for c in cfg3 cfg5 cfg2; do
    timeout -k 10 400 python -u tools/kbench.py --config $c --spp 0 --reps 2 \
        --var ZRT_PRIM_BPC=7 --var ZRT_PRIM_BPC=6 --var ZRT_PRIM_BPC=5 \
        --var ZRT_PRIM_BPC=4 --var ZRT_PRIM_BPC=3 2>&1 \
      | grep mrays | sed "s/^/{\"cfg\": \"$c\"} /" >> $log || { cat $log; exit 1; }
  done
done
cat $log
