#!/bin/bash
# pass sets x lead on the current kernels (-DZRT_SETS_ENV build), full spp, one process per config
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-sets}
mkdir -p $out
for c in cfg3 cfg5 cfg2; do
  ZRT_LIB=tools/bin/setsenv/libzrt.so timeout -k 10 400 python -u tools/kbench.py --config $c --spp 0 --reps 2 \
    --var "ZRT_SETS=2,ZRT_LEAD=20" --var "ZRT_SETS=3,ZRT_LEAD=20" --var "ZRT_SETS=3,ZRT_LEAD=35" \
    --var "ZRT_SETS=2,ZRT_LEAD=10" --var "ZRT_SETS=2,ZRT_LEAD=30" --var "ZRT_SETS=4,ZRT_LEAD=20" --var "ZRT_SETS=2,ZRT_LEAD=20" \
    > $out/sets_$c.log 2>&1 || { tail $out/sets_$c.log; exit 1; }
  grep mrays $out/sets_$c.log
done
