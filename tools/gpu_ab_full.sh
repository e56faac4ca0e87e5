#!/bin/bash
# A/B of library builds at the configs' full sample counts (multi-pass frames):
# cfg3 256 spp, cfg2 64 spp, cfg5 512 spp; alternating processes, 2 rounds.
#   LIBS="old:tools/bin/old/libzrt.so new:" [CFGS="cfg3 cfg2 cfg5"] [VARS="FLAGS=48"] [ROUNDS=2] bash tools/gpu_ab_full.sh TAG
# VARS: extra kbench variants per process (FLAGS=48: one stream + per-kernel ms)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-abfull}
mkdir -p $out
log=$out/ab.log
: > $log
LIBS=${LIBS:-"old:tools/bin/old/libzrt.so new:"}
vargs=""
for v in $VARS; do vargs="$vargs --var $v"; done
for c in ${CFGS:-cfg3 cfg2 cfg5}; do
  for rep in $(seq ${ROUNDS:-2}); do
    for spec in $LIBS; do
      name=${spec%%:*}; L=${spec#*:}
      ZRT_LIB=$L timeout -k 10 300 python -u tools/kbench.py --config $c --spp 0 --reps 2 --var "" $vargs 2>&1 \
        | grep mrays | sed "s/^/{\"lib\": \"$name\", \"cfg\": \"$c\"} /" >> $log || { cat $log; exit 1; }
    done
  done
done
cat $log
