#!/bin/bash
# A/B of library builds + environment settings at the configs' full sample
# counts, alternating processes, 2 rounds:
#   SPECS="name:libpath:ENV=V,ENV2=W ..." CFGS="cfg3 cfg2 cfg5" bash tools/gpu_ab_env.sh TAG
# (an empty libpath = the working tree's library; images must be identical)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-abenv}
mkdir -p $out
log=$out/ab.log
: > $log
for c in ${CFGS:-cfg3 cfg2 cfg5}; do
  for rep in 1 2; do
    for spec in $SPECS; do
      name=${spec%%:*}; rest=${spec#*:}; L=${rest%%:*}; envs=${rest#*:}
      [ "$envs" = "$rest" ] && envs=""
      env ZRT_LIB=$L ${envs//,/ } timeout -k 10 300 python -u tools/kbench.py --config $c --spp 0 --reps 2 --var "" 2>&1 \
        | grep mrays | sed "s/^/{\"lib\": \"$name\", \"cfg\": \"$c\"} /" >> $log || { cat $log; exit 1; }
    done
  done
done
cat $log
