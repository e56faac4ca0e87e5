#!/bin/bash
# Re-sweep of the schedule knobs on the current tree (-DZRT_SETS_ENV build:
# ZRT_PARK_T / ZRT_PARK_R / ZRT_LEAD / ZRT_SETS from the environment), every
# variant in one process per config and round (tools/kbench.py, full spp).
#   bash tools/gpu_knobs.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-knobs}
mkdir -p $out
log=$out/knobs.log
: > $log
L=${LIB:-tools/bin/setsenv/libzrt.so}
V=${VARS:-"ZRT_PARK_T=12 ZRT_PARK_T=16 ZRT_PARK_R=16 ZRT_PARK_R=24 ZRT_LEAD=15 ZRT_LEAD=25"}
vargs='--var ""'
for c in ${CFGS:-cfg3 cfg5 cfg2}; do
  for rep in $(seq ${ROUNDS:-2}); do
    args=(--var "")
    for v in $V; do args+=(--var "$v"); done
    ZRT_LIB=$L timeout -k 10 600 python -u tools/kbench.py --config $c --spp 0 --reps 2 "${args[@]}" 2>&1 \
      | grep mrays | sed "s/^/{\"cfg\": \"$c\", \"round\": $rep} /" >> $log || { cat $log; exit 1; }
  done
done
cat $log | cut -c1-160
