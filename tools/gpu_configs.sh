#!/bin/bash
# Every BASELINE config at its own size on one GPU (render wall time,
# tools/kbench.py): the default kernels, then FLAGS=2 (ZRT_FLAG_LANE_WALK:
# wf_kernel for every launch, the round-1 path) in the same process; then the
# CLI end to end (tools/gpu_cli.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-configs}
mkdir -p $out
log=$out/configs.log
: > $log
for c in cfg1 cfg2 cfg3 cfg5 cfg4; do
  r=2; [ $c = cfg4 ] && r=1
  timeout -k 10 300 python -u tools/kbench.py --config $c --spp 0 --reps $r --var "" --var "FLAGS=2" >> $log 2>&1 || { cat $log; exit 1; }
  echo "^ $c" >> $log
done
cat $log
bash tools/gpu_cli.sh
