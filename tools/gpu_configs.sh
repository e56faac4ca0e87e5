#!/bin/bash
# Every BASELINE config at its own size on one GPU (render wall time, tools/kbench.py),
# then the CLI end to end (tools/gpu_cli.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
log=gpurun_out/configs.log
: > $log
for c in cfg1 cfg2 cfg3 cfg5 cfg4; do
  r=2; [ $c = cfg4 ] && r=1
  timeout -k 10 240 python -u tools/kbench.py --config $c --spp 0 --reps $r --var "" >> $log 2>&1 || { cat $log; exit 1; }
  echo "^ $c" >> $log
done
cat $log
bash tools/gpu_cli.sh
