#!/bin/bash
# occupancy A/B on whatever box this is: cfg3 at 256 spp, default vs 6 waves/SIMD
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
log=gpurun_out/minw_${1:-x}.log
{ hostname; rocm-smi --showclocks 2>/dev/null | grep -E "sclk|mclk|fclk" | head -4; } > $log 2>&1
timeout -k 10 300 python -u tools/kbench.py --spp ${2:-256} --reps 2 --var "" --var ZRT_WF_MINW=6 \
    --var ZRT_WF_MINW=6,ZRT_WF_MINW0=7 --var "" >> $log 2>&1
rc=$?; cat $log; exit $rc
