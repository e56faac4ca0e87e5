#!/bin/bash
# L2 hit rate per launch (so per bounce) of one one-stream frame: a kernel
# trace for the durations and one --pmc pass of TCC_HIT/TCC_MISS (no trace
# domains beside --pmc).  tools/l2_bounce.py pairs them per dispatch.
#   tools/gpu_l2_bounce.sh <tag> [config]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-r05bf}
cfg=${2:-cfg5}
out=gpurun_out/$tag/l2_$cfg
mkdir -p $out
export TMPDIR=/tmp
cmd="python3 bench.py --config $cfg --one-set --steps 1 --warmup 0 --no-cpu-baseline --no-wall-clock"
timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $out/pmc_l2 -o run -- \
    $cmd > $out/pmc_l2.json 2> $out/pmc_l2.err
rc=$?; echo "l2 $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/l2_bounce.py $out/pmc_l2 > $out/l2_bounce_$cfg.txt && cat $out/l2_bounce_$cfg.txt
