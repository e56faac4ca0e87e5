#!/bin/bash
# rocprofv3 passes of ONE bench command with exclusive kernel durations
# (bench.py --one-set: every pass on one HIP stream), for
# tools/roofline_profile.py: kernel trace + stats, SQ VALU counters, L2 hit,
# FETCH_SIZE, WRITE_SIZE (separate --pmc passes; no trace domains beside --pmc).
#   tools/gpu_roofline.sh <tag> [config]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-r03}
cfg=${2:-cfg3}
out=gpurun_out/$tag/roof_$cfg
mkdir -p $out
export TMPDIR=/tmp
cmd="python3 bench.py --config $cfg --one-set --steps 1 --warmup 0 --no-cpu-baseline --no-wall-clock"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    $cmd > $out/prof_bench.json 2> $out/prof_bench.err
rc=$?; echo "roof $cfg trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for grp in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  case $i in 1) d=pmc_sq1;; 2) d=pmc_l2;; 3) d=pmc_FETCH_SIZE;; 4) d=pmc_WRITE_SIZE;; esac
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $out/$d -o run -- \
      $cmd > $out/$d.json 2> $out/$d.err
  rc=$?; echo "roof $cfg pmc $d rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/roofline_profile.py $out --config $cfg --command "$cmd" --out $out/roofline_$cfg.json > /dev/null
find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats_$cfg.csv \;
echo "roof $cfg done"
