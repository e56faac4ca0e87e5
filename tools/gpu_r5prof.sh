#!/bin/bash
# Round-5 profiling pass:
#   1. rocprofv3 kernel trace of the two-stream bench frame (cfg3) -> timeline
#      with the critical path attributed per kernel (tools/timeline.py);
#   2. the cfg5 one-stream roofline profile (tools/gpu_roofline.sh);
#   3. a kernel trace of the 1- and 8-rank tile sets of cfg3 on one GPU
#      (tools/rank_time.py), every rank's frame summarised.
#   tools/gpu_r5prof.sh <tag> [steps...]   steps: two roof5 rank8 (default: all)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-r05b}
shift
steps=${*:-two roof5 rank8}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for s in $steps; do
case $s in
two)
  cmd="python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-wall-clock"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/two -o run -- \
      $cmd > $out/two_bench.json 2> $out/two_bench.err
  rc=$?; echo "two-stream trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tr=$(find $out/two -name "*kernel_trace.csv" | head -1)
  python3 tools/timeline.py $tr --frame 0 --command "rocprofv3 --kernel-trace --stats -- $cmd" \
      --out $out/timeline_twostream_cfg3.json > $out/timeline_twostream_cfg3.txt
  python3 tools/timeline.py $tr --all > $out/timeline_frames_cfg3.log
  cat $out/timeline_twostream_cfg3.txt $out/timeline_frames_cfg3.log
  find $out/two -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats_twostream_cfg3.csv \;
  ;;
roof5)
  bash tools/gpu_roofline.sh $tag cfg5 || exit 1
  ;;
rank8)
  cmd="python3 -u tools/rank_time.py --config cfg3 --ranks 1,8 --reps 1"
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $out/rank8 -o run -- \
      $cmd > $out/rank_time_cfg3.log 2> $out/rank_time_cfg3.err
  rc=$?; echo "rank8 trace rc=$rc"; cat $out/rank_time_cfg3.log; [ $rc -eq 0 ] || exit $rc
  tr=$(find $out/rank8 -name "*kernel_trace.csv" | head -1)
  python3 tools/timeline.py $tr --all > $out/rank8_frames_cfg3.log
  cat $out/rank8_frames_cfg3.log
  ;;
esac
done
