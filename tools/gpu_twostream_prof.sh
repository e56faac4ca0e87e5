#!/bin/bash
# rocprofv3 kernel trace of the headline bench command itself (two pass sets
# on two streams: the kernels overlap, so their summed durations exceed the
# frame; DESIGN.md 5.7 reports the exclusive one-stream profile instead).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-twostream}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-wall-clock > $out/bench.json 2> $out/bench.err
rc=$?; echo "twostream prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats_twostream.csv \;
cat $out/kernel_stats_twostream.csv | cut -c1-200
