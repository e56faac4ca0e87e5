#!/bin/bash
# Full GPU pass: parity tests -> headline bench -> rocprofv3 kernel trace ->
# FETCH_SIZE/WRITE_SIZE passes.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-r01}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; cat $out/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/prof_bench.json 2> $out/prof_bench.err
rc=$?; echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $out/pmc_$c -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $out/pmc_$c.json 2> $out/pmc_$c.err
  rc=$?; echo "pmc $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
find $out -name "*kernel_stats.csv" -exec cat {} \;
