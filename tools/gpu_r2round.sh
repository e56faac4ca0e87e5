#!/bin/bash
# Full GPU pass: parity tests -> headline bench (+ wall clock, CPU baseline)
# -> rocprofv3 kernel trace -> FETCH_SIZE / WRITE_SIZE passes -> SQ/TCC
# counter passes per launch type (kbench cfg3 64 spp).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-r02}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 900 python3 bench.py > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; cat $out/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-wall-clock > $out/prof_bench.json 2> $out/prof_bench.err
rc=$?; echo "rocprof rc=$rc"; cat $out/prof_bench.json
[ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $out/pmc_$c -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-wall-clock > $out/pmc_$c.json 2> $out/pmc_$c.err
  rc=$?; echo "pmc $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
i=0
mkdir -p $out/sq
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $out/sq/p$i -o run -- \
      python3 tools/kbench.py --config cfg3 --spp 64 --reps 1 > $out/sq/p$i.log 2>&1
  rc=$?; echo "sq pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
find $out/prof -name "*kernel_stats.csv" -exec cat {} \;
