#!/bin/bash
# A/B of library builds, alternating processes on one box: cfg3 64 spp, cfg5
# 32 spp, cfg2 64 spp; then the GPU parity tests on the working tree's build.
#   LIBS="old:tools/bin/old/libzrt.so new:" bash tools/gpu_ab.sh TAG
# (an empty path = the working tree's zig_raytracing_contest_amd/libzrt.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-ab}
mkdir -p $out
log=$out/ab.log
: > $log
LIBS=${LIBS:-"old:tools/bin/old/libzrt.so new:"}
for c in "cfg3 64" "cfg5 32" "cfg2 64"; do
  set -- $c
  for rep in 1 2; do
    for spec in $LIBS; do
      name=${spec%%:*}; L=${spec#*:}
      ZRT_LIB=$L timeout -k 10 200 python -u tools/kbench.py --config $1 --spp $2 --reps 2 --var "" 2>&1 \
        | grep mrays | sed "s/^/{\"lib\": \"$name\", \"cfg\": \"$1\"} /" >> $log || { cat $log; exit 1; }
    done
  done
done
cat $log
[ "${SKIP_TESTS:-0}" = 1 ] && exit 0
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > $out/pytest_gpu.log 2>&1
rc=$?; tail -3 $out/pytest_gpu.log; exit $rc
