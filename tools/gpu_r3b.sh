#!/bin/bash
# Round-3 measurement batch: headline bench, sweep-build round profiles
# (park + primary), then an A/B of the given libraries (cfg3, cfg2, cfg5).
#   LIBS="base: x:tools/bin/x/libzrt.so" bash tools/gpu_r3b.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-r03b}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python3 bench.py > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 400 $out/bench.json
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_parkprof.sh $tag || exit $?
if [ -n "$LIBS" ]; then
  bash tools/gpu_ab_full.sh $tag || exit $?
fi
