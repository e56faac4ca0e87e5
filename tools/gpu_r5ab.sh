#!/bin/bash
# Round-5 variant A/B: full-spp frames per library (tools/gpu_ab_full.sh) and
# the 1- / 8-rank tile sets of cfg3 (tools/rank_time.py) per library.
#   LIBS="base:tools/bin/base/libzrt.so x:tools/bin/x/libzrt.so" RLIBS="base:... x:..." bash tools/gpu_r5ab.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-r05ab}
out=gpurun_out/$tag
mkdir -p $out
if [ -n "$LIBS" ]; then
  bash tools/gpu_ab_full.sh $tag || exit 1
fi
for spec in $RLIBS; do
  name=${spec%%:*}; L=${spec#*:}
  ZRT_LIB=$L timeout -k 10 300 python3 -u tools/rank_time.py --config cfg3 --ranks 1,8 --reps 2 \
      > $out/rank_time_$name.log 2>&1
  rc=$?; echo "rank_time $name rc=$rc"; cat $out/rank_time_$name.log; [ $rc -eq 0 ] || exit $rc
done
