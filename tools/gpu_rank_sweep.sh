#!/bin/bash
# The 8-rank cfg3 tile set's per-rank frame time under pass-set / lead
# settings: tools/rank_time.py on a -DZRT_SETS_ENV build.
#   bash tools/gpu_rank_sweep.sh TAG   (LIB=tools/bin/setsenv/libzrt.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-ranks}
mkdir -p $out
L=${LIB:-tools/bin/setsenv/libzrt.so}
timeout -k 10 200 python -u tools/rank_time.py --ranks 1,8 > $out/rank_default.log 2>&1 || exit 1
for v in ${VARS:-"ZRT_SETS=1" "ZRT_SETS=2,ZRT_LEAD=0" "ZRT_SETS=2,ZRT_LEAD=35" "ZRT_SETS=3" "ZRT_SETS=4"}; do
  env $(echo $v | tr ',' ' ') ZRT_LIB=$L timeout -k 10 200 python -u tools/rank_time.py --ranks 8 2>&1 \
    | sed "s/^/{\"var\": \"$v\"} /" >> $out/rank_sweep.log || exit 1
done
cat $out/rank_default.log $out/rank_sweep.log | cut -c1-400
