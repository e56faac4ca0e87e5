cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r05w
for v in "" "ZRT_SETS=3" "ZRT_SETS=4" "ZRT_SETS=3 ZRT_LEAD=0" "ZRT_SETS=1"; do
  env $v ZRT_LIB=tools/bin/setsenv/libzrt.so timeout -k 10 300 python3 -u tools/rank_time.py --config cfg3 --ranks 1,8 --reps 2 2>&1 | sed "s/^/{\"var\": \"$v\"} /" >> gpurun_out/r05w/rank_sets.log || exit 1
done
cat gpurun_out/r05w/rank_sets.log
