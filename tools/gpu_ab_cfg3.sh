cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r03t; mkdir -p $out; log=$out/ab.log; : > $log
for rep in 1 2 3; do for spec in old:tools/bin/old/libzrt.so comb:tools/bin/comb/libzrt.so base: ; do
  name=${spec%%:*}; L=${spec#*:}
  ZRT_LIB=$L timeout -k 10 300 python -u tools/kbench.py --config cfg3 --spp 0 --reps 2 --var "" 2>&1 | grep mrays | sed "s/^/{\"lib\": \"$name\", \"cfg\": \"cfg3\"} /" >> $log || exit 1
done; done
cat $log
