#!/bin/bash
# Shade-kernel phase profile (ZRT_SWEEP builds, s_memtime + active lanes per
# phase, zrt_shade_profile) for several sweep libraries, cfg3 64 spp:
#   LIBS="name:path ..." bash tools/gpu_shadeprof.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-sp}
mkdir -p $out
for spec in ${LIBS:-sweep:tools/bin/sweep/libzrt.so}; do
  name=${spec%%:*}; L=${spec#*:}
  ZRT_LIB=$L ZRT_PARK_PROFILE=1 timeout -k 10 200 python -u tools/kbench.py --config ${CFG:-cfg3} --spp ${SPP:-64} --reps 1 --var "" \
    > $out/sp_$name.log 2>&1 || { tail $out/sp_$name.log; exit 1; }
  echo "== $name"; grep -h "zrt_shade_profile\|mrays" $out/sp_$name.log | tail -2
done
