#!/bin/bash
# VERDICT r5 #3 experiment: per-bounce park time and L2 hit of cfg5 (and
# cfg3) with the bounce queues ordered by the Morton code of the paths'
# origins inside each XCD region (-DZRT_OSORT_EXP build, ZRT_OSORT=1; one
# stream), against the same build without the ordering.
#   bash tools/gpu_osort_exp.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-osort}
mkdir -p $out
export TMPDIR=/tmp
L=tools/bin/osort/libzrt.so
for cfg in ${CFGS:-cfg5 cfg3}; do
  for mode in base sort; do
    d=$out/${cfg}_$mode
    mkdir -p $d
    if [ $mode = sort ]; then E="ZRT_OSORT=1 ZRT_OSORT_FROM=${FROM:-1}"; else E=""; fi
    env $E ZRT_LIB=$L timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv \
        -d $d/pmc_l2 -o run -- python3 bench.py --config $cfg --one-set --steps 1 --warmup 0 --no-cpu-baseline \
        --no-wall-clock > $d/bench.json 2> $d/bench.err
    rc=$?; echo "$cfg $mode rc=$rc"; [ $rc -eq 0 ] || { tail -5 $d/bench.err; exit $rc; }
    python3 tools/l2_bounce.py $d/pmc_l2 > $d/l2_bounce.txt
    grep -o '"img_sha1": "[0-9a-f]*"' $d/bench.json | head -1
  done
done
