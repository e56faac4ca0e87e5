#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace/--stats only).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-r01}
shift
out=gpurun_out/pmc/$tag
mkdir -p $out
export TMPDIR=/tmp
rocprofv3 -L > $out/counters_list.txt 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --stats --output-format csv -d $out/p$i -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $out/p${i}_bench.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
