#!/bin/bash
# PMC passes over a kbench run (one counter group per rocprofv3 run,
# --kernel-trace only).  usage: gpu_pmc_kb.sh TAG "KBENCH ARGS" GROUP...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1; kb=$2; shift 2
out=gpurun_out/pmc/$tag
mkdir -p $out
export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $out/p$i -o run -- \
      python3 tools/kbench.py $kb > $out/p${i}.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
