#!/bin/bash
# Counter availability + LDS/issue counters of the park kernel (one-stream bench, cfg3)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-lds}
shift   # the rest are counter groups, one rocprofv3 pass each
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $out/avail.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*LDS[A-Z_0-9]*\|SQ_INST[A-Z_0-9]*\|SQ_WAIT[A-Z_0-9]*\|TA_[A-Z_0-9]*BUSY[A-Z_0-9]*\|SQ_BUSY[A-Z_0-9]*" $out/avail.txt | sort -u > $out/names.txt || true
cmd="python3 bench.py --config cfg3 --one-set --steps 1 --warmup 0 --no-cpu-baseline --no-wall-clock"
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $out/p$i -o run -- $cmd > $out/p$i.log 2>&1
  echo "pass $i rc=$?"
done
