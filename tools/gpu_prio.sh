#!/bin/bash
# Stream priority of the second pass set (tools/bin/sets: -DZRT_SETS_ENV reads
# ZRT_PRIO: -1 = the device's greatest priority, 1 = its least), full spp,
# one process per variant (the stream is created once per context), 2 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-prio}
mkdir -p $out
log=$out/prio.log
: > $log
export ZRT_LIB=tools/bin/sets/libzrt.so
for rep in 1 2; do
  for c in cfg3 cfg5 cfg2; do
    for v in "" ZRT_PRIO=-1 ZRT_PRIO=1; do
      timeout -k 10 400 python -u tools/kbench.py --config $c --spp 0 --reps 2 --var "$v" 2>&1 \
        | grep mrays | sed "s/^/{\"cfg\": \"$c\", \"prio\": \"$v\"} /" >> $log || { cat $log; exit 1; }
    done
  done
done
cat $log
