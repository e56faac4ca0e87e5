#!/bin/bash
# Small frames: park kernel (default) vs lane walk (FLAGS=2) for the bounce
# launches, one process per config, at a few sample counts.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-small}
mkdir -p $out
log=$out/small.log
: > $log
for spec in cfg1:1 cfg1:16 cfg2:1 cfg2:4 cfg3:1 cfg3:3 cfg3:8 cfg5:3; do
  c=${spec%%:*}; n=${spec#*:}
  timeout -k 10 120 python -u tools/kbench.py --config $c --spp $n --reps 5 --var "" --var FLAGS=2 --var "" --var FLAGS=2 2>&1 \
    | grep mrays | sed "s/^/{\"cfg\": \"$c\", \"spp\": $n} /" >> $log || { cat $log; exit 1; }
done
cat $log
