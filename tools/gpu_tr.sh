#!/bin/bash
# Park schedule sweep (ZRT_SWEEP build reads ZRT_PARK_T / ZRT_PARK_R), one
# process per config, every variant image-checked against the first.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-tr}
mkdir -p $out
V=""
for t in 8 12 16 20; do for r in 12 16 24; do V="$V --var ZRT_PARK_T=$t,ZRT_PARK_R=$r"; done; done
for c in "cfg3 64" "cfg5 32"; do
  set -- $c
  ZRT_LIB=tools/bin/sweep/libzrt.so timeout -k 10 400 python -u tools/kbench.py --config $1 --spp $2 --reps 2 $V \
    > $out/tr_$1.log 2>&1 || { tail $out/tr_$1.log; exit 1; }
  grep mrays $out/tr_$1.log
done
