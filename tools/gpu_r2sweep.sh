#!/bin/bash
# Park-kernel schedule sweep (kbench, one process per config; images must stay identical).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r02d}
mkdir -p $out
export TMPDIR=/tmp
V3=""
for t in 4 8 12 16; do for r in 8 16; do V3="$V3 --var ZRT_PARK=2,ZRT_PARK_T=$t,ZRT_PARK_R=$r"; done; done
timeout -k 10 600 python3 -u tools/kbench.py --config cfg3 --spp 64 --reps 2 --var "" $V3 \
   --var ZRT_PARK=1,ZRT_PARK_T=8,ZRT_PARK_R=8 --var ZRT_PARK=1,ZRT_PARK_T=16,ZRT_PARK_R=16 \
   --var ZRT_WF_DEBUG=1 --var ZRT_PARK=2,ZRT_PARK_T=8,ZRT_PARK_R=16,ZRT_WF_DEBUG=1 --var ZRT_PARK=1,ZRT_PARK_T=8,ZRT_PARK_R=16,ZRT_WF_DEBUG=1 > $out/kbench_cfg3.log 2>&1
rc=$?; echo "kbench cfg3 rc=$rc"; grep -v zrt_launch $out/kbench_cfg3.log
[ $rc -eq 0 ] || exit $rc
V5=""
for t in 4 8 16; do for r in 8 16; do V5="$V5 --var ZRT_PARK=2,ZRT_PARK_T=$t,ZRT_PARK_R=$r"; done; done
timeout -k 10 600 python3 -u tools/kbench.py --config cfg5 --spp 32 --reps 2 --var "" $V5 \
   --var ZRT_PARK=1,ZRT_PARK_T=8,ZRT_PARK_R=16 > $out/kbench_cfg5.log 2>&1
rc=$?; echo "kbench cfg5 rc=$rc"; cat $out/kbench_cfg5.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u tools/kbench.py --config cfg2 --spp 64 --reps 2 --var "" --var ZRT_PARK=2,ZRT_PARK_T=8,ZRT_PARK_R=16 \
   --var ZRT_PARK=1,ZRT_PARK_T=8,ZRT_PARK_R=16 > $out/kbench_cfg2.log 2>&1
rc=$?; echo "kbench cfg2 rc=$rc"; cat $out/kbench_cfg2.log
exit $rc
