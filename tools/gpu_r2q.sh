#!/bin/bash
# Park-kernel round profile (s_memtime per round, -DZRT_SWEEP builds) of the
# previous commit's build vs the working tree, cfg3 64 spp and cfg5 32 spp;
# then one SQ counter pass on the working tree (issue ports per launch type).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r02q}
mkdir -p $out
export TMPDIR=/tmp
for c in "cfg3 64" "cfg5 32"; do
  set -- $c
  for lib in old new; do
    if [ $lib = old ]; then L=tools/bin/old/sweep.so; else L=tools/bin/sweep/libzrt.so; fi
    ZRT_LIB=$L timeout -k 10 200 python3 -u tools/kbench.py --config $1 --spp $2 --reps 1 --var ZRT_PARK_PROFILE=1 \
      > $out/prof_${1}_$lib.log 2>&1
    rc=$?; echo "prof $1 $lib rc=$rc"; grep -v "^W\|^E" $out/prof_${1}_$lib.log
    [ $rc -eq 0 ] || exit $rc
  done
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU \
    --kernel-trace --output-format csv -d $out/sq/p1 -o run -- python3 tools/kbench.py --config cfg3 --spp 64 --reps 1 > $out/sq/p1.log 2>&1
rc=$?; echo "sq rc=$rc"; exit $rc
