#!/bin/bash
# Staggered pass-set start and small frames (tools/bin/sets: -DZRT_SETS_ENV):
# kbench at full spp (cfg3, cfg2), cfg3 at the CLI's 3 spp, then the CLI
# itself with 1 vs 2 sets (LD_LIBRARY_PATH overrides the CLI's RUNPATH).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-stagger}
mkdir -p $out
log=$out/stagger.log
: > $log
export ZRT_LIB=tools/bin/sets/libzrt.so
for rep in 1 2; do
  for c in cfg3 cfg2; do
    timeout -k 10 300 python -u tools/kbench.py --config $c --spp 0 --reps 2 \
        --var ZRT_SETS=2 --var ZRT_SETS=2,ZRT_STAGGER=1 --var ZRT_SETS=3,ZRT_STAGGER=1 2>&1 \
      | grep mrays | sed "s/^/{\"cfg\": \"$c\"} /" >> $log || { cat $log; exit 1; }
  done
done
unset ZRT_LIB
for rep in 1 2; do
  for spec in old:tools/bin/old/libzrt.so new:; do
    name=${spec%%:*}; L=${spec#*:}
    ZRT_LIB=$L timeout -k 10 300 python -u tools/kbench.py --config cfg3 --spp 0 --reps 3 --var "" 2>&1 \
      | grep mrays | sed "s/^/{\"lib\": \"$name\", \"cfg\": \"cfg3\"} /" >> $log || { cat $log; exit 1; }
  done
done
export ZRT_LIB=tools/bin/sets/libzrt.so
timeout -k 10 300 python -u tools/kbench.py --config cfg3 --spp 3 --reps 5 \
    --var ZRT_SETS=1 --var ZRT_SETS=2 --var ZRT_SETS=1 --var ZRT_SETS=2 2>&1 \
  | grep mrays | sed "s/^/{\"cfg\": \"cfg3 3spp\"} /" >> $log || { cat $log; exit 1; }
unset ZRT_LIB
python3 -c "
from zig_raytracing_contest_amd import scenes
scenes.write_gltf(scenes.get_scene('contest'), '$out/contest.gltf')
" || exit 1
cp config.json $out/
cd $out
for i in 1 2 3 4; do
  for n in 1 2; do
    LD_LIBRARY_PATH=../../tools/bin/sets ZRT_SETS=$n timeout -k 10 120 ../../zig_raytracing_contest_amd/bin/zrt \
        --in contest.gltf --out o$n.png --height 1080 --camera "Camera 1" > l.log 2>&1 || exit $?
    echo "sets=$n $(grep -E 'Rendered|Done' l.log | sed 's/info: //' | tr '\n' ' ')" >> stagger.log
  done
done
rm -f *.bin contest.gltf
cmp o1.png o2.png && echo "cli images identical" >> stagger.log
cat stagger.log
