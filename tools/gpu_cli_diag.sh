#!/bin/bash
# Small-frame diagnosis: the CLI's 3-spp 1080p render, 5 runs (stages), one
# run under rocprofv3 kernel trace, and first/second/third render in-process.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=$PWD/gpurun_out/${1:-clidiag}
mkdir -p $out
export TMPDIR=/tmp
python3 -c "
from zig_raytracing_contest_amd import scenes
scenes.write_gltf(scenes.get_scene('contest'), '$out/contest.gltf')
" || exit 1
cp config.json $out/
cd $out
for i in 1 2 3 4 5; do
  timeout -k 10 120 ../../zig_raytracing_contest_amd/bin/zrt --in contest.gltf --out o.png --height 1080 --camera "Camera 1" > l$i.log 2>&1 || exit $?
  echo "$(grep -E 'Compiled|Rendered|Rays|Done' l$i.log | sed 's/info: //' | tr '\n' ' ')"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d prof -o run -- \
  ../../zig_raytracing_contest_amd/bin/zrt --in contest.gltf --out o.png --height 1080 --camera "Camera 1" > lp.log 2>&1 || exit $?
grep -E 'Rendered|Done' lp.log
find prof -name "*kernel_stats.csv" -exec cat {} \;
cd ../..
timeout -k 10 120 python3 tools/first_render.py || exit $?
rm -f $out/*.bin
