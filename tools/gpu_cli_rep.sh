#!/bin/bash
# CLI wall clock, host vs device grid build, alternating, 4 runs each
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/cli
python3 -c "
from zig_raytracing_contest_amd import scenes
scenes.write_gltf(scenes.get_scene('contest'), 'gpurun_out/cli/contest.gltf')
" || exit 1
cp config.json gpurun_out/cli/
cd gpurun_out/cli
for i in 1 2 3 4; do
  for db in 0 1; do
    ZRT_DEVICE_BUILD=$db timeout -k 10 120 ../../zig_raytracing_contest_amd/bin/zrt --in contest.gltf --out o$db.png --height 1080 --camera "Camera 1" > l.log 2>&1 || exit $?
    echo "device_build=$db $(grep -E 'Compiled|Uploaded|Done' l.log | sed 's/info: //' | tr '\n' ' ')"
  done
done
rm -f *.bin
