#!/bin/bash
# CLI end-to-end on the GPU box: write the contest scene as glTF, render with zrt.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/cli
python3 -c "
from zig_raytracing_contest_amd import scenes
scenes.write_gltf(scenes.get_scene('contest'), 'gpurun_out/cli/contest.gltf')
scenes.write_gltf(scenes.get_scene('cornell'), 'gpurun_out/cli/cornell.gltf')
" || exit 1
cp config.json gpurun_out/cli/
cd gpurun_out/cli
timeout -k 10 300 ../../zig_raytracing_contest_amd/bin/zrt --in contest.gltf --out contest.png --height 1080 --camera "Camera 1" > zrt_contest.log 2>&1
rc=$?; cat zrt_contest.log; echo "zrt rc=$rc"
[ $rc -eq 0 ] || exit $rc
ZRT_DEVICE_BUILD=0 timeout -k 10 300 ../../zig_raytracing_contest_amd/bin/zrt --in contest.gltf --out contest_dev.png --height 1080 --camera "Camera 1" > zrt_contest_dev.log 2>&1
rc=$?; cat zrt_contest_dev.log; echo "zrt (host build + upload) rc=$rc"
[ $rc -eq 0 ] || exit $rc
cmp contest.png contest_dev.png && echo "built-into-context and host grid builds: identical PNG"
rc=$?
rm -f *.bin
exit $rc
