#!/bin/bash
# Start-up split of the zrt CLI: tools/startup_probe.py plus
# three CLI runs with ZRT_TIMING=1 (context creation's stages).
#   bash tools/gpu_startup.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-startup}
mkdir -p $out
timeout -k 10 300 python -u tools/startup_probe.py --runs ${RUNS:-5} > $out/startup.log 2>&1 || { tail $out/startup.log; exit 1; }
tmp=$(mktemp -d)
python -c "import sys; sys.path.insert(0, '$PWD'); from zig_raytracing_contest_amd import scenes; scenes.write_gltf(scenes.get_scene('contest'), '$tmp/c.gltf')"
cp config.json $tmp/
for i in 1 2 3; do
  (cd $tmp && ZRT_TIMING=1 timeout -k 10 60 $OLDPWD/zig_raytracing_contest_amd/bin/zrt --in c.gltf --out o.png --height 1080 --camera "Camera 1") >> $out/cli_timing.log 2>&1 || exit 1
done
rm -rf $tmp
tail -1 $out/startup.log
