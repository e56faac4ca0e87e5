#!/bin/bash
# A/B (tools/gpu_ab.sh, no tests) + the sweep build's R / T sweep on cfg3 64 spp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r02s}
mkdir -p $out
SKIP_TESTS=1 bash tools/gpu_ab.sh ${1:-r02s} || exit 1
ZRT_LIB=tools/bin/sweep/libzrt.so timeout -k 10 300 python3 -u tools/kbench.py --config cfg3 --spp 64 --reps 1 --var ZRT_PARK_PROFILE=1 \
  --var ZRT_PARK_T=8 --var ZRT_PARK_T=16 --var ZRT_PARK_T=20 --var ZRT_PARK_R=12 > $out/sweep_cfg3.log 2>&1
rc=$?; echo "sweep rc=$rc"; grep -v "^W\|^E" $out/sweep_cfg3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -3 $out/pytest_gpu.log; exit $rc
