#!/bin/bash
# Round 2 first pass: DPP probe, park smoke, GPU parity suite, kbench A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r02b}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/bin/dpp_probe > $out/dpp_probe.json 2>&1
echo "dpp_probe rc=$?"; cat $out/dpp_probe.json
timeout -k 10 120 python3 -u tools/park_smoke.py > $out/park_smoke.log 2>&1
rc=$?; echo "park_smoke rc=$rc"; cat $out/park_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u tools/kbench.py --config cfg3 --spp 64 --reps 2 --var "" --var ZRT_PARK=2 --var ZRT_PARK=1 \
   --var ZRT_PARK=2,ZRT_PARK_T=16 --var ZRT_PARK=2,ZRT_PARK_T=32 --var ZRT_PARK=2,ZRT_PARK_T=48 \
   --var ZRT_PARK=2,ZRT_PARK_R=16 --var ZRT_PARK=2,ZRT_PARK_R=48 > $out/kbench_cfg3.log 2>&1
rc=$?; echo "kbench cfg3 rc=$rc"; cat $out/kbench_cfg3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u tools/kbench.py --config cfg5 --spp 32 --reps 2 --var "" --var ZRT_PARK=2 --var ZRT_PARK=1 > $out/kbench_cfg5.log 2>&1
rc=$?; echo "kbench cfg5 rc=$rc"; cat $out/kbench_cfg5.log
exit $rc
