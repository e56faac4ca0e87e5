#!/bin/bash
# one-process A/B sweep of env variants on cfg3 (args: kbench --var values)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
args=()
for v in "$@"; do args+=(--var "$v"); done
timeout -k 10 500 python -u tools/kbench.py --spp 64 --reps 2 "${args[@]}" > gpurun_out/sweep.log 2>&1
rc=$?; cat gpurun_out/sweep.log; exit $rc
