#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (no PMC in this pass).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
tag=${1:-r01}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$tag -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof/${tag}_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof/${tag}_bench.log
find gpurun_out/prof/$tag -name "*stats*" | head
exit $rc
