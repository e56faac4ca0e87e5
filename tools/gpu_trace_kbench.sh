#!/bin/bash
# rocprofv3 kernel trace of a kbench run (per-dispatch durations)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-kb}; shift
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag -o run -- \
    python3 tools/kbench.py "$@" > gpurun_out/$tag/kbench.log 2>&1
rc=$?; echo "rc=$rc"; cat gpurun_out/$tag/kbench.log | grep -v "^W2026"
exit $rc
