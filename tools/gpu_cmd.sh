#!/bin/bash
# run an arbitrary python command on the GPU box with a time limit; output to gpurun_out/cmd.log
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 ${TMO:-600} "$@" > gpurun_out/cmd.log 2>&1
rc=$?; echo "rc=$rc"; tail -40 gpurun_out/cmd.log
exit $rc
