#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
echo "== conv_continue $(date +%T)"
timeout -k 10 300 python -u tools/conv_continue.py > gpurun_out/conv_continue.log 2>&1; rc=$?
cat gpurun_out/conv_continue.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
bash tools/gpu.sh convtable bench20 bench1000 || exit $?
cat gpurun_out/convtable.log
bash tools/r5_host.sh
