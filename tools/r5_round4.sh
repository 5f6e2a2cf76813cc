#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TESTK="direct or convergence or persistent or fused or ipc"
bash tools/gpu.sh tests-k mp convtable || exit $?
grep "|" gpurun_out/convtable.log
