#!/bin/bash
# Persistent-path validation after a planner change: the persistent / direct / convergence GPU tests,
# the multi-process tests, the strong-scaling proxy, and the driver's N=4 / N=8 command rehearsed on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TESTK="persistent or direct or pstream or convergence or fused or ipc"
bash tools/gpu.sh tests-k mp proxy rehearse4 rehearse8 || exit $?
grep "N=" gpurun_out/proxy.log
tail -1 gpurun_out/rehearse4.log | cut -c1-400
tail -1 gpurun_out/rehearse8.log | cut -c1-400
