#!/bin/bash
# Direct-pipeline fused checks: kernel trace of one rank tile (check every 20 steps), the
# convergence / direct / persistent / multi-process GPU tests, and the convergence table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/pcd -o run -- python -u tools/prof_conv_direct.py 512 8 > gpurun_out/pcd.log 2>&1 || exit 1
grep check= gpurun_out/pcd.log
python tools/seq_trace.py $(ls /tmp/pcd/*/*.db /tmp/pcd/*.db 2>/dev/null | head -1) > gpurun_out/pcd_seq.txt
head -4 gpurun_out/pcd_seq.txt
export TESTK="direct or convergence or persistent or fused or ipc"
bash tools/gpu.sh tests-k mp convtable || exit $?
grep "|" gpurun_out/convtable.log
