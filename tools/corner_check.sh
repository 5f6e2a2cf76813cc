#!/bin/bash
# Unit balance of the streaming launch (tools/timeline.py --units), the bench, its kernel trace,
# the whole GPU suite, and the strong-scaling proxy (persistent plans share the edge weights).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/timeline.py 4096x4096:7:70 2048x4096:7:70 --json gpurun_out/tl_units.json --units \
  > gpurun_out/tl_units.log 2>&1 || exit 1
grep "K=7" gpurun_out/tl_units.log | tail -3
bash tools/gpu.sh bench20 bench1000 prof tests-nox proxy
