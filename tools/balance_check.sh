#!/bin/bash
# Unit balance of the direct pipeline (halo units sized with their wait), the per-rank
# strong-scaling proxy, the bench, and the whole GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/timeline.py 2048x4096:7:70:direct 2048x4096:8:72:direct 1024x4096:7:70:direct \
  --json gpurun_out/tl_direct.json --units > gpurun_out/tl_direct.log 2>&1 || exit 1
grep "==" gpurun_out/tl_direct.log
python tools/unit_balance.py gpurun_out/tl_direct.json 2
bash tools/gpu.sh proxy bench20 bench1000 tests-nox
