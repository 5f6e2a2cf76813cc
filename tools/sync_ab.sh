#!/bin/bash
# Interleaved A/B of the engine's end-of-run synchronisation in the driver's bench command:
# sync_mode 1 (event + spin on hipEventQuery) vs 2 (hipStreamSynchronize), five runs each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for r in 1 2 3 4 5; do
  for m in 1 2; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --sync-mode $m > gpurun_out/sync_ab_$m.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/sync_ab_$m.json').read().strip().splitlines()[-1]); print('mode $m run $r', round(d['ms_per_step']*1e3, 3), 'us/step')"
  done
done
