#!/bin/bash
set -o pipefail
export HEAT2D_NO_BUILD=1
mkdir -p gpurun_out
for i in 1 2; do for sm in 2 0 1 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --sync-mode $sm > gpurun_out/sm.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/sm.json')); print('sync_mode $sm', '%.4e' % d['value'], ['%.1f' % (x*1e6) for x in d['repeats_s']])"
done; done
