#!/bin/bash
set -o pipefail
export HEAT2D_NO_BUILD=1
mkdir -p gpurun_out
for i in 1 2 3; do for pw in 0.3 1.0 0.05; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --prewarm-s $pw > gpurun_out/pw.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/pw.json')); print('prewarm $pw', '%.4e' % d['value'], ['%.1f' % (x*1e6) for x in d['repeats_s']])"
done; done
