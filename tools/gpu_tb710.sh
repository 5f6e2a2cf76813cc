#!/bin/bash
set -o pipefail
export HEAT2D_NO_BUILD=1
mkdir -p gpurun_out
for i in 1 2 3; do for tb in 7 10; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --tblock $tb > gpurun_out/tb.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/tb.json')); print('20 steps tblock $tb', '%.4e' % d['value'], ['%.1f' % (x*1e6) for x in d['repeats_s']])"
done; done
