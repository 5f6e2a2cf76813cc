#!/bin/bash
set -o pipefail
export HEAT2D_NO_BUILD=1
mkdir -p gpurun_out
for i in 1 2 3; do for tb in 7 8; do
  timeout -k 10 120 python bench.py --steps 1000 --warmup 200 --tblock $tb > gpurun_out/tb.json 2>gpurun_out/tb.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/tb.json')); print('tblock $tb', '%.4e' % d['value'], '%.3f us/step' % (d['ms_per_step']*1e3))"
done; done
