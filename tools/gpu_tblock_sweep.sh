#!/bin/bash
# Driver-style bench (20 steps) and 1000 steps at several halo depths (chunk depths) K.
set -o pipefail
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1
for tb in 5 6 7 8 10 12; do
  for st in 20 1000; do
    timeout -k 10 120 python bench.py --steps $st --warmup 5 --tblock $tb > gpurun_out/tb.json 2>gpurun_out/tb.err || { echo "failed tb=$tb"; tail -3 gpurun_out/tb.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/tb.json')); print('tblock $tb steps $st', '%.4e' % d['value'], '%.3f us/step' % (d['ms_per_step']*1e3), ['%.1f' % (x*1e6) for x in d['repeats_s']])"
  done
done
