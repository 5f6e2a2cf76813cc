#!/bin/bash
# Round-2 GPU check: full GPU test suite, then the driver-style bench (3 samples each).
set -o pipefail
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" ; tail -3 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit 1
fi
for args in "--steps 20 --warmup 5" "--steps 20 --warmup 5" "--steps 20 --warmup 5" "--steps 1000 --warmup 200" ${EXTRA_ARGS}; do
  timeout -k 10 120 python bench.py $args > gpurun_out/bench.json 2>gpurun_out/bench.err || { echo "bench failed: $args"; tail -5 gpurun_out/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench.json')); print('$args', '%.4e' % d['value'], '%.3f us/step' % (d['ms_per_step']*1e3), d['config']['tblock'])"
done
