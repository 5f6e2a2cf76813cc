#!/bin/bash
# Round-2 evidence run: full GPU test suite, smoke(), the driver-style bench (3 samples) and a
# 1000-step bench, then a rocprofv3 kernel-stats profile of the bench.
set -o pipefail
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for args in "--steps 20 --warmup 5" "--steps 20 --warmup 5" "--steps 20 --warmup 5" "--steps 1000 --warmup 200"; do
  timeout -k 10 120 python bench.py $args > gpurun_out/bench.json 2>gpurun_out/bench.err || { echo "bench failed: $args"; tail -5 gpurun_out/bench.err; exit 1; }
  cp gpurun_out/bench.json "gpurun_out/bench_$(echo $args | tr ' ' '_').json"
  python -c "import json,sys; d=json.load(open('gpurun_out/bench.json')); print('$args', '%.4e' % d['value'], '%.3f us/step' % (d['ms_per_step']*1e3))"
done
rm -rf gpurun_out/prof_r2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2 -o bench --output-format csv -- python3 bench.py --steps 1000 --warmup 200 > gpurun_out/prof_r2.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/prof_r2.log; exit 1; }
find gpurun_out/prof_r2 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/prof_r2_kernel_stats.csv
head -5 gpurun_out/prof_r2_kernel_stats.csv
