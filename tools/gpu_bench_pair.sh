#!/bin/bash
# bench.py as the driver runs it (defaults) and a short driver-style run
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && tail -1 gpurun_out/bench_default.json &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_20.json 2> gpurun_out/bench_20.err && tail -1 gpurun_out/bench_20.json &&
timeout -k 10 300 python -u bench.py --steps 1000 --warmup 5 > gpurun_out/bench_1000.json 2> gpurun_out/bench_1000.err && tail -1 gpurun_out/bench_1000.json
