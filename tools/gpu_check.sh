#!/bin/bash
# One GPU session: kernel/engine tests, smoke, headline bench (ref + fp32).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_ref.json 2> gpurun_out/bench_ref.err || exit $?
cat gpurun_out/bench_ref.json
timeout -k 10 300 python bench.py --precision fp32 > gpurun_out/bench_fp32.json 2> gpurun_out/bench_fp32.err || exit $?
cat gpurun_out/bench_fp32.json
