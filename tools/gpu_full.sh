#!/bin/bash
# GPU session: full GPU test-suite, optional sweep (SWEEP_ARGS), headline bench.
set -o pipefail
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
if [ -n "$SWEEP_ARGS" ]; then
  timeout -k 10 900 python tools/sweep.py ${SWEEP_ARGS} > gpurun_out/sweep.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/sweep.txt
fi
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2>gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
