#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1
timeout -k 10 600 python -m pytest tests/test_gpu_engine.py -x -q  > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/multitile_bench.py > gpurun_out/mt.txt 2>&1 || exit $?
grep -v amdgpu gpurun_out/mt.txt
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2>gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
