#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1
timeout -k 10 600 python -m pytest tests/test_gpu_engine.py -x -q  > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python tools/sweep.py --n 4096 --steps 200 --rounds 2 ${SWEEP_ARGS} > gpurun_out/sweep3.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/sweep3.txt
