#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/bench_table.py --tune --json gpurun_out/table_ref.json > gpurun_out/table_ref.md 2>&1 || exit $?
grep -v amdgpu gpurun_out/table_ref.md
timeout -k 10 600 python tools/bench_table.py --tune --precision fp32 --json gpurun_out/table_fp32.json > gpurun_out/table_fp32.md 2>&1 || exit $?
grep -v amdgpu gpurun_out/table_fp32.md
