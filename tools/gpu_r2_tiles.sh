#!/bin/bash
# GPU suite + full small/medium-grid tile sweep (profiles/tile_sweep_r2.txt)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tile_sweep.py > gpurun_out/tile_sweep_r2.txt 2>&1 && grep -A3 "==" gpurun_out/tile_sweep_r2.txt
