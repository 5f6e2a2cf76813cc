#!/bin/bash
# the whole GPU test suite, one process, bounded
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_suite.log
exit $rc
