#!/bin/bash
# Pipeline-option matrix and a kernel-trace timeline of the multi-rank pipeline on one GPU.
#   OT_CFGS: configs for the matrix (';'-separated), OT_ARGS: the traced config.
set -o pipefail
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_engine.py -q -x -k "rccl or overlap or convergence" > gpurun_out/ot_tests.log 2>&1; rc=$?; tail -2 gpurun_out/ot_tests.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/ot_matrix.txt
IFS=';' read -ra CFGS <<< "${OT_CFGS:-mode=2;concurrent=1 comm_boundary=0;concurrent=1;concurrent=0}"
for cfg in "${CFGS[@]}"; do
  timeout -k 10 120 python tools/overlap_trace.py one $cfg 2>&1 | grep us/step | tee -a gpurun_out/ot_matrix.txt || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ot -o ot --output-format csv -- python3 tools/overlap_trace.py one ${OT_ARGS:-concurrent=1} > gpurun_out/ot.log 2>&1 || exit $?
f=$(find gpurun_out/ot -name "*kernel_trace.csv" | head -1)
python tools/trace_timeline.py "$f" 30
