#!/bin/bash
# Pipeline-option matrix and a kernel-trace timeline of the multi-rank pipeline on one GPU.
set -o pipefail
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_engine.py -q -x -k "rccl" > gpurun_out/ot_tests.log 2>&1; rc=$?; tail -2 gpurun_out/ot_tests.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/ot_matrix.txt
for cfg in "mode=2" "concurrent=1 contiguous_halo=0 comm_cus=0" "concurrent=1 contiguous_halo=1 comm_cus=0" \
           "concurrent=1 contiguous_halo=1 comm_cus=0 boundary_rows=8" "concurrent=1 contiguous_halo=1 comm_cus=4" \
           "concurrent=1 contiguous_halo=1 comm_cus=8" "concurrent=1 contiguous_halo=1 comm_cus=8 boundary_rows=8" \
           "concurrent=1 contiguous_halo=1 comm_cus=16" "concurrent=1 contiguous_halo=0 comm_cus=8" \
           "concurrent=0 contiguous_halo=1 comm_cus=0" "concurrent=0 contiguous_halo=1 comm_cus=8" \
           "concurrent=1 contiguous_halo=1 comm_cus=0" "mode=2"; do
  timeout -k 10 120 python tools/overlap_trace.py one $cfg 2>&1 | grep us/step | tee -a gpurun_out/ot_matrix.txt || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ot -o ot --output-format csv -- python3 tools/overlap_trace.py one ${OT_ARGS:-comm_cus=8 contiguous_halo=1} > gpurun_out/ot.log 2>&1 || exit $?
f=$(find gpurun_out/ot -name "*kernel_trace.csv" | head -1)
python tools/trace_timeline.py "$f" 30
