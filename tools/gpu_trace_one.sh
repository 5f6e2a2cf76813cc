#!/bin/bash
# Kernel-trace timeline of one overlap_trace.py configuration (OT_ARGS).
set -o pipefail
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1
export TMPDIR=/tmp
rm -rf gpurun_out/ot
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ot -o ot --output-format csv -- python3 tools/overlap_trace.py one ${OT_ARGS} > gpurun_out/ot.log 2>&1 || exit $?
grep us/step gpurun_out/ot.log
f=$(find gpurun_out/ot -name "*kernel_trace.csv" | head -1)
python tools/trace_timeline.py "$f" ${OT_WIN:-30}
