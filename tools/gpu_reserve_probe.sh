#!/bin/bash
# Pipeline option matrix (one process per configuration), then a trace.
set -o pipefail
export HEAT2D_NO_BUILD=1
B="concurrent=1 contiguous_halo=1 boundary_rows=8"
for rep in 1 2; do
for cfg in "mode=2" "$B reserve_waves=16" "$B reserve_waves=16 device_fence_events=1" "$B reserve_waves=32 device_fence_events=1" \
  "concurrent=0 contiguous_halo=1 boundary_rows=8 reserve_waves=32 device_fence_events=1" "mode=1 $B reserve_waves=16 device_fence_events=1" \
  "mode=1 $B reserve_waves=16"; do
  timeout -k 10 120 python tools/overlap_trace.py one $cfg 2>&1 | grep us/step || exit $?
done
done
OT_ARGS="$B reserve_waves=16 device_fence_events=1" bash tools/gpu_trace_one.sh
