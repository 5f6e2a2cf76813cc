#!/bin/bash
# GPU suite, bench, default-pipeline self-exchange timing and the ops-path probe.
set -o pipefail
bash tools/gpu_full.sh || exit $?
export HEAT2D_NO_BUILD=1
for cfg in "mode=2" "concurrent=1" "concurrent=0" "mode=1"; do
  timeout -k 10 120 python tools/overlap_trace.py one $cfg 2>&1 | grep us/step || exit $?
done
timeout -k 10 120 python tools/event_gap_probe.py 2>&1 | grep -v amdgpu.ids
