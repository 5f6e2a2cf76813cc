#!/bin/bash
# Tiled path with the speculative launch after a check: convergence tests, then the small-grid
# kernel trace and the convergence table.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== tests $(date +%T)"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py \
  -k "tiled or fused or convergence" > gpurun_out/tiled_tests.log 2>&1 || { tail -30 gpurun_out/tiled_tests.log; exit 1; }
tail -2 gpurun_out/tiled_tests.log
echo "== profconv $(date +%T)"
timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/profconv2 -o run -- python -u tools/prof_conv.py 80 64 > gpurun_out/profconv2.log 2>&1 || { tail -5 gpurun_out/profconv2.log; exit 1; }
grep check= gpurun_out/profconv2.log
db=$(ls /tmp/profconv2/*/*.db /tmp/profconv2/*.db 2>/dev/null | head -1)
python tools/seq_trace.py "$db" tile_lds > gpurun_out/profconv2_seq.txt; head -8 gpurun_out/profconv2_seq.txt
echo "== conv table $(date +%T)"
timeout -k 10 300 python -u tools/conv_table.py > gpurun_out/conv_table_r5.md 2>&1 || { tail -5 gpurun_out/conv_table_r5.md; exit 1; }
cat gpurun_out/conv_table_r5.md
