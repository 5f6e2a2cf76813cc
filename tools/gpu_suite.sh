#!/bin/bash
# One GPU session: the GPU test-suite, smoke(), the headline bench, the multi-rank proxy
# (row-periodic RCCL self-exchange on one GPU: the per-rank shape of the N>1 bench) and,
# with TABLE=1, the reference-size tables.
set -o pipefail
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_ref.json 2> gpurun_out/bench_ref.err || exit $?
cat gpurun_out/bench_ref.json
timeout -k 10 120 python tools/overlap_trace.py one 2>&1 | grep us/step | tee gpurun_out/proxy.txt || exit $?
if [ "${TABLE:-0}" = "1" ]; then
  timeout -k 10 600 python tools/bench_table.py --json gpurun_out/table_ref.json > gpurun_out/table_ref.md 2>&1 || exit $?
  timeout -k 10 600 python tools/bench_table.py --precision fp32 --json gpurun_out/table_fp32.json > gpurun_out/table_fp32.md 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/table_ref.md
fi
