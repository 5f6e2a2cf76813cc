#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1
timeout -k 10 600 python -m pytest tests/test_gpu_engine.py -x -q -k "lds or convergence" > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
for n in 320 640 1280; do
  timeout -k 10 300 python tools/sweep.py --n $n --steps 1000 --rounds 2 --K 1,2,4,8 --H 4,8,16,0 --prec 0 --boundary 1 > gpurun_out/small_$n.txt 2>&1 || exit $?
  grep -E "BEST|grid" gpurun_out/small_$n.txt; sort -k6 -n gpurun_out/small_$n.txt | grep prec | head -4
done
timeout -k 10 600 python tools/bench_table.py > gpurun_out/table_ref2.md 2>&1 || exit $?
grep -v amdgpu gpurun_out/table_ref2.md | head -5
