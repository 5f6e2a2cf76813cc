#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1
timeout -k 10 600 python tools/sweep.py --n 4096 --steps 400 --rounds 2 > gpurun_out/sweep.txt 2>&1 || exit $?
cat gpurun_out/sweep.txt | tail -45
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ref -o run --output-format csv -- python bench.py --steps 200 --warmup 16 > gpurun_out/prof_ref.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_ref -o run --output-format csv -- python bench.py --steps 200 --warmup 16 > gpurun_out/pmc_ref.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d gpurun_out/pmc_mem -o run --output-format csv -- python bench.py --steps 200 --warmup 16 --precision fp32 > gpurun_out/pmc_mem.log 2>&1 || exit $?
find gpurun_out/prof_ref gpurun_out/pmc_ref gpurun_out/pmc_mem -name "*.csv" | head
