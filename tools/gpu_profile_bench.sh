#!/bin/bash
# rocprofv3 evidence for the headline bench (kernel trace + stats, and PMC counter passes).
set -o pipefail
mkdir -p gpurun_out/prof
export HEAT2D_NO_BUILD=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o bench --output-format csv -- python bench.py --steps 1000 --warmup 200 > gpurun_out/prof/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE -d gpurun_out/prof/pmc_sq -o bench --output-format csv -- python tools/prof_one.py --K 8 --steps 64 > gpurun_out/prof/pmc_sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc_fetch -o bench --output-format csv -- python tools/prof_one.py --K 8 --steps 64 > gpurun_out/prof/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmc_write -o bench --output-format csv -- python tools/prof_one.py --K 8 --steps 64 > gpurun_out/prof/pmc_write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/prof/pmc_mix -o bench --output-format csv -- python tools/prof_one.py --K 8 --steps 64 > gpurun_out/prof/pmc_mix.log 2>&1 || exit $?
echo profiled
