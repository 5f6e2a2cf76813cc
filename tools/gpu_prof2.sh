#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/sweep.py --n 4096 --steps 200 --rounds 2 --K 4,6,8 --H 0,16 --occ 1 > gpurun_out/sweep_fixed.txt 2>&1 || exit $?
timeout -k 10 300 python tools/sweep.py --n 4096 --steps 200 --rounds 2 --K 4,6,8 --H 0,16 --occ 1 --periodic > gpurun_out/sweep_periodic.txt 2>&1 || exit $?
grep -v amdgpu gpurun_out/sweep_fixed.txt; grep -v amdgpu gpurun_out/sweep_periodic.txt
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc_k4 -o run --output-format csv -- python tools/prof_one.py --K 4 --steps 64 > gpurun_out/pmc_k4.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc_k4p -o run --output-format csv -- python tools/prof_one.py --K 4 --steps 64 --periodic > gpurun_out/pmc_k4p.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_k4 -o run --output-format csv -- python tools/prof_one.py --K 4 --steps 64 > gpurun_out/kt_k4.log 2>&1 || exit $?
echo done
