#!/bin/bash
# Sweep + counters of the streaming kernel after the packed-sum / edge-aligned-strip changes.
set -o pipefail
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1
timeout -k 10 300 python tools/sweep.py --n 4096 --steps 400 --rounds 2 --K 6,8,10,12 --H 0,48,96 --prec 0,1 --ew 1.0,1.15,1.3 > gpurun_out/sweep3.txt 2>&1 || exit $?
grep -v amdgpu gpurun_out/sweep3.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/kt3 -o run --output-format csv -- python bench.py --steps 200 --warmup 16 > gpurun_out/kt3.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc3 -o run --output-format csv -- python tools/prof_one.py --K 8 --steps 64 > gpurun_out/pmc3.log 2>&1 || exit $?
find gpurun_out/kt3 gpurun_out/pmc3 -name "*.csv"
echo done
