#!/bin/bash
# PMC of the 4096^2 ref kernel (K=8, one wave per SIMD): VALU instructions per cell-update
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc4096
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc4096/a -o run -- python3 $R/tools/prof_tile.py 4096 4096 8 80 > $R/gpurun_out/pmc4096/a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $R/gpurun_out/pmc4096/b -o run -- python3 $R/tools/prof_tile.py 4096 4096 8 80 > $R/gpurun_out/pmc4096/b.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmc4096/t -o run -- python3 $R/tools/prof_tile.py 4096 4096 8 400 > $R/gpurun_out/pmc4096/t.log 2>&1 || exit 1
echo done
