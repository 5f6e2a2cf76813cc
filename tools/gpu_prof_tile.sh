#!/bin/bash
# kernel trace of short tiles (strong-scaling per-rank shapes) vs the full 4096^2 tile
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_tile
for shape in "512 4096 8" "512 4096 4" "4096 4096 8" "1024 4096 8"; do
  set -- $shape
  tag="r$1_c$2_k$3"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_tile/$tag -o run -- python3 $R/tools/prof_tile.py $1 $2 $3 400 > $R/gpurun_out/prof_tile/$tag.log 2>&1 || { echo "fail $tag"; tail -5 $R/gpurun_out/prof_tile/$tag.log; exit 1; }
  cat $R/gpurun_out/prof_tile/$tag.log | grep units
done
for pmcset in "SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU"; do
  for shape in "512 4096 8" "4096 4096 8"; do
    set -- $shape
    tag="pmc_r$1_k$3_$(echo $pmcset | cut -c1-12 | tr ' ' _)"
    timeout -s KILL 90 rocprofv3 --pmc $pmcset -d $R/gpurun_out/prof_tile/$tag -o run -- python3 $R/tools/prof_tile.py $1 $2 $3 80 > $R/gpurun_out/prof_tile/$tag.log 2>&1 || { echo "pmc fail $tag"; tail -5 $R/gpurun_out/prof_tile/$tag.log; exit 1; }
  done
done
echo done
