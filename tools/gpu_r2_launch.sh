#!/bin/bash
# Per-launch cost: kernel durations and dispatch gaps of the streaming kernel at 4096^2 (K=8)
# and at the 8-GPU strong-scaling tile 512x4096 (K=4, 6, 8), from rocprofv3 kernel traces.
set -o pipefail
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1 TMPDIR=/tmp
for cfg in "4096 0 8" "4096 512 6" "4096 512 4" "4096 512 8"; do
  set -- $cfg
  d=gpurun_out/lt_$1_$2_$3
  rm -rf $d
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format rocpd -d $d -o lt -- python3 tools/prof_one.py --n $1 --rows $2 --K $3 --steps 480 > $d.log 2>&1 || { echo "trace failed $cfg"; tail -5 $d.log; exit 1; }
  db=$(find $d -name "*.db" | head -1)
  echo "== n=$1 rows=$2 K=$3"; python3 tools/rocpd_summary.py "$db" stream
done
