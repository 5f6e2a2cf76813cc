#!/bin/bash
# VALU instruction count, waves and clock of the 4096^2 streaming launches (K=8 and K=7), one
# counter pass each, compared with profiles/pmc_r2_4096.md.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for K in 8 7; do
  echo "== pmc K=$K $(date +%T)"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT \
    --kernel-trace -d /tmp/pmc$K -o run -- python bench.py --steps $((K * 5)) --warmup 0 --prewarm-s 0 --repeat 1 --no-verify --tblock $K \
    > gpurun_out/pmc$K.log 2>&1 || { tail -5 gpurun_out/pmc$K.log; exit 1; }
  db=$(ls /tmp/pmc$K/*/*.db /tmp/pmc$K/*.db 2>/dev/null | head -1)
  python tools/rocpd_summary.py "$db" stream_kernel > gpurun_out/pmc_k${K}_summary.txt 2>&1
  head -30 gpurun_out/pmc_k${K}_summary.txt
done
