#!/bin/bash
# Host-side cost of the bench's 20-step region: submit/total medians, then one HIP-API + kernel
# timeline of the last timed run (rocprofv3 --hip-trace --kernel-trace, no counters).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== plain $(date +%T)"
timeout -k 10 200 python -u tools/host_trace.py 4096 20 100 > gpurun_out/host_plain.log 2>&1 || { tail -5 gpurun_out/host_plain.log; exit 1; }
cat gpurun_out/host_plain.log
echo "== traced $(date +%T)"
timeout -k 10 180 rocprofv3 --hip-trace --kernel-trace -d /tmp/hosttr -o run -- python -u tools/host_trace.py 4096 20 20 > gpurun_out/host_tr.log 2>&1 || { tail -5 gpurun_out/host_tr.log; exit 1; }
db=$(ls /tmp/hosttr/*/*.db /tmp/hosttr/*.db 2>/dev/null | head -1)
python tools/host_trace.py --db "$db" > gpurun_out/host_timeline.txt
cat gpurun_out/host_timeline.txt | tail -60
