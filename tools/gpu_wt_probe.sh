#!/bin/bash
# write-through (sc1) vs plain output stores of the streaming kernel: per-rank strong-scaling proxy
set -o pipefail
mkdir -p gpurun_out
for wt in 0 1; do
  echo "== wt_store=$wt"
  timeout -k 10 300 python -u tools/strong_proxy.py 4096 960 4,6,8 0 wt_store=$wt 1,2,4,8 || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/wt_probe.txt
