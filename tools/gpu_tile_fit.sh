#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/tile_fit.txt
for cfg in "80 64 32 4 1024 4" "80 64 32 4 1024 2" "80 64 32 4 1024 1" "160 128 64 4 1024 1" "160 128 64 4 1024 2" "4 4 32 4 256 1"; do
  timeout -k 10 300 python -u tools/tile_fit.py $cfg 2,4,6,8,12 >> gpurun_out/tile_fit.txt 2>&1 || exit 1
done
cat gpurun_out/tile_fit.txt
