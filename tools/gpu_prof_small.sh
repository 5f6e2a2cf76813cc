#!/bin/bash
# kernel trace of the LDS-tiled kernel on the reference's small grids (dispatch duration vs gap)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_small
for shape in "80 64 16 tiled:8:1024:64" "80 64 8 tiled:8:1024:64" "80 64 16 tiled:8:256:64" "640 512 16 tiled:16:1024:128"; do
  set -- $shape
  tag="r$1_c$2_k$3_$(echo $4 | tr : _)"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_small/$tag -o run -- python3 $R/tools/prof_tile.py $1 $2 $3 1600 $4 > $R/gpurun_out/prof_small/$tag.log 2>&1 || { echo "fail $tag"; tail -5 $R/gpurun_out/prof_small/$tag.log; exit 1; }
  db=$(ls $R/gpurun_out/prof_small/$tag/*/*.db 2>/dev/null | head -1 || true)
  [ -z "$db" ] && db=$(find $R/gpurun_out/prof_small/$tag -name '*.db' | head -1)
  echo "== $tag"; python3 $R/tools/rocpd_summary.py $db tile
done
