#!/bin/bash
# A/B of the persistent plan's halo-band weight (EngineOptions::pstream_halo_weight) on the
# strong-scaling proxy's N=4 / N=8 rank tiles at the bench's depth 8, interleaved, two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for round in 1 2; do
  for w in 1.0 1.1 1.15 1.2; do
    timeout -k 10 200 python -u tools/strong_proxy.py 4096 840 8 0 pstream_halo_weight=$w 4,8 > gpurun_out/phw_${w}_$round.log 2>&1 || exit 1
    echo "w=$w round $round: $(grep direct gpurun_out/phw_${w}_$round.log | sed 's/ *us\/step alone,/ alone/;s/(units [0-9]*) -> speedup.*//' | tr '\n' ' ')"
  done
done
