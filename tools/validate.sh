#!/bin/bash
# Validation on one GPU box: smoke, the whole GPU suite, the bench (20 / 1000 steps), its
# kernel trace, the small-grid check trace, and an A/B of the stencil's integrity checks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu.sh smoke tests-nox bench20 bench1000 prof profconv || exit $?
timeout -k 10 300 python -u tools/ab_kernel.py 4096 4096 1000 7 'checks:tblock=7,tiled=0' \
  'nochecks:tblock=7,tiled=0,debug_kernel=2' > gpurun_out/ab_checks.log 2>&1
cat gpurun_out/ab_checks.log
