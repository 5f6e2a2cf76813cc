#!/bin/bash
# Round-5 second validation: the whole GPU suite, the convergence table (with the multi-rank
# proxy rows), the bench (20 / 1000 steps) and the host-side trace of the 20-step region.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu.sh smoke tests-nox convtable bench20 bench1000 || exit $?
bash tools/r5_host.sh
