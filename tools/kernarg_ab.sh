#!/bin/bash
# GPU-box A/B of the kernel-argument settings (round 5, docs/ARCHITECTURE.md "Kernel arguments"):
# tests/test_gpu_engine.py under each environment given as NAME=ENV... arguments, e.g.
#   bash tools/kernarg_ab.sh pool= nopool=HEAT2D_STREAM_POOL=0 host=HIP_FORCE_DEV_KERNARG=0
# TESTK selects tests (-k).  Stops at the first run whose log shows a GPU fault.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1 TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%=*}
  envs=${spec#*=}
  log=gpurun_out/ab_$name.log
  echo "== $name ($envs) $(date +%T)"
  # shellcheck disable=SC2086
  env $envs timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -q --timeout 300 \
    --timeout-method thread -rf ${TESTK:+-k "$TESTK"} > "$log" 2>&1
  rc=$?
  tail -n 2 "$log"
  grep -c "integrity check failed" "$log" | sed 's/^/integrity failures: /'
  if grep -q "illegal memory access\|Memory access fault\|HSA_STATUS_ERROR" "$log" || [ $rc -gt 1 ]; then
    echo "== $name: GPU fault or abort (rc=$rc): stopping"
    exit 3
  fi
done
echo "== done"
