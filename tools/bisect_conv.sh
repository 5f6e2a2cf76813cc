#!/bin/bash
# Which earlier tests make test_fused_convergence_matches_oracle[0-*] fail?  (GPU box, diagnostics)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1
i=0
for k in "ipc_direct or fused_convergence_matches_oracle" "not ipc_direct and not fused_convergence_intervals and not tiled_chunks and not fused_convergence_tiled and not fused_convergence_rccl" \
         "ipc_direct_self_exchange_row_periodic or fused_convergence_matches_oracle" "ipc_direct_2d or fused_convergence_matches_oracle" \
         "ipc_direct_convergence_and_reprime or ipc_direct_rejects or output_store or fused_convergence_matches_oracle"; do
  i=$((i+1))
  timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -q --timeout 120 --timeout-method thread -rf -k "$k" > gpurun_out/bisect_$i.log 2>&1
  rc=$?
  echo "$i [$k] rc=$rc: $(tail -1 gpurun_out/bisect_$i.log) :: $(grep -o 'FAILED [^ ]*' gpurun_out/bisect_$i.log | tr '\n' ' ')"
  if [ $rc -gt 1 ]; then exit $rc; fi
done
