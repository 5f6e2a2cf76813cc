cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1
i=0
for k in "fused_convergence_matches_oracle or ipc_direct" "fused_convergence_matches_oracle or rccl" "fused_convergence_matches_oracle or tiled" "fused_convergence_matches_oracle or timeline or strong_scaling or bench_shape" "fused_convergence_matches_oracle or multitile or periodic or overlap or pipeline_auto" "fused_convergence_matches_oracle or stream or every or rows_per or int32 or fp32 or lds or naive or convergence_matches"; do
  i=$((i+1))
  timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -q --timeout 120 --timeout-method thread -rf -k "$k" > gpurun_out/bis_$i.log 2>&1; rc=$?
  echo "$i [$k] rc=$rc: $(tail -1 gpurun_out/bis_$i.log)"
  if [ $rc -gt 1 ]; then exit $rc; fi
done
timeout -k 10 300 python -u tools/pstream_check.py check > gpurun_out/pcheck.log 2>&1; rc=$?; echo "pcheck rc=$rc"; tail -30 gpurun_out/pcheck.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/pstream_check.py time > gpurun_out/ptime.log 2>&1; rc=$?; echo "ptime rc=$rc"; tail -20 gpurun_out/ptime.log
