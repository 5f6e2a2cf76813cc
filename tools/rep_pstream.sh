# diagnostics: the two-process persistent worker, repeated (fresh processes each time)
cd $GRAFT_REPO_ROOT
export HEAT2D_NO_BUILD=1
for dbg in ${DBGS:-0}; do
for i in $(seq 1 ${REPS:-6}); do
  H2D_DEBUG_KERNEL=$dbg timeout -k 5 60 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port $((29500+i)) tests/_pstream_ranks_worker.py > gpurun_out/rep_${dbg}_${i}.txt 2>&1
  echo "dbg=$dbg run $i: $(grep -o '"ok[2]*": [a-z]*' gpurun_out/rep_${dbg}_${i}.txt | tr '\n' ' ') $(grep 'wrong' gpurun_out/rep_${dbg}_${i}.txt | tr '\n' ' ')"
done
done
