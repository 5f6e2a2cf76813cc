# Does another engine's (idle) streams slow the multi-rank proxy?  (hardware-queue mapping)
mkdir -p gpurun_out; export HEAT2D_NO_BUILD=1 HEAT2D_KEEP_HW_QUEUES=1
for q in 4 8 16; do
echo "--- GPU_MAX_HW_QUEUES=$q: none first"; GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python tools/engine_ab.py none "signal_exchange=2" "signal_exchange=2" 2>&1 | grep "^\[" || exit 1
done
echo "--- GPU_MAX_HW_QUEUES=4, rccl, none, rccl"; timeout -k 10 120 python tools/engine_ab.py "signal_exchange=2" none "signal_exchange=2" 2>&1 | grep "^\[" || exit 1
