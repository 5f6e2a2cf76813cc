set -o pipefail
export HEAT2D_NO_BUILD=1
for cfg in "mode=2" "mode=2 comm_cus=8" "mode=2 comm_cus=8 comm_cu_layout=1" "mode=2 comm_cus=8 comm_cu_layout=2" "mode=2 comm_cus=32 comm_cu_layout=1" "mode=2 comm_cus=64 comm_cu_layout=1" "mode=2 comm_cus=1 comm_cu_layout=1" "concurrent=1 contiguous_halo=1 comm_cus=8 comm_cu_layout=1" "concurrent=1 contiguous_halo=1 comm_cus=32 comm_cu_layout=1"; do
  timeout -k 10 120 python tools/overlap_trace.py one $cfg 2>&1 | grep us/step || exit $?
done
