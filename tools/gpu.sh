#!/bin/bash
# One parameterised driver for GPU-box work (run under gpurun from the repo root):
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/gpu.sh tests smoke bench20 timeline'
# Every step runs under its own time limit and writes under gpurun_out/; the first failing step
# ends the script (no GPU step runs after a fault, abort or time-out).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1 TMPDIR=/tmp

step() {  # step NAME SECONDS CMD...: run, log, stop the script on failure
  local name=$1 secs=$2
  shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then
    echo "== $name FAILED rc=$rc"
    exit $rc
  fi
}

for s in "$@"; do
  case "$s" in
    tests) step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    tests-nox) step tests-nox 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf ;;
    engine-file) step engine-file 600 python -u -m pytest tests/test_gpu_engine.py -q --timeout 300 --timeout-method thread -rf ;;
    serial) step serial 600 python -u -m pytest tests/test_gpu_engine.py -v --timeout 300 --timeout-method thread -rf -k serial_tiles_long ;;
    tests-k) step tests-k 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf -k "$TESTK" ;;
    mp) step mp 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multiprocess_gpu.py ;;
    pcheck) step pcheck 300 python -u tools/pstream_check.py check ;;
    ptime) step ptime 300 python -u tools/pstream_check.py time ;;
    convtable) step convtable 600 python -u tools/conv_table.py ;;
    pmcpst) step pmcpst 120 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU --kernel-trace --stats -d gpurun_out/pmcpst -o run -- python tools/prof_pstream.py 512 128 ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench20) step bench20 300 python bench.py --steps 20 --warmup 5 ;;
    bench1000) step bench1000 300 python bench.py --steps 1000 --warmup 200 ;;
    timeline) step timeline 300 python -u tools/timeline.py 4096x4096:7:20 4096x4096:7:70 2048x4096:7:70 \
                1024x4096:7:70 512x4096:6:60 512x4096:6:60:direct 1024x4096:7:70:direct \
                --json gpurun_out/timeline.json ;;
    timeline2) step timeline2 300 python -u tools/timeline.py 512x4096:6:60 512x4096:6:60:direct 1024x4096:7:70 \
                 8192x4096:7:70 8192x4096:7:70:direct2d 4096x4096:7:70 --json gpurun_out/timeline2.json ;;
    rehearse4) step rehearse4 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
                 --master-port 29611 bench.py --gpus 4 --steps 42 --warmup 14 --persistent on ;;
    rehearse8) step rehearse8 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
                 --master-port 29612 bench.py --gpus 8 --steps 42 --warmup 14 --persistent on ;;
    profconv) step profconv 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profconv -o run -- python tools/prof_conv.py 80 64 ;;
    proxy) step proxy 600 python -u tools/strong_proxy.py 4096 840 6,7,8 0 '' 1,2,4,8 ;;
    prof) step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- \
            python bench.py --steps 20 --warmup 5 --repeat 3 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== all done ($(date +%T))"
