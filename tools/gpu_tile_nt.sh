set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_engine.py -k "tiled or conv or fused" > gpurun_out/tiled_tests.log 2>&1 && tail -2 gpurun_out/tiled_tests.log &&
bash tools/gpu_tile_fit.sh &&
timeout -k 10 500 python -u tools/tile_sweep.py --sizes 80x64,160x128,320x256,640x512,1280x1024 --quick > gpurun_out/tile_sweep_nt.txt 2>&1; grep -A4 "==" gpurun_out/tile_sweep_nt.txt
