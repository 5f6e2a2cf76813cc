set -o pipefail
timeout -k 10 200 python -u tools/clock_probe.py 80 64 tiled=1 tile_width=32 tile_k=12 tile_rows=4 tile_threads=1024 tile_cpl=1 small_grid_lds=0 &&
timeout -k 10 200 python -u tools/clock_probe.py 4096 4096 && (rocm-smi --showclocks 2>&1 | tail -15 || true)
