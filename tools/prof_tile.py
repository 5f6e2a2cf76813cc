"""One engine, one tile shape, N steps (for rocprofv3 kernel traces / counters).
usage: prof_tile.py ROWS COLS K STEPS [direct | tiled:TX:NT:RY]"""
import sys

import torch  # noqa: F401

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
rows, cols, K, steps = (int(x) for x in sys.argv[1:5])
mode = sys.argv[5] if len(sys.argv) > 5 else ""
direct = mode == "direct"
if mode.startswith("tiled"):
    tx, nt, ry = (int(v) for v in mode.split(":")[1:])
    e = n.Engine(rows, cols, device=0, small_grid_lds=False, tiled=1, tile_k=K, tile_rows=tx, tile_threads=nt,
                 tile_width=ry)
elif direct:
    e = n.Engine(rows, cols, periodic_x=True, tblock=K, device=0, ranks=[0], transport=n.TRANSPORT_IPC)
    e.ipc_open([e.ipc_handle()])
    e.ipc_prime()
else:
    e = n.Engine(rows, cols, tblock=K, device=0, small_grid_lds=False, tiled=0)
e.run(steps)
e.synchronize()
if not mode.startswith("tiled"):
    print("units", e.num_units(K), "H", e.rows_per_wave(K))
