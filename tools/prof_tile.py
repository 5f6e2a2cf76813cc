"""One engine, one tile shape, N steps (for rocprofv3 kernel traces / counters).
usage: prof_tile.py ROWS COLS K STEPS [direct]"""
import sys

import torch  # noqa: F401

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
rows, cols, K, steps = (int(x) for x in sys.argv[1:5])
direct = len(sys.argv) > 5 and sys.argv[5] == "direct"
if direct:
    e = n.Engine(rows, cols, periodic_x=True, tblock=K, device=0, ranks=[0], transport=n.TRANSPORT_IPC)
    e.ipc_open([e.ipc_handle()])
    e.ipc_prime()
else:
    e = n.Engine(rows, cols, tblock=K, device=0, small_grid_lds=False, tiled=0)
e.run(steps)
e.synchronize()
print("units", e.num_units(K), "H", e.rows_per_wave(K))
