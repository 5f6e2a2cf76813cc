"""Planner knobs at 4096^2 (ref, K=8): edge weight and unit height, us/step (best of 3 x 400 steps)."""
import os
import sys
import time

import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
side = int(sys.argv[1]) if len(sys.argv) > 1 else 4096


def t(**kw):
    e = n.Engine(side, side, device=0, small_grid_lds=False, tiled=0, **kw)
    e.run(200)
    best = 1e9
    for _ in range(3):
        e.synchronize()
        t0 = time.perf_counter()
        e.run(400)
        e.synchronize()
        best = min(best, (time.perf_counter() - t0) / 400 * 1e6)
    return best, e.num_units(kw.get("tblock", 8)), e.rows_per_wave(kw.get("tblock", 8))


for ew in (1.2, 1.3, 1.4, 1.5, 1.6, 1.8):
    for rw in (1.0, 1.1, 1.2, 1.3, 1.5):
        us, u, h = t(tblock=8, edge_weight=ew, row_edge_weight=rw)
        print(f"K=8 col_w={ew:4.2f} row_w={rw:4.2f}: {us:6.3f} us/step  units={u} H={h}", flush=True)
