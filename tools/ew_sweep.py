"""Edge weights of the planner at 4096^2 ref, K=7 (the bench default): us/step, median of 5."""
import os
import statistics
import sys
import time

import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()


def t(**kw):
    e = n.Engine(4096, 4096, device=0, small_grid_lds=False, tiled=0, tblock=7, **kw)
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        e.run(70)
        e.synchronize()
    xs = []
    for _ in range(5):
        e.synchronize()
        t0 = time.perf_counter()
        e.run(420)
        e.synchronize()
        xs.append((time.perf_counter() - t0) / 420 * 1e6)
    return statistics.median(xs), e.num_units(7)


for ew, rw in ((1.2, -1.0), (1.1, -1.0), (1.15, -1.0), (1.25, -1.0), (1.3, -1.0), (1.2, 1.1), (1.2, 1.3), (1.2, -1.0)):
    us, u = t(edge_weight=ew, row_edge_weight=rw)
    print(f"K=7 col_w={ew:4.2f} row_w={rw:5.2f}: {us:6.3f} us/step units={u}", flush=True)
