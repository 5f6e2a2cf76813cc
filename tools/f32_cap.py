"""fp32 path at 4096^2: wave capacity (units per round) x depth, us/step (median of 5 x 400)."""
import os
import statistics
import sys
import time

import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
for K in (8, 6, 10):
    for cap in (0, 1024, 2048, 3072):
        e = n.Engine(4096, 4096, precision=1, tblock=K, device=0, small_grid_lds=False, tiled=0, wave_capacity=cap)
        t_end = time.perf_counter() + 0.4
        while time.perf_counter() < t_end:
            e.run(K * 10)
            e.synchronize()
        xs = []
        for _ in range(5):
            e.synchronize()
            t0 = time.perf_counter()
            e.run(400)
            e.synchronize()
            xs.append((time.perf_counter() - t0) / 400 * 1e6)
        print(f"fp32 K={K} cap={cap}: {statistics.median(xs):6.3f} us/step units={e.num_units(K)}", flush=True)
        del e
