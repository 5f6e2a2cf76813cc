"""Per-rank tiles of 4096^2 strong scaling (rows x 4096), alone: 20-step and 840-step runs per
halo depth, to pick the bench's depth by tile height.  Median of 50 (20 steps) / 5 (840)."""
import os
import statistics
import sys
import time

import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()


def med(e, st, reps):
    xs = []
    for _ in range(reps):
        e.synchronize()
        t0 = time.perf_counter()
        e.run(st)
        e.synchronize()
        xs.append((time.perf_counter() - t0) / st * 1e6)
    return statistics.median(xs)


for rows in (512, 1024, 2048):
    for tb in (5, 6, 7, 8):
        e = n.Engine(rows, 4096, tblock=tb, device=0, small_grid_lds=False, tiled=0)
        t_end = time.perf_counter() + 0.5
        while time.perf_counter() < t_end:
            e.run(20)
        print(f"{rows}x4096 tblock {tb}: 20 steps {med(e, 20, 50):6.3f} us/step, 840 steps {med(e, 840, 5):6.3f} us/step",
              flush=True)
        del e
