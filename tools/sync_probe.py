"""Fixed cost of a short timed run (the driver's --steps 20): end-of-run sync modes x K.

For each (sync_mode, tblock): an untimed pre-warm, then `reps` repetitions of the bench's timed
region (torch sync; t0; engine.run(steps); torch sync; t1).  Prints min / median µs.
"""
import statistics
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
side = 4096
for tb in (8, 10):
    for mode in (0, 1, 2, 3):
        e = n.Engine(side, side, tblock=tb, device=0, small_grid_lds=False, sync_mode=mode)
        t_end = time.perf_counter() + 0.3
        while time.perf_counter() < t_end:
            e.run(64)
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e.run(steps)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e6)
        print(f"K={tb} sync_mode={mode} steps={steps}: min {min(ts):7.1f} us  median {statistics.median(ts):7.1f} us"
              f"  -> {side*side*steps/min(ts)*1e6:.3e} cups (best)", flush=True)
        del e
