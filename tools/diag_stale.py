"""Diagnostic: does a local multi-tile engine read memory it never wrote?  Fill the device
allocator's free memory with a large finite junk value first (torch allocates and releases it),
then run the serial / signalled pipelines and compare with the oracle step count by step count."""
import sys

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
nx, ny = 257, 509


def junk(v):
    free, _ = torch.cuda.mem_get_info()
    x = torch.full((int(free * 0.5) // 4,), v, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    del x
    torch.cuda.empty_cache()


def gather(e):
    out = np.zeros((nx, ny), np.float32)
    for t in range(e.num_tiles()):
        g = e.geom(t)
        out[g["gx0"]:g["gx0"] + g["xcell"], g["gy0"]:g["gy0"] + g["ycell"]] = e.download(t)
    return out


for gx, gy, opts in ((2, 1, dict(overlap=False)), (1, 2, dict(overlap=False)), (2, 1, dict(signal_exchange=2)),
                     (1, 1, dict())):
    for conv in (False, True):
        for steps in (1, 8, 9, 17, 45):
            junk(3.0e30)
            kw = dict(convergence=True, interval=9, sensitivity=0.0, fused_check=0) if conv else {}
            e = n.Engine(nx, ny, gridx=gx, gridy=gy, boundary=1, tblock=8, device=0, small_grid_lds=False, tiled=0,
                         **opts, **kw)
            e.run(steps)
            got = gather(e)
            d = got != n.oracle_run(nx, ny, steps, boundary=1)["grid"]
            r, c = np.nonzero(d)
            print(f"{gx}x{gy} {opts} conv={conv} {steps}: wrong {int(d.sum())}"
                  + (f" rows {r.min()}-{r.max()} cols {c.min()}-{c.max()} max|v| {np.abs(got).max():.3g}"
                     if d.any() else ""), flush=True)
            del e
