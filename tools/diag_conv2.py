"""Diagnostic: long single runs of local multi-tile engines (serial pipeline) — does the grid
drift from the oracle without host syncs between chunks, and does convergence get detected?"""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
nx, ny = 257, 509
kw = dict(convergence=True, interval=9, sensitivity=1.93e13)


def gather(e):
    out = np.zeros((nx, ny), np.float32)
    for t in range(e.num_tiles()):
        g = e.geom(t)
        out[g["gx0"]:g["gx0"] + g["xcell"], g["gy0"]:g["gy0"] + g["ycell"]] = e.download(t)
    return out


for gx, gy, opts in ((2, 1, dict(overlap=False)), (1, 2, dict(overlap=False)), (1, 2, dict(signal_exchange=2))):
    for steps in (45, 99, 200, 600):
        e = n.Engine(nx, ny, gridx=gx, gridy=gy, boundary=1, tblock=8, device=0, small_grid_lds=False, tiled=0,
                     **opts)
        e.run(steps)
        d = gather(e) != n.oracle_run(nx, ny, steps, boundary=1)["grid"]
        r, c = np.nonzero(d)
        print(f"{gx}x{gy} {opts} plain {steps}: wrong {int(d.sum())}"
              + (f" rows {r.min()}-{r.max()} cols {c.min()}-{c.max()}" if d.any() else ""), flush=True)
        for fused in (0, -1):
            e = n.Engine(nx, ny, gridx=gx, gridy=gy, boundary=1, tblock=8, device=0, small_grid_lds=False, tiled=0,
                         fused_check=fused, **opts, **{**kw, "sensitivity": 0.0})
            e.run(steps)
            d = gather(e) != n.oracle_run(nx, ny, steps, boundary=1)["grid"]
            r, c = np.nonzero(d)
            print(f"   conv(never) fused={fused} {steps}: wrong {int(d.sum())}"
                  + (f" rows {r.min()}-{r.max()} cols {c.min()}-{c.max()}" if d.any() else ""), flush=True)
    for fused in (0, -1):
        e = n.Engine(nx, ny, gridx=gx, gridy=gy, boundary=1, tblock=8, device=0, small_grid_lds=False, tiled=0,
                     fused_check=fused, **opts, **kw)
        st = e.run(3000)
        print(f"   conv fused={fused} run(3000): converged {st['converged']} steps {st['steps_done']} "
              f"resid {st['residual']:.6g} chunks {st['chunks']}", flush=True)
