"""Diagnostics: the sequence of test_fused_convergence_matches_oracle[0-2-1] — a converging
2-tile serial engine, then a second engine created while the first is alive, the first
released — repeated; does the second engine compute wrong tiles, and does the order of
creation / release matter?"""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
nx, ny = 257, 509
CONV = dict(convergence=True, interval=9, sensitivity=1.93e13)
ref9 = n.oracle_run(nx, ny, 9, boundary=1)["grid"]


def make(fused, **kw):
    return n.Engine(nx, ny, gridx=2, gridy=1, boundary=1, tblock=8, device=0, fused_check=fused, small_grid_lds=False,
                    tiled=0, overlap=False, **kw)


def gather(e):
    out = np.zeros((nx, ny), np.float32)
    for t in range(e.num_tiles()):
        g = e.geom(t)
        out[g["gx0"]:g["gx0"] + g["xcell"], g["gy0"]:g["gy0"] + g["ycell"]] = e.download(t)
    return out


reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
for order in ("create-then-release", "release-then-create"):
    bad = 0
    for i in range(reps):
        a = make(-1, **CONV)
        a.run(3000)
        if order == "create-then-release":
            b = make(0, **{**CONV, "sensitivity": 0.0})
            del a
        else:
            del a
            b = make(0, **{**CONV, "sensitivity": 0.0})
        b.run(9)
        d = gather(b) != ref9
        if d.any():
            bad += 1
            r, c = np.nonzero(d)
            print(f"  {order} rep {i}: wrong {int(d.sum())} rows {r.min()}-{r.max()}", flush=True)
        del b
    print(f"{order}: {bad}/{reps} wrong", flush=True)
