"""Diagnostic: convergence checks on local multi-tile engines, segment by segment against the
oracle — which step first differs, and the residual of every check."""
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


cases = [(2, 1, dict(overlap=False), 0), (1, 2, dict(overlap=False), -1), (1, 2, dict(overlap=False), 0),
         (1, 1, {}, 0), (1, 2, dict(signal_exchange=2), -1)]
for gx, gy, opts, fused in cases:
    for seg in (9, 27):
        e = n.Engine(nx, ny, gridx=gx, gridy=gy, boundary=1, tblock=8, device=0, fused_check=fused,
                     small_grid_lds=False, tiled=0, **opts, **kw)
        print(f"== {gx}x{gy} {opts} fused={fused} seg={seg} pipeline={e.pipeline()}", flush=True)
        done = 0
        while done < 120:
            st = e.run(seg)
            done = st["steps_done"]
            ref = n.oracle_run(nx, ny, done, boundary=1)["grid"]
            refc = n.oracle_run(nx, ny, done, boundary=1, **kw)
            got = gather(e)
            d = got != ref
            r = np.nonzero(d)[0]
            c = np.nonzero(d)[1]
            print(f"  done {done}: resid {st['residual']:.6g} conv {st['converged']} chunks {st['chunks']} "
                  f"oracle-conv {refc['converged']} {refc['steps_done']} resid {refc['residual']:.6g} | wrong "
                  f"{int(d.sum())} rows {r.min() if len(r) else '-'}-{r.max() if len(r) else '-'} cols "
                  f"{c.min() if len(c) else '-'}-{c.max() if len(c) else '-'}", flush=True)
            if d.any() or st["converged"]:
                break
        del e
