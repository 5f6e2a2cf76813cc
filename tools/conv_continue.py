"""Diagnostic: a fused-convergence run that converges, then a re-prime and a continuation, on the
direct pipeline's row-periodic self-exchange (and a lone tile) — per variant, whether the converged
grid and the continued grid equal the oracle, and where they differ.
usage: python tools/conv_continue.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()


def where(got, ref):
    bad = got != ref
    if not bad.any():
        return "equal"
    r, c = np.nonzero(bad)
    return f"{int(bad.sum())} cells differ, rows {r.min()}-{r.max()}, cols {c.min()}-{c.max()}"


def sens_at_60(nx, ny, boundary, per):
    r = [n.oracle_run(nx, ny, s, boundary=boundary, periodic_x=per[0], convergence=True, interval=20,
                      sensitivity=0.0)["residual"] for s in (40, 60)]
    return 0.5 * (r[0] + r[1])


def case(name, nx, ny, K, direct, persistent, boundary=0, cont=16, cols=128):
    per = (True, False) if direct else (False, False)
    kw = dict(convergence=True, interval=20, sensitivity=sens_at_60(nx, ny, boundary, per))
    extra = dict(periodic_x=True, ranks=[0], transport=n.TRANSPORT_IPC) if direct else dict(small_grid_lds=False, tiled=0)
    e = n.Engine(nx, ny, tblock=K, device=0, boundary=boundary, halo_timeout_s=5.0, persistent=persistent,
                 pstream_cols=cols, **extra, **kw)
    if direct:
        e.ipc_open([e.ipc_handle()])
        e.ipc_prime()
    ref = n.oracle_run(nx, ny, 200, boundary=boundary, periodic_x=per[0], **kw)
    st = e.run(200)
    first = where(e.download(0), ref["grid"])
    if direct:
        e.ipc_prime()
    e.run(cont)
    ref2 = n.oracle_run(nx, ny, int(ref["steps_done"]) + cont, boundary=boundary, periodic_x=per[0])
    print(f"{name}: converged {st['converged']} at {st['steps_done']} (oracle {ref['steps_done']}), "
          f"persistent launches {e.pstream_launches()}; first {first}; continued {cont}: "
          f"{where(e.download(0), ref2['grid'])}", flush=True)


case("direct 512x4096 K8 persistent", 512, 4096, 8, True, -1)
case("direct 512x4096 K8 per-chunk", 512, 4096, 8, True, 0)
case("direct 96x300 K8 per-chunk", 96, 300, 8, True, 0, cols=256)
case("direct 512x4096 K8 persistent, continue 3", 512, 4096, 8, True, -1, cont=3)
case("lone 256x1000 K6 persistent", 256, 1000, 6, False, 1, boundary=1, cols=256)
case("lone 256x1000 K6 per-chunk", 256, 1000, 6, False, 0, boundary=1, cols=256)
