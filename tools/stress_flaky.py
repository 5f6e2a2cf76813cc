"""Diagnostics: repeat the configurations whose GPU tests failed intermittently (2-D direct
self-exchange; two local tiles through the serial pipeline) many times in one process and count
wrong results, per variant (store flavour, fences), to find the mechanism."""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
cache = {}


def ref(key, fn):
    if key not in cache:
        cache[key] = fn()
    return cache[key]


def gather(e, nx, ny):
    out = np.zeros((nx, ny), np.float32)
    for t in range(e.num_tiles()):
        g = e.geom(t)
        out[g["gx0"]:g["gx0"] + g["xcell"], g["gy0"]:g["gy0"] + g["ycell"]] = e.download(t)
    return out


def run2d(**kw):
    nx, ny, K, b = 257, 4096, 5, 1
    steps = 3 * K + 11
    e = n.Engine(nx, ny, periodic_x=True, periodic_y=True, boundary=b, tblock=K, device=0, ranks=[0],
                 transport=n.TRANSPORT_IPC, halo_timeout_s=5.0, poison=True, **kw)
    e.ipc_open([e.ipc_handle()])
    e.ipc_prime()
    e.run(steps)
    got = e.download(0)
    r = ref(("2d", steps), lambda: n.oracle_run(nx, ny, steps, boundary=b, periodic_x=True, periodic_y=True)["grid"])
    return got, r


def runserial(**kw):
    nx, ny = 257, 509
    e = n.Engine(nx, ny, gridx=2, gridy=1, boundary=1, tblock=8, device=0, small_grid_lds=False, tiled=0,
                 overlap=False, convergence=True, interval=9, sensitivity=0.0, fused_check=0, **kw)
    e.run(27)
    got = gather(e, nx, ny)
    r = ref(("serial", 27), lambda: n.oracle_run(nx, ny, 27, boundary=1)["grid"])
    return got, r


for name, fn, variants in (("2d-direct", run2d, [{}, {"wt_store": 0}, {"direct_acquire": 0}, {"direct_release": 0}]),
                           ("serial-2x1", runserial, [{}, {"wt_store": 0}])):
    for kw in variants:
        bad = 0
        first = None
        for i in range(reps):
            got, r = fn(**kw)
            d = got != r
            if d.any():
                bad += 1
                if first is None:
                    rr, cc = np.nonzero(d)
                    first = (i, int(d.sum()), int(rr.min()), int(rr.max()), int(cc.min()), int(cc.max()),
                             int(np.isnan(got).sum()))
        print(f"{name} {kw}: {bad}/{reps} wrong; first (rep, cells, rows, cols, nan) {first}", flush=True)
