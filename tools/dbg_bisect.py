"""Diagnostics: bit-exactness of small single-tile runs under the kernel debug switches
(EngineOptions::debug_kernel), to localise a wrong-cell pattern."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
cases = [(257, 509, 1, 8, 2), (203, 611, 0, 2, 7), (203, 611, 1, 7, 17), (64, 256, 1, 8, 23), (4096, 4096, 0, 7, 20)]
for dbg in (0, 1, 2, 4, 8):
    for nx, ny, bnd, K, steps in cases:
        e = n.Engine(nx, ny, boundary=bnd, tblock=K, device=0, small_grid_lds=False, tiled=0, debug_kernel=dbg)
        try:
            e.run(steps)
            got = e.download(0)
            ref = n.oracle_run(nx, ny, steps, boundary=bnd)["grid"]
            bad = got != ref
            r, c = np.nonzero(bad)
            print(f"dbg={dbg} {nx}x{ny} b={bnd} K={K} steps={steps}: wrong {int(bad.sum())}"
                  + (f" rows {sorted(set(r.tolist()))[:8]} cols {sorted(set(c.tolist()))[:12]}" if bad.any() else ""), flush=True)
        except Exception as ex:  # noqa: BLE001
            print(f"dbg={dbg} {nx}x{ny}: {type(ex).__name__}: {ex}", flush=True)
        del e
