"""Diagnostics: the local two-tile serial pipeline with checks every 9 steps, engines created and
released in the order of the failing suite test (the next engine built while the previous one is
alive, the previous one released right before the next run).  Prints per attempt whether the run
converged at the oracle's step with its grid."""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
CONV = dict(convergence=True, interval=9, sensitivity=1.93e13)
nx, ny = 257, 509
ref = n.oracle_run(nx, ny, 3000, boundary=1, **CONV)
order = sys.argv[1] if len(sys.argv) > 1 else "create-first"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
eng = None
for rep in range(reps):
    for gx, gy in ((2, 1), (1, 2)):
        for fused in (-1, 0):
            if order == "release-first":
                eng = None
            eng = n.Engine(nx, ny, gridx=gx, gridy=gy, boundary=1, tblock=8, device=0, fused_check=fused,
                           small_grid_lds=False, tiled=0, overlap=False, **CONV)
            try:
                st = eng.run(3000)
            except RuntimeError as ex:
                print(f"rep {rep} {gx}x{gy} fused={fused}: ERROR {ex}", flush=True)
                sys.exit(1)
            got = np.zeros((nx, ny), np.float32)
            for t in range(eng.num_tiles()):
                g = eng.geom(t)
                got[g["gx0"]:g["gx0"] + g["xcell"], g["gy0"]:g["gy0"] + g["ycell"]] = eng.download(t)
            ok = st["converged"] and st["steps_done"] == ref["steps_done"] and np.array_equal(got, ref["grid"])
            print(f"rep {rep} {order} {gx}x{gy} fused={fused}: {'ok' if ok else 'WRONG'} steps {st['steps_done']}",
                  flush=True)
