"""Direct-pipeline fence variants on the per-rank strong-scaling tile (row-periodic self-exchange),
each checked bit-exact against the CPU oracle on a small grid first."""
import os
import sys
import time

import numpy as np
import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()


def mk(rows, cols, K, rel, acq):
    e = n.Engine(rows, cols, periodic_x=True, tblock=K, device=0, ranks=[0], transport=n.TRANSPORT_IPC,
                 halo_timeout_s=5.0, direct_release=rel, direct_acquire=acq)
    e.ipc_open([e.ipc_handle()])
    e.ipc_prime()
    return e


for rel in (0, 1, 2):
    for acq in (0, 1, 2):
        e = mk(96, 700, 8, rel, acq)
        e.run(45)
        ok = np.array_equal(e.download(0), n.oracle_run(96, 700, 45, periodic_x=True)["grid"])
        del e
        res = []
        for rows, K in ((512, 6), (512, 8), (1024, 8), (2048, 8)):
            e = mk(rows, 4096, K, rel, acq)
            e.run(240)
            best = 1e9
            for _ in range(3):
                e.synchronize()
                t0 = time.perf_counter()
                e.run(960)
                e.synchronize()
                best = min(best, (time.perf_counter() - t0) / 960 * 1e6)
            res.append(f"{rows}xK{K} {best:5.2f}")
            del e
        print(f"release={rel} acquire={acq} exact={ok}: " + "  ".join(res), flush=True)
