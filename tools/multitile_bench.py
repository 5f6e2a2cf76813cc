"""Single-GPU rehearsal of the multi-rank pipeline: one grid as 1x1 vs GRIDX×GRIDY local tiles
(halo exchange by device copies, boundary-first overlap) and a periodic 1-rank RCCL
self-exchange.  Prints us/step per configuration (min over rounds, interleaved)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import heat2d_amd  # noqa: E402

n = heat2d_amd.native()
N = int(os.environ.get("MT_N", "8192"))
steps = int(os.environ.get("MT_STEPS", "200"))
cases = {}
for (gx, gy) in [(1, 1), (2, 1), (4, 1), (8, 1), (2, 2), (2, 4)]:
    for ov in (True, False):
        if (gx, gy) == (1, 1) and not ov:
            continue
        cases[f"local {gx}x{gy} overlap={ov}"] = n.Engine(N, N, gridx=gx, gridy=gy, device=0, overlap=ov,
                                                          small_grid_lds=False, tiled=0)
for ov in (True, False):
    e = n.Engine(4096, 4096, periodic_x=True, periodic_y=True, boundary=1, device=0, ranks=[0],
                 transport=n.TRANSPORT_RCCL, overlap=ov, small_grid_lds=False, tiled=0)
    e.init_rccl(n.Engine.rccl_unique_id(), 1, 0)
    cases[f"rccl-self 4096^2 periodic overlap={ov}"] = e
for cc in (0, 1):
    e = n.Engine(4096, 4096, periodic_x=True, boundary=1, device=0, ranks=[0], transport=n.TRANSPORT_RCCL,
                 concurrent=cc, small_grid_lds=False, tiled=0)
    e.init_rccl(n.Engine.rccl_unique_id(), 1, 0)
    cases[f"rccl-self 4096^2 periodic-x concurrent={cc}"] = e
    cases[f"local 4096^2 periodic-x concurrent={cc}"] = n.Engine(4096, 4096, periodic_x=True, boundary=1, device=0,
                                                                 concurrent=cc, small_grid_lds=False, tiled=0)
cases["local 4096^2 periodic 1x1 overlap=True"] = n.Engine(4096, 4096, periodic_x=True, periodic_y=True, boundary=1,
                                                           device=0, small_grid_lds=False, tiled=0)
cases["single 4096^2 (no exchange)"] = n.Engine(4096, 4096, device=0, small_grid_lds=False, tiled=0)
for e in cases.values():
    e.run(16)
res = {k: [] for k in cases}
for r in range(3):
    for k, e in cases.items():
        e.synchronize()
        t0 = time.perf_counter()
        st = e.run(steps)
        e.synchronize()
        res[k].append((time.perf_counter() - t0) / steps * 1e6)
for k, v in res.items():
    print(f"{k:45s} {min(v):8.2f} us/step")
