"""Table-4-style measurement on one MI355X: 1000 steps of each reference grid with and without
the convergence check every 20 steps (sensitivity 0: the check runs but never stops the run,
as in the reference's timed runs), device-side fused check vs the host-synchronised one.
Prints a markdown table (seconds for 1000 steps, like Report.pdf Tables 1 and 4)."""
import os
import sys
import time

import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
grids = [(80, 64), (160, 128), (320, 256), (640, 512), (1280, 1024), (2560, 2048), (4096, 4096)]
steps = 1000


def timed(direct=False, **kw):
    if direct:  # one rank's tile of a multi-GPU run: row-periodic self-exchange, direct IPC pipeline
        e = n.Engine(device=0, periodic_x=True, ranks=[0], transport=n.TRANSPORT_IPC, halo_timeout_s=5.0, **kw)
        e.ipc_open([e.ipc_handle()])
        e.ipc_prime()
    else:
        e = n.Engine(device=0, boundary=1, **kw)  # grad semantics (zero ghost ring), as the reference's MPI code
    e.run(200)
    best = 1e9
    for _ in range(3):
        e.synchronize()
        t0 = time.perf_counter()
        st = e.run(steps)
        e.synchronize()
        best = min(best, time.perf_counter() - t0)
    assert st["steps_done"] == e.steps_done()
    return best, st["path"]


# bring the GPU to its steady power state first: the small grids alone barely load it
_w = n.Engine(4096, 4096, device=0, tiled=0, small_grid_lds=False)
_t_end = time.perf_counter() + 1.5
while time.perf_counter() < _t_end:
    _w.run(70)
    _w.synchronize()
del _w

print("| grid | no check (s) | check every 20, fused (s) | overhead | check every 20, host-synced (s) | overhead | path |")
print("|---|---|---|---|---|---|---|")
for nx, ny in grids:
    t0, path = timed(nx=nx, ny=ny)
    conv = dict(convergence=True, interval=20, sensitivity=0.0)
    t1, _ = timed(nx=nx, ny=ny, **conv)
    t2, _ = timed(nx=nx, ny=ny, fused_check=0, **conv)
    print(f"| {nx}x{ny} | {t0:.3e} | {t1:.3e} | {100 * (t1 / t0 - 1):+.1f} % | {t2:.3e} | {100 * (t2 / t0 - 1):+.1f} % "
          f"| {path} |", flush=True)
# multi-rank rows (one GPU): a rank's tile of 4096^2 over 8 / 4 GPUs through the direct pipeline in a
# row-periodic self-exchange (the decision through the IPC all-reduce; persistent launches between checks)
for nx, ny, K in ((512, 4096, 8), (1024, 4096, 8)):
    t0, path = timed(direct=True, nx=nx, ny=ny, tblock=K)
    conv = dict(convergence=True, interval=20, sensitivity=0.0)
    t1, _ = timed(direct=True, nx=nx, ny=ny, tblock=K, **conv)
    t2, _ = timed(direct=True, nx=nx, ny=ny, tblock=K, fused_check=0, **conv)
    print(f"| {nx}x{ny} rank tile, direct | {t0:.3e} | {t1:.3e} | {100 * (t1 / t0 - 1):+.1f} % | {t2:.3e} | "
          f"{100 * (t2 / t0 - 1):+.1f} % | {path} |", flush=True)
