"""Per-rank proxy of 4096^2 strong scaling on ONE GPU: the tile a rank owns at N GPUs
(4096/N rows x 4096 columns), run (a) alone without halos and (b) row-periodic through the
direct IPC pipeline (its halo units push to / wait on its own receive buffers, the same
protocol and kernel as between GPUs).  Prints us/step per (N, K) and the implied speedup.
"""
import sys
import time

import torch  # noqa: F401

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
side = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 960
Ks = [int(k) for k in sys.argv[3].split(",")] if len(sys.argv) > 3 else [4, 6, 8, 10, 12, 16]
cap = int(sys.argv[4]) if len(sys.argv) > 4 else 0  # wave_capacity override (0: occupancy query)
# extra engine options, "name=value,name=value" (e.g. wt_store=0)
opts = {kv.split("=")[0]: (float if "." in kv.split("=")[1] else int)(kv.split("=")[1]) for kv in sys.argv[5].split(",") if kv} if len(sys.argv) > 5 else {}
Ns = [int(v) for v in sys.argv[6].split(",")] if len(sys.argv) > 6 else [1, 2, 4, 8, 16]


def timed(e, steps, reps=3):
    e.run(steps // 4)
    best = 1e9
    for _ in range(reps):
        e.synchronize()
        t0 = time.perf_counter()
        e.run(steps)
        e.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best / steps * 1e6


t1 = None
for N in Ns:
    rows = side // N
    for K in Ks:
        plain = n.Engine(rows, side, tblock=K, device=0, small_grid_lds=False, tiled=0, wave_capacity=cap, **opts)
        up = timed(plain, steps)
        del plain
        if N == 1:
            if K == 8:
                t1 = up
            print(f"N={N:2d} tile {rows}x{side} K={K:2d}: {up:7.2f} us/step alone", flush=True)
            continue
        try:
            e = n.Engine(rows, side, periodic_x=True, tblock=K, device=0, ranks=[0], transport=n.TRANSPORT_IPC,
                         halo_timeout_s=5.0, wave_capacity=cap, **opts)
            e.ipc_open([e.ipc_handle()])
            e.ipc_prime()
            ud = timed(e, steps)
            nu = e.num_units(K)
            del e
        except Exception as ex:  # noqa: BLE001
            ud, nu = float("nan"), 0
            print("  direct failed:", ex)
        sp = (t1 / ud) if t1 else float("nan")
        print(f"N={N:2d} tile {rows}x{side} K={K:2d}: {up:7.2f} us/step alone, {ud:7.2f} direct "
              f"(units {nu}) -> speedup {sp:5.2f} eff {sp / N:5.2f}", flush=True)
