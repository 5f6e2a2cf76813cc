"""Planner knobs around the default chunk depth at 4096^2 (ref): wave capacity (units per round)
and edge weights for K = 6, 7, 8; us/step, median of 5 x 420 steps after a 0.3 s pre-warm."""
import os
import statistics
import sys
import time

import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
side = int(sys.argv[1]) if len(sys.argv) > 1 else 4096


def t(K, **kw):
    e = n.Engine(side, side, device=0, small_grid_lds=False, tiled=0, tblock=K, **kw)
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        e.run(K * 10)
        e.synchronize()
    xs = []
    for _ in range(5):
        e.synchronize()
        t0 = time.perf_counter()
        e.run(420)
        e.synchronize()
        xs.append((time.perf_counter() - t0) / 420 * 1e6)
    return statistics.median(xs), e.num_units(K), e.rows_per_wave(K)


for K in (7, 8, 6):
    for cap in (0, 1008, 992, 960):
        us, u, h = t(K, wave_capacity=cap)
        print(f"K={K} cap={cap:4d}: {us:6.3f} us/step units={u} H={h}", flush=True)
for K in (7,):
    for ew, rw in ((1.0, 1.0), (1.1, 1.1), (1.3, 1.15), (1.5, 1.2)):
        us, u, h = t(K, edge_weight=ew, row_edge_weight=rw)
        print(f"K={K} col_w={ew:4.2f} row_w={rw:4.2f}: {us:6.3f} us/step units={u} H={h}", flush=True)
