"""Tuning sweep of the streaming kernel: time per step for (precision, K, H) in ONE process,
interleaved rounds (cdna_hip_programming.md §5.4 rule 24).  Usage on the GPU box:

    python tools/sweep.py --n 4096 --steps 400 --rounds 3 > gpurun_out/sweep.txt
"""
import argparse
import itertools
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import heat2d_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--ny", type=int, default=0)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--K", default="1,2,4,6,8,10,12,16")
    ap.add_argument("--H", default="0,16,32,64,128")
    ap.add_argument("--prec", default="0,1")
    ap.add_argument("--boundary", type=int, default=0)
    ap.add_argument("--ew", default="1.15")
    ap.add_argument("--periodic", action="store_true")
    a = ap.parse_args()
    n = heat2d_amd.native()
    ny = a.ny or a.n
    cases = list(itertools.product([int(p) for p in a.prec.split(",")], [int(k) for k in a.K.split(",")],
                                   [int(h) for h in a.H.split(",")], [float(o) for o in a.ew.split(",")]))
    engines = {}
    for p, K, H, ew in cases:
        e = n.Engine(a.n, ny, precision=p, tblock=K, rows_per_wave=H, device=0, small_grid_lds=False, tiled=0,
                     edge_weight=ew, boundary=a.boundary, periodic_x=a.periodic, periodic_y=a.periodic)
        e.run(K * 4)
        engines[(p, K, H, ew)] = e
    res = {c: [] for c in cases}
    for r in range(a.rounds):
        for c in cases:
            e = engines[c]
            e.synchronize()
            t0 = time.perf_counter()
            st = e.run(a.steps)
            e.synchronize()
            dt = time.perf_counter() - t0
            res[c].append((dt, st["device_ms"] / 1e3))
    print(f"grid {a.n}x{ny}, {a.steps} steps; us/step (wall min, device min), Gcups")
    best = {}
    for c in cases:
        w = min(x[0] for x in res[c])
        d = min(x[1] for x in res[c])
        cups = a.n * ny * a.steps / w
        H = engines[c].rows_per_wave(c[1])
        nu = engines[c].num_units(c[1])
        print(f"prec={'ref' if c[0] == 0 else 'fp32'} K={c[1]:2d} H={c[2]:3d}(eff {H:3d},{nu:5d}u) ew={c[3]} "
              f"{w / a.steps * 1e6:8.2f} {d / a.steps * 1e6:8.2f}  {cups / 1e9:9.1f}")
        if c[0] not in best or cups > best[c[0]][1]:
            best[c[0]] = (c, cups)
    for p, (c, cups) in best.items():
        print(f"BEST prec={p}: K={c[1]} H={c[2]} ew={c[3]} -> {cups / 1e9:.1f} Gcups")


if __name__ == "__main__":
    main()
