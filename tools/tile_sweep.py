"""Small/medium-grid path sweep on one GPU: the whole-grid LDS solver, the streaming kernel
and LDS-tiled configurations (width RY, steps per launch K, tile rows TX, workgroup size NT, cells per lane CPL), at the reference's
published grid sizes (Report.pdf p.21/p.26).  Prints us/step (best of 3, device time).

  python tools/tile_sweep.py [--steps 1000] [--sizes 80x64,160x128,...] [--precision ref|fp32]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import heat2d_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=1000)
ap.add_argument("--sizes", default="80x64,160x128,320x256,640x512,1280x1024,2560x2048")
ap.add_argument("--precision", default="ref")
ap.add_argument("--quick", action="store_true", help="fewer tiled configurations")
a = ap.parse_args()
n = heat2d_amd.native()
prec = 0 if a.precision == "ref" else 1


def best_us(e, steps):
    e.run(min(steps, 200))
    return min(e.run(steps)["device_ms"] for _ in range(3)) * 1e3 / steps


for size in a.sizes.split(","):
    nx, ny = (int(v) for v in size.split("x"))
    rows = []
    if n.lds_solver_fits(nx, ny):
        rows.append(("lds", best_us(n.Engine(nx, ny, precision=prec, device=0, tiled=0), a.steps)))
    rows.append(("stream K8", best_us(n.Engine(nx, ny, precision=prec, device=0, tiled=0, small_grid_lds=False), a.steps)))
    auto = n.Engine(nx, ny, precision=prec, device=0)
    rows.append((f"auto {auto.tile_config() + [auto.tile_threads(), auto.tile_cpl()] if auto.tiled() else ''}", best_us(auto, a.steps)))
    widths = (32, 64, 128)
    ks = (4, 8, 12, 16) if not a.quick else (6, 8, 12, 16)
    txs = (4, 8, 16, 32, 64) if not a.quick else (4, 8, 16, 32)
    for w in widths:
        for K in ks:
            for tx in txs:
                for nt in ((256, 1024) if not a.quick else (1024,)):
                    for cpl in (1, 2, 4):
                        if w // cpl > 64:
                            continue
                        try:
                            e = n.Engine(nx, ny, precision=prec, device=0, tiled=1, tile_width=w, tile_k=K,
                                         tile_rows=tx, tile_threads=nt, tile_cpl=cpl, small_grid_lds=False)
                        except Exception:
                            continue
                        rows.append((f"tiled RY={w:3d} K={K:2d} TX={tx:2d} NT={nt:4d} CPL={cpl}", best_us(e, a.steps)))
    rows.sort(key=lambda r: r[1])
    print(f"== {nx}x{ny} ({a.precision}, {a.steps} steps): best {rows[0][0]} {rows[0][1]:.3f} us/step", flush=True)
    for name, us in rows[:8]:
        print(f"   {name:32s} {us:8.3f} us/step  {nx * ny / us / 1e3:8.2f} Gcups", flush=True)
    for name, us in rows:
        if name.startswith(("lds", "stream", "auto")) and (name, us) not in rows[:8]:
            print(f"   {name:32s} {us:8.3f} us/step  {nx * ny / us / 1e3:8.2f} Gcups", flush=True)
