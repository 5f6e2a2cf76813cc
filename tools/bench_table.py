"""Re-run the reference's published grid sizes (Report.pdf Tables 1, 4, 10, 12)
on one MI355X and print a markdown table next to the published times.

    python tools/bench_table.py [--steps 1000] [--precision ref] [--convergence]

Each configuration runs through the same engine as the CLI (automatic path: LDS-tiled kernel
for small and medium grids, streaming kernel otherwise; ``--tune`` times the candidates first), W=200 untimed warm-up steps after a
0.2 s pre-warm, then the timed run (min of 3).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import heat2d_amd  # noqa: E402

# Published seconds for 1000 steps (Report.pdf p.21, p.23, p.26, p.28).
SIZES = [(80, 64), (160, 128), (320, 256), (640, 512), (1280, 1024), (2560, 2048)]
CUDA_1000 = {(80, 64): 9.15e-3, (160, 128): 2.19e-2, (320, 256): 7.14e-2, (640, 512): 3.27e-1, (1280, 1024): 1.86,
             (2560, 2048): 7.84}
MPI_BEST = {(80, 64): (9.30e-3, "1/4"), (160, 128): (2.91e-2, "1/4"), (320, 256): (1.04e-1, "1/4"),
            (640, 512): (2.13e-1, "20/160"), (1280, 1024): (2.52e-1, "20/160"), (2560, 2048): (5.18e-1, "20/160")}
MPI_SERIAL = {(80, 64): 2.53e-2, (160, 128): 9.87e-2, (320, 256): 7.52e-1, (640, 512): 3.01, (1280, 1024): 12.7,
              (2560, 2048): 50.9}
EXTRA = [(4096, 4096), (8192, 8192), (16384, 16384)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--precision", default="ref", choices=("ref", "fp32"))
    ap.add_argument("--boundary", default="ghost-zero", choices=("fixed", "ghost-zero"),
                    help="the timed reference tables are grad1612 (ghost-zero) runs")
    ap.add_argument("--json", default=None)
    ap.add_argument("--tune", action="store_true", help="autotune K / rows-per-wave per size (setup, untimed)")
    a = ap.parse_args()
    n = heat2d_amd.native()
    prec = 0 if a.precision == "ref" else 1
    bnd = 0 if a.boundary == "fixed" else 1
    rows = []
    from heat2d_amd.config import Config
    from heat2d_amd.solver import autotune

    for (nx, ny) in SIZES + EXTRA:
        cfg = Config(nx=nx, ny=ny, precision=a.precision, boundary=a.boundary)
        kw = {}
        if a.tune and nx * ny <= (1 << 22):
            kw = autotune(cfg, cfg.model(), 0)["engine_kw"]
        e = n.Engine(nx, ny, precision=prec, boundary=bnd, device=0, **kw)
        t_end = time.perf_counter() + 0.2
        while time.perf_counter() < t_end:
            e.run(64)
        e.run(200)
        best = None
        path = ""
        for _ in range(3):
            e.synchronize()
            t0 = time.perf_counter()
            st = e.run(a.steps)
            e.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
            path = st["path"]
        cups = nx * ny * a.steps / best
        rows.append(dict(grid=[nx, ny], steps=a.steps, seconds=best, cups=cups, path=path, engine_kw=kw,
                         cuda_ref_s=CUDA_1000.get((nx, ny)), mpi_best_s=MPI_BEST.get((nx, ny), (None, ""))[0],
                         mpi_best_cfg=MPI_BEST.get((nx, ny), (None, ""))[1], mpi_serial_s=MPI_SERIAL.get((nx, ny))))
    print(f"| grid | MI355X s ({a.steps} steps, {a.precision}) | cell-updates/s | path | ref CUDA s | ×CUDA | "
          f"ref best MPI s (nodes/tasks) | ×MPI best | ×MPI 1/1 |")
    print("|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        nx, ny = r["grid"]
        f = lambda v: "—" if v is None else f"{v:.3g}"  # noqa: E731
        sp = lambda ref: "—" if ref is None else f"{ref / r['seconds']:.0f}"  # noqa: E731
        print(f"| {nx}×{ny} | {r['seconds']:.3e} | {r['cups']:.3e} | {r['path']} | {f(r['cuda_ref_s'])} | "
              f"{sp(r['cuda_ref_s'])} | {f(r['mpi_best_s'])} {r['mpi_best_cfg']} | {sp(r['mpi_best_s'])} | "
              f"{sp(r['mpi_serial_s'])} |")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
