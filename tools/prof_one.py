"""Run ONE streaming-kernel configuration for profiling (rocprofv3 --pmc / --kernel-trace)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import heat2d_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--rows", type=int, default=0, help="tile rows (default: --n)")
ap.add_argument("--steps", type=int, default=64)
ap.add_argument("--K", type=int, default=4)
ap.add_argument("--H", type=int, default=0)
ap.add_argument("--prec", type=int, default=0)
ap.add_argument("--ew", type=float, default=1.15)
ap.add_argument("--boundary", type=int, default=0)
ap.add_argument("--periodic", action="store_true")
a = ap.parse_args()
n = heat2d_amd.native()
e = n.Engine(a.rows or a.n, a.n, precision=a.prec, tblock=a.K, rows_per_wave=a.H, device=0, small_grid_lds=False, tiled=0,
             boundary=a.boundary, edge_weight=a.ew, periodic_x=a.periodic, periodic_y=a.periodic)
st = e.run(a.steps)
e.synchronize()
print(st)
