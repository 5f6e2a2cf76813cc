"""Print the analytic cost models (heat2d_amd/utils/model.py).

  python tools/model.py report   # the report's Tables 14-19 (strips/blocks time, speedup, efficiency)
  python tools/model.py mi355x   # predicted strong scaling on 1/2/4/8 MI355X: 4096^2, 8192^2, 16384^2
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from heat2d_amd.utils import model as M  # noqa: E402


def report():
    for kind, nums in (("strips", (14, 15, 16)), ("blocks", (17, 18, 19))):
        tab = M.report_tables(M.REPORT_GRIDS, M.REPORT_PROCS, kind)
        for title, idx, num in (("time (s)", 1, nums[0]), ("speedup", 2, nums[1]), ("efficiency", 3, nums[2])):
            print(f"\nTable {num} (model, {kind}): {title}; P = {M.REPORT_PROCS}")
            for (m, n), rows in tab.items():
                print(f"{m}x{n:<6}" + "".join(f"{r[idx]:>11.4g}" for r in rows))


def mi355x():
    for side in (4096, 8192, 16384):
        for layout in ("rows", "blocks"):
            print(f"\n{side}^2 strong scaling, {layout}, 1000 steps (model)")
            print("GPUs  tile         K  us/step   time(s)   speedup  efficiency  cell-updates/s")
            for r in M.strong_scaling(side, [1, 2, 4, 8], layout, 1000):
                print(f"{r['gpus']:>4}  {r['tile'][0]:>5}x{r['tile'][1]:<6} {r['K']:>2} {r['us_per_step']:8.2f} "
                      f"{r['time_s']:9.5f} {r['speedup']:9.2f} {r['efficiency']:10.2f}  {r['cups']:.3e}")


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "both"
    if what in ("report", "both"):
        report()
    if what in ("mi355x", "both"):
        mi355x()
