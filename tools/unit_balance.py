"""Work-unit balance of streaming launches from a `tools/timeline.py ... --json OUT --units` file:
per edge class (f0 plain, f1 column edge, f2 row edge, f3 corner; +signal/push halo units of the
direct pipeline) the body time (halo-ready -> end) median / max and per (h + K) cost relative to
plain units, the launch span, and the slowest units with their placement (XCD, SE, CU, SIMD).

usage: python tools/unit_balance.py OUT.json [launch index, default 2]"""
import json
import sys

import numpy as np

KUNIT_NS = 1 << 4  # Unit::flags bit of a halo unit facing N / S (kernels.h kUnitNS)


def analyse(case, L):
    a = np.array(L["unit_rows"], dtype=np.int64)
    start, ready, end, hw, strip, x0, h, flags = (a[:, i] for i in range(8))
    K = L["K"]
    body = (end - ready) * 0.01
    wait = (ready - start) * 0.01
    edge = flags & 3
    ns = (flags & KUNIT_NS) != 0
    print(f"== {case}: K={K} units={len(a)} span {L['span_us']:.2f} us, wait med {np.median(wait):.2f} "
          f"max {wait.max():.2f}")
    plain = (edge == 0) & ~ns
    ref = np.median(body[plain] / (h[plain] + K)) if plain.any() else None
    for name, m in (("plain", plain), ("col edge", (edge == 1) & ~ns), ("row edge", (edge == 2) & ~ns),
                    ("corner", (edge == 3) & ~ns), ("halo (N/S)", ns)):
        if not m.any():
            continue
        rel = np.median(body[m] / (h[m] + K)) / ref if ref else float("nan")
        print(f"   {name:10s} n {int(m.sum()):4d} h {int(h[m].min())}-{int(h[m].max())} body med {np.median(body[m]):6.2f} "
              f"max {body[m].max():6.2f}  per (h+K) x{rel:.3f}")
    hwid = hw & 0xFFFF
    idx = np.argsort(-body)[:8]
    print("   slowest: " + "; ".join(
        f"{body[i]:.2f} us strip {int(strip[i])} x0 {int(x0[i])} h {int(h[i])} flags {int(flags[i])} "
        f"xcc {int(hw[i] >> 16)} se {int((hwid[i] >> 13) & 3)} cu {int((hwid[i] >> 8) & 15)}" for i in idx))


def main():
    d = json.load(open(sys.argv[1]))
    li = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    for r in d:
        Ls = r["launches"]
        if not Ls or "unit_rows" not in Ls[min(li, len(Ls) - 1)]:
            continue
        analyse(r["case"], Ls[min(li, len(Ls) - 1)])


if __name__ == "__main__":
    main()
