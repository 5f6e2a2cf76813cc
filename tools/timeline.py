"""Per-wave timeline of streaming launches (EngineOptions::timeline, s_memrealtime at 100 MHz).

For each recorded launch: dispatch spread (first to last wave start), halo wait, per-unit body
time (ready -> end) by unit class, launch span, and the gap to the next launch — the parts of
the per-launch fixed cost that ``profiles/launch_cost_r2.md`` could only fit as one number.

Usage: python tools/timeline.py ROWSxCOLS:K[:steps][:alone|direct|direct2d[:opt=value...]] ... [--json out.json]
       [--units]  (with --json: every unit's raw stamps and geometry, for per-XCD / per-position analysis)
  direct = the tile row-periodic through the IPC direct pipeline (its own neighbour);
  direct2d = periodic in both dimensions (its own neighbour in all eight directions).
"""
import json
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

TICK_US = 0.01


def summarize(K, st, units):
    start, ready, end = st[:, 0].astype(np.int64), st[:, 1].astype(np.int64), st[:, 2].astype(np.int64)
    t0 = start.min()
    body = (end - ready) * TICK_US
    wait = (ready - start) * TICK_US
    h = np.array([u[2] for u in units])
    flags = np.array([u[3] for u in units])
    edge = flags & 3
    out = {
        "K": K, "units": int(len(st)),
        "dispatch_spread_us": float((start.max() - t0) * TICK_US),
        "wait_us": [float(np.median(wait)), float(wait.max())],
        "body_us": [float(body.min()), float(np.median(body)), float(body.max())],
        "end_spread_us": float((end.max() - end.min()) * TICK_US),
        "span_us": float((end.max() - t0) * TICK_US),
        "h": [int(h.min()), float(np.median(h)), int(h.max())],
        "t_first": int(t0), "t_last": int(end.max()),
    }
    # body time per row-level by unit class: fit body = a + b * (K*h + K*(K-1))
    rl = K * h + K * (K - 1)
    for cls, m in (("plain", edge == 0), ("edge", edge != 0)):
        if m.sum() >= 3 and np.ptp(rl[m]) > 0:
            b, a = np.polyfit(rl[m], body[m], 1)
            out[f"fit_{cls}"] = [float(a), float(b)]
        elif m.sum() > 0:
            out[f"body_{cls}_median"] = float(np.median(body[m]))
    return out


def run_case(n, spec):
    parts = spec.split(":")
    rows, cols = (int(v) for v in parts[0].split("x"))
    K = int(parts[1])
    steps = int(parts[2]) if len(parts) > 2 and parts[2] else 4 * K
    direct = len(parts) > 3 and parts[3] in ("direct", "direct2d")
    kw = dict(tblock=K, device=0, small_grid_lds=False, tiled=0, timeline=64)
    for extra in parts[4:]:  # engine options, name=value (e.g. direct_acquire=2)
        name, value = extra.split("=")
        kw[name] = float(value) if "." in value else int(value)
    if direct:
        # direct2d: periodic in both dimensions — all eight neighbours are the tile itself (the
        # per-rank shape of a 2-D block decomposition)
        e = n.Engine(rows, cols, periodic_x=True, periodic_y=parts[3] == "direct2d", ranks=[0],
                     transport=n.TRANSPORT_IPC, halo_timeout_s=5.0, **kw)
        e.ipc_open([e.ipc_handle()])
        e.ipc_prime()
    else:
        e = n.Engine(rows, cols, **kw)
    for _ in range(20):  # warm: clocks and caches
        e.run(steps)
    e.reset_halo_wait()
    e.run(steps)
    tl = e.timeline()
    hw = e.halo_wait()
    res = {"case": spec, "launches": []}
    prev_last = None
    for Kc, st in tl:
        units = e.unit_list(0, Kc, 3 if direct else 0)
        s = summarize(Kc, st, units)
        if "--units" in sys.argv:  # per-unit raw data: start, ready, end, hw id, and the unit's strip, x0, h, flags
            s["unit_rows"] = [[int(v) for v in st[i, :4]] + [int(units[i][0]), int(units[i][1]), int(units[i][2]),
                                                             int(units[i][3])] for i in range(len(st))]
        if prev_last is not None:
            s["gap_from_prev_us"] = float((s["t_first"] - prev_last) * TICK_US)
        prev_last = s["t_last"]
        res["launches"].append(s)
    first, last = res["launches"][0]["t_first"], res["launches"][-1]["t_last"]
    res["device_span_us"] = float((last - first) * TICK_US)
    res["us_per_step"] = res["device_span_us"] / steps
    res["halo_wait"] = hw
    del e
    return res


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out_json = None
    if "--json" in sys.argv:
        out_json = sys.argv[sys.argv.index("--json") + 1]
        args = [a for a in args if a != out_json]
    n = native()
    results = []
    for spec in args:
        r = run_case(n, spec)
        results.append(r)
        print(f"== {spec}: device span {r['device_span_us']:.1f} us = {r['us_per_step']:.2f} us/step; "
              f"halo wait {r['halo_wait']}", flush=True)
        for L in r["launches"]:
            extra = {k: v for k, v in L.items() if k.startswith("fit_") or k.startswith("body_") and k != "body_us"}
            print(f"   K={L['K']} units={L['units']} h={L['h']} dispatch {L['dispatch_spread_us']:.2f} "
                  f"wait(med,max) {L['wait_us'][0]:.2f},{L['wait_us'][1]:.2f} body(min,med,max) "
                  f"{L['body_us'][0]:.2f},{L['body_us'][1]:.2f},{L['body_us'][2]:.2f} end-spread "
                  f"{L['end_spread_us']:.2f} span {L['span_us']:.2f} gap {L.get('gap_from_prev_us', float('nan')):.2f} "
                  f"{json.dumps(extra)}", flush=True)
    if out_json:
        with open(out_json, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
