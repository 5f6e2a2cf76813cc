"""Summarise a rocprofv3 SQLite database (rocpd): per-kernel dispatch durations, the gaps between
consecutive dispatches of one queue, and PMC counters summed per kernel name.
usage: rocpd_summary.py DB [name-substring]"""
import sqlite3
import statistics
import sys
from collections import defaultdict

db = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
c = sqlite3.connect(db)


def cols(t):
    return [r[1] for r in c.execute(f"pragma table_info({t})")]


kd = cols("rocpd_kernel_dispatch")
sym = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
rows = c.execute("select id, kernel_id, start, end, queue_id from rocpd_kernel_dispatch order by start").fetchall()
by = defaultdict(list)
last_end = {}
gaps = defaultdict(list)
for did, kid, s, e, q in rows:
    name = sym.get(kid, str(kid))
    by[name].append((e - s) / 1e3)
    if q in last_end:
        gaps[name].append((s - last_end[q]) / 1e3)
    last_end[q] = e
for name, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    if flt and flt not in name:
        continue
    g = gaps.get(name, [0.0])
    short = name if len(name) < 70 else name[:67] + "..."
    print(f"{short:70s} n={len(d):5d} mean={statistics.mean(d):9.2f}us med={statistics.median(d):9.2f} "
          f"gap_med={statistics.median(g):7.2f}us")
try:
    pmc = {r[0]: r[1] for r in c.execute("select id, name from rocpd_info_pmc")}
    ev = c.execute("select e.pmc_id, e.value, d.kernel_id from rocpd_pmc_event e join rocpd_kernel_dispatch d "
                   "on e.event_id = d.event_id").fetchall()
    agg = defaultdict(float)
    cnt = defaultdict(set)
    for pid, v, kid in ev:
        name = sym.get(kid, str(kid))
        if flt and flt not in name:
            continue
        agg[(name, pmc.get(pid, pid))] += v
    for (name, p), v in sorted(agg.items()):
        print(f"PMC {name[:50]:50s} {p:24s} {v:.4e}")
except Exception as ex:  # noqa: BLE001
    print("no pmc:", ex)
