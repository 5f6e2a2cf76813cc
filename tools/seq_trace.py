"""Kernel-trace sequence statistics of a rocprofv3 database: mean duration of each kernel grouped by
the kernel that ran before it on the same queue (a launch right after a different kernel may pay
cold instruction / scalar caches).  usage: python tools/seq_trace.py DB [name-substring]"""
import sqlite3
import statistics
import sys
from collections import defaultdict


def short(name):
    name = name.split("(")[0]
    for key in ("tile_lds_kernel", "stream_kernel", "pstream_kernel", "reduce", "decide", "copy", "fill"):
        if key in name:
            i = name.find("ILb")
            return key + (name[i:i + 40] if i >= 0 else "")
    return name[:50]


def main(db, flt=""):
    c = sqlite3.connect(db)
    sym = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    rows = c.execute("select kernel_id, start, end, queue_id from rocpd_kernel_dispatch order by start").fetchall()
    prev = {}
    groups = defaultdict(list)
    for kid, s, e, q in rows:
        name = short(sym.get(kid, str(kid)))
        groups[(name, prev.get(q, "-"))].append((e - s) / 1e3)
        prev[q] = name
    for (name, before), d in sorted(groups.items(), key=lambda kv: -len(kv[1])):
        if flt and flt not in name:
            continue
        print(f"{name:56s} after {before:56s} n={len(d):6d} mean={statistics.mean(d):8.2f}us "
              f"med={statistics.median(d):8.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
