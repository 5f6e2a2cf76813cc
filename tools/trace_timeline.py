"""Summarise a rocprofv3 kernel_trace.csv as a steady-state timeline.

Prints, for a window of consecutive kernels in the middle of the trace, start/end offsets
(us) relative to the window start, duration, queue and a short kernel name; then per-name
mean durations and the mean period of the most frequent kernel.
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"stream_kernel<(\d+), (\w+), (\w+)>|stream_kernelILi(\d+)ELb(\d)ELb(\d)", name)
    if m:
        return "stream_k" + (m.group(1) or m.group(4))
    name = re.sub(r"\(.*", "", name)
    return name.split("::")[-1][:40]


rows = list(csv.DictReader(open(sys.argv[1])))
win = int(sys.argv[2]) if len(sys.argv) > 2 else 40
key_s = next(k for k in rows[0] if "Start_Timestamp" in k)
key_e = next(k for k in rows[0] if "End_Timestamp" in k)
key_q = next((k for k in rows[0] if k in ("Stream_Id", "Queue_Id")), None)
ev = sorted((int(r[key_s]), int(r[key_e]), r.get(key_q, "?"), short(r["Kernel_Name"])) for r in rows)
core = [x for x in ev if "rocclr" not in x[3]]
mid = len(core) * 3 // 4
w = core[mid:mid + win]
t0 = w[0][0]
for s, e, q, nm in w:
    print(f"{(s - t0) / 1e3:9.2f} {(e - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f}  q={q:>3} {nm}")
dur = defaultdict(list)
for s, e, q, nm in ev[len(ev) // 4:]:
    dur[nm].append((e - s) / 1e3)
print("--- mean durations (us), last 3/4 of trace")
for nm, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    print(f"{nm:42s} n={len(v):5d} mean={sum(v) / len(v):8.2f}")
