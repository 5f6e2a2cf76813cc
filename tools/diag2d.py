"""Diagnostic: the 2-D direct self-exchange (periodic x and y, one rank) run chunk by chunk
against the oracle — where and when do cells go wrong, and which units own them."""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
nx, ny, tb = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (257, 4096, 5)))
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
steps = 3 * tb + 11


def ranges(v):
    v = sorted(set(int(x) for x in v))
    out, s = [], None
    for i, x in enumerate(v):
        if s is None:
            s = x
        if i + 1 == len(v) or v[i + 1] != x + 1:
            out.append(f"{s}-{x}" if x > s else f"{s}")
            s = None
    return ",".join(out)


order = sys.argv[5] if len(sys.argv) > 5 else "pf"
for poison in [c == "p" for c in order]:
    for rep in range(reps):
        e = n.Engine(nx, ny, periodic_x=True, periodic_y=True, boundary=1, tblock=tb, device=0, ranks=[0],
                     transport=n.TRANSPORT_IPC, halo_timeout_s=5.0, poison=poison)
        e.ipc_open([e.ipc_handle()])
        e.ipc_prime()
        K0, _ = e.next_chunk(0, steps)
        if rep == 0:
            units = e.unit_list(0, K0, 3)
            print(f"K={K0} units={len(units)} halo={sum(1 for u in units if (u[3] & 16) or u[7])}")
            last = max(u[0] for u in units)
            for i, u in enumerate(units):
                if u[0] in (0, last) and (u[1] > nx - 40 or u[1] < 12):
                    print(f"  #{i} strip={u[0]} x0={u[1]} h={u[2]} flags={u[3]} cb={u[4]} out=[{u[5]},{u[6]}) "
                          f"links={u[7]:#06x}")
        done = 0
        while done < steps:
            k, _ = e.next_chunk(done, steps)
            e.run(k)
            done += k
            got = e.download(0)
            ref = n.oracle_run(nx, ny, done, boundary=1, periodic_x=True, periodic_y=True)["grid"]
            d = got != ref
            if d.any():
                rows, cols = np.nonzero(d)
                print(f"poison={poison} rep={rep}: wrong after {done} steps (k={k}): {int(d.sum())} cells "
                      f"(nan {int(np.isnan(got).sum())}), rows {ranges(rows)} cols {ranges(cols)}; "
                      f"e.g. got {got[rows[0], cols[0]]} ref {ref[rows[0], cols[0]]}", flush=True)
                break
        else:
            print(f"poison={poison} rep={rep}: ok", flush=True)
        del e
