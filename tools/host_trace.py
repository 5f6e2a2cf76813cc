"""Host-side cost of a short timed run (the bench's 20-step region) on one GPU.

Runs the bench's lone-tile engine, then R timed runs of S steps, each timed in three pieces:
submit (``run`` returns), then ``synchronize``; prints the medians.  Under
``rocprofv3 --hip-trace --kernel-trace`` the database's HIP API regions and kernel dispatches of
the LAST timed run are printed as one timeline (``--db`` after the run).

usage: python tools/host_trace.py [N] [S] [R]          (default 4096 20 50)
       python tools/host_trace.py --db DB              (timeline of the last run in a database)
"""
import sqlite3
import statistics
import sys
import time


def run(n=4096, steps=20, reps=50):
    sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
    import heat2d_amd  # noqa: F401  (kernel-argument default)
    import torch
    from heat2d_amd._native import native
    nat = native()
    for mode in (2, 3, 0, 1):
        for st in (1, steps):
            e = nat.Engine(n, n, boundary=0, precision=0, tblock=7, device=0, small_grid_lds=False, sync_mode=mode)
            for _ in range(200):
                e.run(st)
            e.synchronize()
            tot, tt = [], []
            for _ in range(reps):
                e.synchronize()
                t0 = time.perf_counter()
                r = e.run(st)
                t1 = time.perf_counter()
                torch.cuda.synchronize()  # the bench's own end (a no-op wait: the run already waited)
                t2 = time.perf_counter()
                tot.append((t1 - t0) * 1e6)
                tt.append((t2 - t0) * 1e6)
            del e
            print(f"{n}x{n} sync_mode {mode} {st:3d} steps x {reps}: run() median {statistics.median(tot):7.1f} us, "
                  f"+ torch sync {statistics.median(tt):7.1f} us ({statistics.median(tt) / st:.3f} us/step)", flush=True)


def timeline(db, last=60):
    c = sqlite3.connect(db)
    regs = c.execute("select name, start, end from regions order by start").fetchall()
    sym = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    ks = c.execute("select kernel_id, start, end from rocpd_kernel_dispatch order by start").fetchall()
    # the timed runs end before the engine's destructor (its hipDeviceSynchronize)
    end = max((r[1] for r in regs if r[0] == "hipDeviceSynchronize"), default=None)
    ev = [(s, e, "api " + n) for n, s, e in regs if end is None or s < end]
    ev += [(s, e, "gpu " + sym.get(k, str(k))[:70]) for k, s, e in ks if end is None or s < end]
    ev = sorted(ev)[-last:]
    t0 = ev[0][0]
    for s, e, n in ev:
        print(f"  +{(s - t0) / 1e3:8.2f} .. +{(e - t0) / 1e3:8.2f} us  {n}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--db":
        timeline(sys.argv[2])
    else:
        run(*[int(x) for x in sys.argv[1:4]])
