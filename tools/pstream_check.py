"""Persistent pipelined stencil: bit-exactness against the oracle and us/step against the
launch-per-chunk kernel, alone and through the row-periodic direct IPC pipeline (the per-rank
shape of 4096^2 strong scaling).

Usage: python tools/pstream_check.py [check] [time] [phases]
(the round-3 depth and strip-width sweeps of profiles/pstream_r3.txt: git 6b5b463)"""
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
what = set(sys.argv[1:]) or {"check", "time"}


def engine(nx, ny, K, pers, direct=False, **kw):
    if direct:
        e = n.Engine(nx, ny, periodic_x=True, tblock=K, device=0, ranks=[0], transport=n.TRANSPORT_IPC,
                     halo_timeout_s=5.0, persistent=pers, **kw)
        e.ipc_open([e.ipc_handle()])
        e.ipc_prime()
        return e
    return n.Engine(nx, ny, tblock=K, device=0, small_grid_lds=False, tiled=0, persistent=pers, halo_timeout_s=5.0, **kw)


if "check" in what:
    for nx, ny, K, steps, boundary, direct in [(300, 517, 7, 37, 0, False), (300, 517, 6, 36, 1, False),
                                               (512, 4096, 6, 60, 0, False), (257, 1000, 4, 41, 1, False),
                                               (96, 300, 5, 3 * 5 + 11, 0, True), (512, 4096, 6, 60, 0, True),
                                               (1024, 4096, 7, 70, 1, True), (300, 701, 8, 37, 1, True),
                                               (2048, 4096, 7, 140, 0, False), (203, 611, 1, 5, 0, False),
                                               (203, 611, 2, 7, 0, False), (203, 611, 3, 9, 1, False),
                                               (64, 611, 1, 5, 0, False), (512, 611, 1, 5, 0, False)]:
      for cols in (256, 128):
          e = engine(nx, ny, K, 1, direct=direct, boundary=boundary, poison=True, pstream_cols=cols)
          units = e.pstream_units(K)
          hs = sorted({u[2] for u in units})
          print(f"  plan: {len(units)} units, h {hs[:3]}..{hs[-3:]}" if units else "  plan: none", flush=True)
          try:
              st = e.run(steps)
          except RuntimeError as ex:
              print(f"check {nx}x{ny} K={K}: FAILED {ex}", flush=True)
              continue
          got = e.download(0)
          ref = n.oracle_run(nx, ny, steps, boundary=boundary, periodic_x=direct)["grid"]
          d = got != ref
          r, c = np.nonzero(d)
          print(f"check {nx}x{ny} K={K} cols={cols} steps={steps} b={boundary} direct={direct}: launches {e.pstream_launches()} "
                f"chunks {st['chunks']} wrong {int(d.sum())}"
                + (f" rows {r.min()}-{r.max()} cols {c.min()}-{c.max()} nan {int(np.isnan(got).sum())}" if d.any() else ""),
                flush=True)
          # continue: a second run (new launch, progress counters continue)
          e.run(steps)
          ref2 = n.oracle_run(nx, ny, 2 * steps, boundary=boundary, periodic_x=direct)["grid"]
          print(f"   second run: wrong {int((e.download(0) != ref2).sum())}", flush=True)
          del e


def timed(e, steps, reps=5):
    e.run(steps)
    best = 1e9
    for _ in range(reps):
        e.synchronize()
        t0 = time.perf_counter()
        e.run(steps)
        e.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best / steps * 1e6


if "time" in what:
    for nx, ny, K, steps in [(512, 4096, 6, 840), (1024, 4096, 7, 840), (2048, 4096, 7, 840), (4096, 4096, 7, 840),
                             (4096, 4096, 7, 20), (512, 4096, 6, 24)]:
        for direct in (False, True):
            row = []
            for pers in (0, 1):
                e = engine(nx, ny, K, pers, direct=direct)
                row.append(timed(e, steps))
                del e
            print(f"time {nx}x{ny} K={K} steps={steps} direct={direct}: per-chunk {row[0]:.3f} us/step, "
                  f"persistent {row[1]:.3f} us/step ({row[0] / row[1]:.3f}x)", flush=True)

if "phases" in what:
    # where a chunk's time goes (per wave, per chunk, us): phase timers of the persistent kernel
    names = ["drain", "start-wait", "flag-wait", "prologue", "steady", "in-loop-wait"]
    for nx, K, cols in ((512, 8, 128), (512, 8, 256), (1024, 8, 256), (1024, 8, 128), (4096, 7, 256)):
        e = engine(nx, 4096, K, 1, direct=True, pstream_cols=cols, phase_timers=True)
        us = timed(e, 840)
        e.reset_halo_wait()
        e.run(840)
        p = e.pstream_phases()
        per = [v / max(1.0, p[0]) for v in p[1:]]
        print(f"phases {nx}x4096 K={K} cols={cols}: {us:.3f} us/step, chunk {us * K:.2f} us; per wave-chunk: "
              + ", ".join(f"{nm} {v:.2f}" for nm, v in zip(names, per)) + f"; sum {sum(per):.2f}", flush=True)
        del e
