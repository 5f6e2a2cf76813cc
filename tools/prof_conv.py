"""Kernel trace of a small grid's 1000 steps without and with the fused check every 20 steps
(run under rocprofv3 --kernel-trace): per-launch time and gaps.  Usage: python tools/prof_conv.py NX NY"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
nx, ny = int(sys.argv[1]), int(sys.argv[2])
for conv in (False, True):
    kw = dict(convergence=True, interval=20, sensitivity=0.0) if conv else {}
    e = n.Engine(nx, ny, device=0, boundary=1, **kw)
    e.run(200)
    for _ in range(3):
        e.synchronize()
        t0 = time.perf_counter()
        e.run(1000)
        e.synchronize()
        print(f"{nx}x{ny} check={conv}: {(time.perf_counter() - t0) * 1e3:.3f} ms per 1000 steps", flush=True)
    del e
