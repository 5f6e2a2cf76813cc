"""Where the convergence check's cost goes on the small reference grids (run under rocprofv3
--kernel-trace): 1000 steps of a grid without and with the fused check every 20 steps."""
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
nx, ny = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "80x64").split("x"))
for conv in (False, True):
    kw = dict(convergence=True, interval=20, sensitivity=0.0) if conv else {}
    e = n.Engine(nx, ny, device=0, boundary=1, **kw)
    e.run(200)
    e.synchronize()
    t0 = time.perf_counter()
    st = e.run(1000)
    e.synchronize()
    print(f"{nx}x{ny} conv={conv}: {time.perf_counter() - t0:.3e} s / 1000 steps, chunks {st['chunks']}, "
          f"path {st['path']}", flush=True)
