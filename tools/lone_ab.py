"""A/B timing of the lone 4096^2 tile (launch per chunk, depth 7) under debug_kernel settings."""
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
for rep in range(2):
    for dbg in [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1").split(",")]:
        e = n.Engine(4096, 4096, tblock=7, device=0, small_grid_lds=False, sync_mode=2, debug_kernel=dbg)
        e.run(2000)
        best = 1e9
        for _ in range(3):
            e.synchronize()
            t0 = time.perf_counter()
            e.run(1000)
            e.synchronize()
            best = min(best, time.perf_counter() - t0)
        print(f"4096^2 K=7 dbg={dbg}: {best / 1000 * 1e6:.3f} us/step", flush=True)
        del e
