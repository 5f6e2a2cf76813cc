"""A/B timing of the persistent direct pipeline (row-periodic per-rank tiles of 4096^2 strong
scaling on one GPU) under EngineOptions::debug_kernel settings.
Usage: python tools/pstream_ab.py DBG[,DBG...] [ROWS,...]"""
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
dbgs = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0").split(",")]
rows = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "512,1024").split(",")]
for nx in rows:
    for dbg in dbgs:
        for pers in (1, 0):
            e = n.Engine(nx, 4096, periodic_x=True, tblock=8, device=0, ranks=[0], transport=n.TRANSPORT_IPC,
                         halo_timeout_s=5.0, persistent=pers, debug_kernel=dbg)
            e.ipc_open([e.ipc_handle()])
            e.ipc_prime()
            steps = 840
            e.run(steps)
            best = 1e9
            for _ in range(3):
                e.synchronize()
                t0 = time.perf_counter()
                e.run(steps)
                e.synchronize()
                best = min(best, time.perf_counter() - t0)
            print(f"{nx}x4096 K=8 dbg={dbg} persistent={pers}: {best / steps * 1e6:.3f} us/step "
                  f"(launches {e.pstream_launches()})", flush=True)
            del e
