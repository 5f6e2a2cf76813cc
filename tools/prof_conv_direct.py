"""Kernel trace of one rank tile's fused convergence checks through the direct pipeline (row-periodic
self-exchange): 1000 steps without and with a check every 20 steps.  Run under
rocprofv3 --kernel-trace, then tools/seq_trace.py.  usage: python tools/prof_conv_direct.py [ROWS] [K]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 512
K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
for conv in (False, True):
    kw = dict(convergence=True, interval=20, sensitivity=0.0) if conv else {}
    e = n.Engine(rows, 4096, device=0, periodic_x=True, ranks=[0], transport=n.TRANSPORT_IPC, halo_timeout_s=5.0,
                 tblock=K, **kw)
    e.ipc_open([e.ipc_handle()])
    e.ipc_prime()
    e.run(200)
    for _ in range(3):
        e.synchronize()
        t0 = time.perf_counter()
        e.run(1000)
        e.synchronize()
        print(f"{rows}x4096 direct K={K} check={conv}: {(time.perf_counter() - t0) * 1e3:.3f} ms per 1000 steps, "
              f"persistent launches {e.pstream_launches()}", flush=True)
    del e
