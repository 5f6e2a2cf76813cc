"""Run the persistent kernel on the per-rank strong-scaling shape (512x4096, row-periodic direct
pipeline, depth 8, 128-column strips) for profiling: python tools/prof_pstream.py [rows] [cols]"""
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 512
cols = int(sys.argv[2]) if len(sys.argv) > 2 else 128
e = n.Engine(rows, 4096, periodic_x=True, tblock=8, device=0, ranks=[0], transport=n.TRANSPORT_IPC,
             halo_timeout_s=5.0, pstream_cols=cols)
e.ipc_open([e.ipc_handle()])
e.ipc_prime()
for _ in range(4):
    e.run(840)
e.synchronize()
print("launches", e.pstream_launches())
