"""Cost of cross-stream event waits between back-to-back stencil launches (4096^2, K=8).

A: kernels back-to-back on one stream; B: + wait on an event recorded once on an idle
stream; C: + record an event after every kernel; D: + wait on an event recorded each
iteration on a second stream after a tiny kernel there; E: B with hipEventDisableTiming
events created by torch (torch events are timing-disabled by default).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from heat2d_amd import ops  # noqa: E402

g, u = ops.alloc_tile(4096, 4096, 8)
v = torch.zeros_like(u)
ops.init_tile(u, g)
s1 = torch.cuda.Stream()
s2 = torch.cuda.Stream()
tiny = torch.zeros(1, device="cuda")


def run(mode, iters=200):
    e_once = torch.cuda.Event()
    with torch.cuda.stream(s2):
        e_once.record()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(s1):
        a, b = u, v
        for i in range(iters):
            if mode == "B":
                s1.wait_event(e_once)
            if mode == "D":
                e = torch.cuda.Event()
                with torch.cuda.stream(s2):
                    tiny.add_(1)
                    e.record()
                s1.wait_event(e)
            ops.stencil(a, b, g, K=8)
            if mode == "C":
                torch.cuda.Event().record()
            a, b = b, a
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


for m in "ABCD":
    run(m, 20)
for r in range(2):
    print("  ".join(f"{m}: {run(m):7.2f} us/chunk" for m in "ABCD"))
