"""Where the ~17 us between the kernels' 154 us and a timed 20-step run go (4096^2, K=7)."""
import os
import statistics
import sys
import time

import ctypes

FLAGS = int(os.environ.get("HOST_OVH_FLAGS", "-1"))
if FLAGS >= 0:  # hipSetDeviceFlags before any HIP use: 1 = hipDeviceScheduleSpin, 2 = Yield, 4 = BlockingSync
    hip = ctypes.CDLL("libamdhip64.so")
    print("hipSetDeviceFlags", FLAGS, "->", hip.hipSetDeviceFlags(ctypes.c_uint(FLAGS)))

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
e = n.Engine(4096, 4096, tblock=7, device=0, small_grid_lds=False, tiled=0, sync_mode=2)
torch.cuda.set_device(0)
t_end = time.perf_counter() + 1.5
while time.perf_counter() < t_end:
    e.run(20)


def med(fn, reps=300):
    xs = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        xs.append((time.perf_counter() - t0) * 1e6)
    return statistics.median(xs), min(xs)


print("engine.run(0)             med %.1f min %.1f us" % med(lambda: e.run(0)))
print("torch.cuda.synchronize()  med %.1f min %.1f us" % med(lambda: torch.cuda.synchronize()))
print("engine.run(20)            med %.1f min %.1f us" % med(lambda: e.run(20)))
print("engine.run(20) + tsync    med %.1f min %.1f us" % med(lambda: (e.run(20), torch.cuda.synchronize())))
print("engine.run(7)             med %.1f min %.1f us" % med(lambda: e.run(7)))
print("engine.run(14)            med %.1f min %.1f us" % med(lambda: e.run(14)))
print("engine.run(21)            med %.1f min %.1f us" % med(lambda: e.run(21)))
print("engine.run(700)/100       med %.2f us/step" % (med(lambda: e.run(700), 20)[0] / 700))
