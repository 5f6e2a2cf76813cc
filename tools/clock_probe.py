"""Does run length change the per-step time of a small grid (GPU clock ramp under a light load)?
  python tools/clock_probe.py NX NY [engine options as k=v ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import heat2d_amd  # noqa: E402

n = heat2d_amd.native()
nx, ny = int(sys.argv[1]), int(sys.argv[2])
kw = {k: int(v) for k, v in (x.split("=") for x in sys.argv[3:])}
e = n.Engine(nx, ny, device=0, **kw)
print("path", e.run(16)["path"], e.tile_config() if e.tiled() else "", flush=True)
for steps in (1000, 10000, 100000, 1000, 300000, 1000):
    t0 = time.perf_counter()
    st = e.run(steps)
    wall = time.perf_counter() - t0
    print(f"{steps:7d} steps: {st['device_ms'] * 1e3 / steps:.3f} us/step device, {wall * 1e6 / steps:.3f} wall", flush=True)
