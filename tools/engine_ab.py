"""A/B of several identical (or differently configured) multi-rank-proxy engines in ONE
process, timed interleaved: 4096^2 tile, row-periodic RCCL self-exchange.

  python tools/engine_ab.py "signal_exchange=2" "signal_exchange=2" ...
Each argument is one engine's kwargs; "none" = a single tile without exchange.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import heat2d_amd  # noqa: E402

n = heat2d_amd.native()
N = int(os.environ.get("OT_N", "4096"))
engines = []
for spec in sys.argv[1:]:
    if spec == "none":
        engines.append((spec, n.Engine(N, N, device=0, tiled=0)))
        continue
    kw = {k: int(v) for k, v in (t.split("=") for t in spec.split())}
    e = n.Engine(N, N, periodic_x=True, boundary=1, device=0, ranks=[0], transport=n.TRANSPORT_RCCL, tiled=0, **kw)
    e.init_rccl(n.Engine.rccl_unique_id(), 1, 0)
    engines.append((spec, e))
for _, e in engines:
    e.run(800)
res = {i: [] for i in range(len(engines))}
for r in range(5):
    for i, (_, e) in enumerate(engines):
        e.synchronize()
        t0 = time.perf_counter()
        e.run(400)
        e.synchronize()
        res[i].append((time.perf_counter() - t0) / 400 * 1e6)
for i, (spec, e) in enumerate(engines):
    v = sorted(res[i])
    print(f"[{i}] {spec:40s} min {v[0]:7.2f} median {v[len(v) // 2]:7.2f} us/step  pipeline={e.pipeline()} "
          f"stream={e.stream_handle():#x}", flush=True)
