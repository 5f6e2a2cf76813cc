"""Multi-rank pipeline shape on one GPU: a 4096^2 tile with a row-periodic RCCL
self-exchange (the per-rank shape of the 1-D row-strip bench at N > 1: two K-deep N/S
halos per chunk).

  python tools/overlap_trace.py matrix        # us/step for a matrix of pipeline options
  python tools/overlap_trace.py one [k=v...]  # one config, e.g. for
      rocprofv3 --kernel-trace -d gpurun_out/ot -o ot --output-format csv -- \
          python3 tools/overlap_trace.py one comm_cus=8 contiguous_halo=1
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import heat2d_amd  # noqa: E402

n = heat2d_amd.native()
N = int(os.environ.get("OT_N", "4096"))


def make(mode="rccl", **kw):
    if mode == "none":
        return n.Engine(N, N, device=0, small_grid_lds=False, tiled=0, **kw)
    if mode == "local":
        return n.Engine(N, N, periodic_x=True, boundary=1, device=0, small_grid_lds=False, tiled=0, **kw)
    e = n.Engine(N, N, periodic_x=True, boundary=1, device=0, ranks=[0], transport=n.TRANSPORT_RCCL,
                 small_grid_lds=False, tiled=0, **kw)
    e.init_rccl(n.Engine.rccl_unique_id(), 1, 0)
    return e


def timeit(e, steps=400):
    e.synchronize()
    t0 = time.perf_counter()
    e.run(steps)
    e.synchronize()
    return (time.perf_counter() - t0) / steps * 1e6


if sys.argv[1:2] == ["one"]:
    kw = {k: int(v) for k, v in (a.split("=") for a in sys.argv[2:])}
    mode = {0: "rccl", 1: "local", 2: "none"}[kw.pop("mode", 0)]
    e = make(mode, **kw)
    e.run(800)
    print(f"{mode} {kw}: {timeit(e):.2f} us/step (capacity {e.wave_capacity(8)}, units {e.num_units(8)})")
    sys.exit(0)

cases = {"none (no exchange)": make("none")}
for spec in (sys.argv[2:] if sys.argv[1:2] == ["matrix"] and len(sys.argv) > 2 else
             ["signal_exchange=2", "signal_exchange=2 reserve_waves=0", "signal_exchange=2 reserve_waves=8",
              "signal_exchange=0 concurrent=1", "signal_exchange=0 concurrent=0"]):
    kw = {k: int(v) for k, v in (t.split("=") for t in spec.split())}
    cases["rccl " + spec] = make("rccl", **kw)
for e in cases.values():
    e.run(800)
res = {k: [] for k in cases}
for r in range(5):  # interleaved repeats: clock drift hits every case alike
    for k, e in cases.items():
        res[k].append(timeit(e))
for k, v in res.items():
    print(f"{k:50s} min {min(v):7.2f}  median {sorted(v)[len(v) // 2]:7.2f} us/step")
