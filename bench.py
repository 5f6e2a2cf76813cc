"""Headline benchmark: cell-updates/s of the 5-point Jacobi heat stencil on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 it is launched
by ``torch.distributed.run`` with one rank per GPU.  A "step" is one Jacobi time step of the
whole grid.  W untimed warm-up steps, then EXACTLY K timed steps bracketed by a barrier and
``torch.cuda.synchronize()`` on both sides; the max over ranks is reported by rank 0 as one
JSON line.

Config (BASELINE.json): 4096×4096 fp32 grid, 1000 steps, center-hot initial field
(synthetic — computed on device from the exact fp64 formula; no dataset involved).
Numerics: the bit-exact reference expression (fp32 storage, fp64 arithmetic exactly as the
reference's C evaluates it) unless ``--precision fp32``.

Scaling: ``--scaling weak`` (default) gives every GPU a 4096×4096 tile; ``--scaling strong``
splits one 4096×4096 grid over the N GPUs.  Decomposition ``--layout rows`` (default): 1-D
row strips (GRIDX = N, the BASELINE's "1D row decomposition with RCCL ghost-row send/recv"),
whose few halo-dependent work units run on a second stream CONCURRENTLY with the interior
while the K-deep ghost rows move over xGMI by RCCL send/recv; ``--layout blocks``: 2-D
near-square blocks (e.g. 2×4).
``vs_baseline`` divides by the reference's best published throughput, 1.01e10 cell-updates/s
(2560×2048, 160 MPI tasks on 20 nodes, Report.pdf p.21 Table 1 — BASELINE.md).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# one hardware queue per engine stream (see heat2d_amd/_native.py); before torch initialises HIP
if os.environ.get("HEAT2D_KEEP_HW_QUEUES") != "1" and int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

BASELINE_CUPS = 1.01e10


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--side", type=int, default=4096, help="grid side (per GPU for weak scaling)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak")
    ap.add_argument("--precision", choices=("ref", "fp32"), default="ref")
    ap.add_argument("--boundary", choices=("fixed", "ghost-zero"), default="fixed")
    ap.add_argument("--tblock", type=int, default=8)
    ap.add_argument("--rows-per-wave", type=int, default=0)
    ap.add_argument("--transport", choices=("auto", "rccl", "torch", "host"), default="auto")
    ap.add_argument("--layout", choices=("rows", "blocks"), default="rows")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--repeat", type=int, default=1, help="timed repetitions (best reported)")
    ap.add_argument("--prewarm-s", type=float, default=0.3,
                    help="seconds of untimed stencil work before the warm-up steps, so the GPU reaches its "
                         "steady power state (the first ~10 ms after idle run at lower clocks)")
    ap.add_argument("--device", choices=("gpu", "cpu"), default="gpu",
                    help="cpu: rehearsal of the distributed contract on the host (gloo), not a benchmark")
    a = ap.parse_args()

    import torch

    from heat2d_amd.config import Config, auto_grid
    from heat2d_amd.parallel.dist import init_distributed
    from heat2d_amd.solver import Solver

    ctx = init_distributed()
    world = ctx.world
    if world != a.gpus and world > 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    gx, gy = (world, 1) if a.layout == "rows" else auto_grid(world)
    if a.scaling == "weak":
        nx, ny = a.side * gx, a.side * gy
    else:
        nx = ny = a.side
    cfg = Config(preset="heat2d", nx=nx, ny=ny, steps=a.steps, gridx=gx, gridy=gy, boundary=a.boundary,
                 precision=a.precision, init="exact", output="none", device=a.device, transport=a.transport,
                 tblock=a.tblock, rows_per_wave=a.rows_per_wave, overlap=not a.no_overlap, quiet=True,
                 report="grad", text_style="grad")
    s = Solver(cfg, ctx)

    on_gpu = a.device == "gpu"

    def sync_barrier():
        if on_gpu:
            torch.cuda.synchronize()
        ctx.barrier()
        if on_gpu:
            torch.cuda.synchronize()

    # pre-warm (untimed, time-based) then the W warm-up steps (untimed)
    run = s.run_steps
    prewarm_steps = 0
    if on_gpu and a.prewarm_s > 0:
        # the batch count is agreed collectively: ranks that ran different step counts would
        # post unmatched halo sends/receives and deadlock
        sync_barrier()
        t0 = time.perf_counter()
        run(64)
        sync_barrier()
        t_batch = ctx.allreduce_max(time.perf_counter() - t0)
        batches = max(0, min(100000, math.ceil(a.prewarm_s / max(t_batch, 1e-6)) - 1))
        run(64 * batches)
        prewarm_steps = 64 * (batches + 1)
        sync_barrier()
    if a.warmup > 0:
        run(a.warmup)
    best = None
    res = None
    times = []
    for _ in range(max(1, a.repeat)):
        sync_barrier()
        t0 = time.perf_counter()
        res = run(a.steps)
        sync_barrier()
        dt = ctx.allreduce_max(time.perf_counter() - t0)
        times.append(dt)
        best = dt if best is None else min(best, dt)
    expect = prewarm_steps + max(0, a.warmup) + a.steps * max(1, a.repeat)
    if res["steps_done"] != expect:
        raise SystemExit(f"bench: step accounting error ({res['steps_done']} != {expect})")
    cups = float(nx) * float(ny) * a.steps / best
    if ctx.rank == 0:
        out = {
            "metric": "cell-updates/sec (whole node), 4096^2 grid 1000 steps",
            "value": cups,
            "unit": "cell-updates/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": best * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": cups / BASELINE_CUPS,
            "dtype": "fp32",
            "compute": ("fp64 expression, bit-exact with the reference" if a.precision == "ref" else "fp32 FMA"),
            "data": "synthetic center-hot initial field (exact formula, generated on device)",
            "elapsed_s": best,
            "repeats_s": times,
            "prewarm_steps": prewarm_steps,
            "config": {
                "model": "heat2d 5-point Jacobi, fixed edges" if a.boundary == "fixed" else "heat2d 5-point Jacobi, zero ghost ring",
                "grid": [nx, ny],
                "grid_per_gpu": [nx // gx, ny // gy],
                "global_batch": nx * ny,
                "seq_len": a.steps,
                "parallelism": (f"rows{gx}" if a.layout == "rows" else f"blocks{gx}x{gy}") if world > 1 else "single",
                "overlap": s.engine.pipeline(),
                "tblock": s.engine.halo_depth(),
                "path": res["path"],
                "transport": cfg.transport,
            },
        }
        print(json.dumps(out), flush=True)
    ctx.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
