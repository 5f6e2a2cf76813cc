"""Headline benchmark: cell-updates/s of the 5-point Jacobi heat stencil on MI355X, with the
speedup and efficiency over GPUs that the reference's Tables 1-3 report (Report.pdf p.21-22).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 it is launched
by ``torch.distributed.run`` with one rank per GPU.  A "step" is one Jacobi time step of the
whole grid.  W untimed warm-up steps, then EXACTLY K timed steps bracketed by a barrier and
``torch.cuda.synchronize()`` on both sides; the max over ranks is reported by rank 0 as one
JSON line.  ``value`` is the whole-job throughput (all GPUs).  The timed run is repeated
(``--repeat``, default 3, each exactly K steps behind its own barrier) and the MEDIAN is
reported, every repetition listed in ``repeats_s``: a 20-step run lasts ~170 µs on one GPU, so
a single host hiccup would otherwise decide the number (one such run took 236 µs).

Default configuration (``--config 4096-strong``, the BASELINE metric): ONE 4096×4096 fp32 grid
split over the N GPUs (strong scaling; 1-D row strips, the layout whose halos are contiguous
rows), center-hot initial field computed on device from the exact fp64 formula (synthetic: no
dataset is involved).  Numerics: the bit-exact reference expression (fp32 storage, fp64
arithmetic exactly as the reference's C evaluates it) unless ``--precision fp32``.
Other BASELINE rows: ``--config 8192x2rows``, ``16384x8blocks``, ``weak-4096``, ``weak-hbm``
(per-GPU tile sized from hipMemGetInfo to fill HBM).

Multi-GPU safety (N > 1): before anything is timed, every candidate (transport, pipeline) —
the requested one, then safer fallbacks — runs a small grid of the same decomposition and
must match the CPU oracle bit for bit on rank 0 (``heat2d_amd/utils/benchmark.py``).  The JSON
says which one passed and what failed.  Speedup/efficiency are measured IN THIS JOB: rank 0
re-runs the same grid (strong) or one tile (weak) on its GPU alone with the same K and W; for
strong scaling it also replays the whole step count and compares every rank's tile with the
single-GPU grid bit for bit (``verified``).

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
# One hardware queue per engine stream (compute and comm must not share one: see
# heat2d_amd/_native.py).  Read once at HIP initialisation, so it is set before torch starts.
if os.environ.get("HEAT2D_KEEP_HW_QUEUES") != "1" and int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"


def main() -> int:
    from heat2d_amd.utils.benchmark import CONFIGS

    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="4096-strong")
    ap.add_argument("--side", type=int, default=0, help="override the config's grid side (per GPU for weak)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default=None, help="override the config's scaling")
    ap.add_argument("--layout", choices=("rows", "blocks"), default=None, help="override the config's layout")
    ap.add_argument("--precision", choices=("ref", "fp32"), default="ref")
    ap.add_argument("--boundary", choices=("fixed", "ghost-zero"), default="fixed")
    # halo depth = deepest chunk, measured at 4096^2 (profiles/tblock_sweep_r2.txt): ref 7 (1000 steps
    # 7.57-7.66 vs 7.61-7.78 us/step with 8; 20 steps run as 7+7+6 either way), fp32 8 (4.35e12 vs
    # 3.79e12 cell-updates/s with 7)
    ap.add_argument("--tblock", type=int, default=0, help="halo depth / deepest chunk (0: 7 for ref, 8 for fp32)")
    ap.add_argument("--rows-per-wave", type=int, default=0)
    ap.add_argument("--transport", choices=("auto", "ipc", "rccl", "torch", "host"), default="auto")
    ap.add_argument("--pipeline", choices=("auto", "signal", "concurrent", "boundary-first", "serial"), default="auto")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--no-gate", action="store_true", help="skip the pre-timing correctness gate (N > 1)")
    ap.add_argument("--no-reference", action="store_true", help="skip the in-job single-GPU reference run")
    ap.add_argument("--repeat", type=int, default=3,
                    help="timed runs of exactly --steps steps each; the MEDIAN is reported (a 20-step run lasts "
                         "~170 us, so one host hiccup would otherwise decide the number), all are in repeats_s")
    ap.add_argument("--prewarm-s", type=float, default=1.5,
                    help="seconds of untimed stencil work before the warm-up steps, so the GPU reaches its "
                         "steady power state: with 0.3 s, the first bench on a box that had been idle timed "
                         "236/194/180 us for its three 20-step runs (steady: ~171 us)")
    ap.add_argument("--sync-mode", type=int, default=2, choices=(0, 1, 2, 3),
                    help="engine end-of-run synchronisation (EngineOptions::sync_mode)")
    ap.add_argument("--device", choices=("gpu", "cpu"), default="gpu",
                    help="cpu: rehearsal of the distributed contract on the host (gloo), not a benchmark")
    a = ap.parse_args()
    user_tblock = a.tblock
    if a.tblock <= 0:
        a.tblock = 8 if a.precision == "fp32" else 7

    import numpy as np
    import torch

    from heat2d_amd._native import native
    from heat2d_amd.config import Config
    from heat2d_amd.parallel.dist import init_distributed
    from heat2d_amd.solver import Solver
    from heat2d_amd.utils import benchmark as B

    ctx = init_distributed()
    world = ctx.world
    if world != a.gpus and world > 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    on_gpu = a.device == "gpu"
    n = native()
    ndev = n.device_count() if on_gpu else 0
    if on_gpu and ndev == 0:
        raise SystemExit("bench: no HIP device (use --device cpu for a host rehearsal)")
    device = (ctx.local_rank % ndev) if on_gpu else -1
    ctx.distinct_devices = on_gpu and world <= ndev
    if on_gpu:
        torch.cuda.set_device(device)

    bc = B.CONFIGS[a.config]
    scaling = a.scaling or bc.scaling
    layout = a.layout or bc.layout
    side = a.side or bc.side
    fill_hbm = side == 0
    if fill_hbm:
        if not on_gpu:
            side = 64
        else:
            free, _total = n.mem_info(device)
            side = B.fill_hbm_side(int(ctx.allreduce_min(free)), G=a.tblock)
    nx, ny, gx, gy = B.grid_for(world, side, scaling, layout)
    ref_tblock = a.tblock  # depth of the in-job single-GPU reference (a whole grid / one tile)
    if user_tblock <= 0 and a.precision == "ref" and nx // gx <= 1024:
        # short per-rank tiles (4096^2 over >= 4 GPUs): the K-cone of ~9-17-row units favours 6
        # (512x4096 alone: 20 steps 2.99 vs 3.12 us/step, 840 steps 2.01 vs 2.20; 1024 rows equal;
        # 2048 rows 7 is best: profiles/small_tile_k_r2.txt)
        a.tblock = 6

    def config(nx_, ny_, steps_, transport, pipeline, gridx, gridy):
        return Config(preset="heat2d", nx=nx_, ny=ny_, steps=steps_, gridx=gridx, gridy=gridy, boundary=a.boundary,
                      precision=a.precision, init="exact", output="none", device=a.device, transport=transport,
                      tblock=a.tblock, rows_per_wave=a.rows_per_wave, overlap=not a.no_overlap, pipeline=pipeline,
                      quiet=True, report="grad", text_style="grad", sync_mode=a.sync_mode)

    # ---- correctness gate + transport/pipeline choice (N > 1) ------------------------------
    cands = B.candidates(a.transport, a.pipeline, world, on_gpu, ctx.distinct_devices, layout)
    gate = None
    if world > 1 and not a.no_gate:
        bnd = 0 if a.boundary == "fixed" else 1
        prec = 0 if a.precision == "ref" else 1

        def make_gate_solver(transport, pipeline, gnx, gny, gsteps):
            c = config(gnx, gny, gsteps, transport, pipeline, gx, gy)
            c.halo_timeout_s = 5.0
            return Solver(c, ctx)

        gate = B.run_gate(ctx, make_gate_solver,
                          lambda gnx, gny, gsteps: n.oracle_run(gnx, gny, gsteps, boundary=bnd, precision=prec)["grid"],
                          cands, gx, gy, a.tblock, log=lambda m: print(m, file=sys.stderr, flush=True))
        if not gate.ok:
            if ctx.rank == 0:
                print(json.dumps({"error": "no transport passed the correctness gate", "gate": gate.tried}), flush=True)
            ctx.shutdown()
            return 3
        transport, pipeline = gate.transport, gate.pipeline
    else:
        transport, pipeline = cands[0]
    transport_cfg = "auto" if transport == "local" else transport

    cfg = config(nx, ny, a.steps, transport_cfg, pipeline, gx, gy)
    s = Solver(cfg, ctx)

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    def sync_barrier():
        sync()
        ctx.barrier()
        # device-level alignment (RCCL all-reduce) when every rank has its own GPU
        if on_gpu and not ctx.device_barrier(device):
            sync()
        # host-level alignment: node-local spin barrier (exit skew ~1 us instead of gloo's tens)
        ctx.node_barrier()

    # ---- pre-warm (untimed, time-based, collectively agreed count) + W warm-up steps --------
    # The pre-warm replays the timed run's exact shape (runs of K steps: the same chunk depths,
    # so the same kernel code is hot in the caches) until the GPU has been busy ~prewarm_s.
    run = s.run_steps
    prewarm_steps = 0
    if on_gpu and a.prewarm_s > 0 and a.steps > 0:
        # ranks that ran different step counts would post unmatched halo sends and deadlock
        sync_barrier()
        t0 = time.perf_counter()
        run(a.steps)
        sync_barrier()
        t_batch = ctx.allreduce_max(time.perf_counter() - t0)
        batches = max(0, min(20000, math.ceil(a.prewarm_s / max(t_batch, 1e-6)) - 1))
        for _ in range(batches):
            run(a.steps)
        prewarm_steps = a.steps * (batches + 1)
        sync_barrier()
    if a.warmup > 0:
        run(a.warmup)

    # ---- timed region -----------------------------------------------------------------------
    res, times = None, []
    for _ in range(max(1, a.repeat)):
        sync_barrier()
        t0 = time.perf_counter()
        res = run(a.steps)
        sync()
        dt = ctx.allreduce_max(time.perf_counter() - t0)
        times.append(dt)
    best = sorted(times)[(len(times) - 1) // 2]  # median (lower median for an even count)
    total_steps = prewarm_steps + max(0, a.warmup) + a.steps * max(1, a.repeat)
    if res["steps_done"] != total_steps:
        raise SystemExit(f"bench: step accounting error ({res['steps_done']} != {total_steps})")
    cups = float(nx) * float(ny) * a.steps / best
    pipeline_used = s.engine.pipeline()
    halo_depth = s.engine.halo_depth()
    path = res["path"]

    # ---- in-job single-GPU reference: speedup / efficiency, and bit-exact verification ------
    t1 = None
    verified = None
    ref_note = None
    if world == 1:
        t1 = best
    elif not a.no_reference and not fill_hbm:
        # strong: the same global grid on rank 0's GPU alone; weak: one GPU's tile alone
        rnx, rny = (nx, ny) if scaling == "strong" else (side, side)
        digests = ctx.gather_objects(B.grid_digest(s.tiles()) if scaling == "strong" else None)
        if ctx.rank == 0:
            e = n.Engine(rnx, rny, boundary=0 if a.boundary == "fixed" else 1,
                         precision=0 if a.precision == "ref" else 1, tblock=ref_tblock,
                         rows_per_wave=a.rows_per_wave, device=device, small_grid_lds=False)
            # the same step count as the multi-GPU run, its last pre-warm run shaped like the timed one
            if prewarm_steps >= a.steps:
                e.run(prewarm_steps - a.steps) if prewarm_steps > a.steps else None
                e.run(a.steps)
            elif prewarm_steps > 0:
                e.run(prewarm_steps)
            if a.warmup > 0:
                e.run(a.warmup)
            ts = []
            for _ in range(max(1, a.repeat)):
                e.synchronize()
                t0 = time.perf_counter()
                e.run(a.steps)
                e.synchronize()
                ts.append(time.perf_counter() - t0)
            t1 = sorted(ts)[(len(ts) - 1) // 2]
            if scaling == "strong":
                full = e.download(0)
                verified = all(B.digest_of_region(full, k) == v for d in digests for k, v in d.items())
            ref_note = (f"rank 0's GPU alone, {'same grid' if scaling == 'strong' else 'one tile'}, "
                        f"same K/W, measured in this job")
            del e
        ctx.barrier()

    # ---- report ---------------------------------------------------------------------------------
    if ctx.rank == 0:
        if t1 is not None:
            if scaling == "strong":
                speedup = t1 / best
                eff = speedup / world
            else:  # weak: each GPU does the work of the 1-GPU run
                eff = t1 / best
                speedup = eff * world
        else:
            speedup = eff = None
        out = {
            "metric": B.metric_label(nx, ny, a.steps),
            "value": cups,
            "unit": "cell-updates/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": best * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": cups / B.BASELINE_CUPS,
            "speedup": speedup,
            "efficiency": eff,
            "t1_ms_per_step": (t1 * 1e3 / a.steps) if t1 is not None else None,
            "speedup_reference": ref_note or ("this run (N=1)" if world == 1 else None),
            "verified": verified,
            "dtype": "fp32",
            "compute": ("fp64 expression, bit-exact with the reference" if a.precision == "ref" else "fp32 FMA"),
            "data": "synthetic center-hot initial field (exact formula, generated on device)",
            "elapsed_s": best,
            "repeats_s": times,
            "timing": f"median of {len(times)} timed runs of exactly {a.steps} steps (max over ranks each)",
            "prewarm_steps": prewarm_steps,
            "gate": (gate.tried if gate is not None else None),
            "config": {
                "name": a.config,
                "model": ("heat2d 5-point Jacobi, fixed edges" if a.boundary == "fixed"
                          else "heat2d 5-point Jacobi, zero ghost ring"),
                "grid": [nx, ny],
                "grid_per_gpu": [nx // gx, ny // gy],
                "global_batch": nx * ny,
                "seq_len": a.steps,
                "parallelism": B.parallelism_label(world, gx, gy),
                "transport": transport,
                "pipeline": pipeline_used,
                "tblock": halo_depth,
                "path": path,
                "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
            },
        }
        print(json.dumps(out), flush=True)
    ctx.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
