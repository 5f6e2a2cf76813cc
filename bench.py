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

Verification of what is timed: before anything else runs on the timed solver, it advances
exactly K steps from the initial field and rank 0 compares every rank's tile with the CPU
oracle bit for bit (grids up to ~2^30 cell-updates; larger ones verify as many leading steps as
fit and say so).  A configuration that fails this is not timed: the next candidate is tried.

Multi-GPU safety (N > 1): every candidate (transport, pipeline) — direct IPC with the measured
fences, direct IPC with system-scope fences, RCCL, host staging — first runs a small grid of the
same decomposition, plain and with convergence checks, and must match the CPU oracle bit for bit
(``heat2d_amd/utils/benchmark.py``).  The JSON says which one passed and what failed.
Speedup/efficiency are measured IN THIS JOB: rank 0 runs the same grid (strong) or one tile
(weak) on its GPU alone with the same K and W; for strong scaling it also replays the whole step
count and compares every rank's tile with the single-GPU grid bit for bit.  For the HBM-filling
weak config the single-GPU tile is timed BEFORE the N-rank solver allocates (both would not fit).

``halo_wait`` (N > 1, direct pipeline): the exposed halo wait of the halo units inside the
stencil kernel (s_memrealtime around the flag poll) during the timed runs — the analogue of the
reference's mpiP ``MPI_Waitall`` share (Report.pdf p.34-37).

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

VERIFY_BUDGET = 1 << 30  # cell-updates the CPU oracle may spend on verifying the timed solver


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
    ap.add_argument("--pipeline", choices=("auto", "direct-sys", "signal", "serial"), default="auto")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--no-gate", action="store_true", help="skip the pre-timing correctness gate (N > 1)")
    ap.add_argument("--no-reference", action="store_true", help="skip the in-job single-GPU reference run")
    ap.add_argument("--no-verify", action="store_true", help="skip the oracle check of the timed solver's first steps")
    ap.add_argument("--repeat", type=int, default=3,
                    help="timed runs of exactly --steps steps each; the MEDIAN is reported (a 20-step run lasts "
                         "~170 us, so one host hiccup would otherwise decide the number), all are in repeats_s")
    ap.add_argument("--prewarm-s", type=float, default=1.5,
                    help="seconds of untimed stencil work before the warm-up steps, so the GPU reaches its "
                         "steady power state: with 0.3 s, the first bench on a box that had been idle timed "
                         "236/194/180 us for its three 20-step runs (steady: ~171 us)")
    ap.add_argument("--sync-mode", type=int, default=2, choices=(0, 1, 2, 3),
                    help="engine end-of-run synchronisation (EngineOptions::sync_mode)")
    ap.add_argument("--persistent", choices=("auto", "on", "off"), default="auto",
                    help="persistent stencil launches (auto: the engine's policy, off when ranks share a GPU; "
                         "on: also then — a rehearsal whose ranks' plans fit the GPU together)")
    ap.add_argument("--device", choices=("gpu", "cpu"), default="gpu",
                    help="cpu: rehearsal of the distributed contract on the host (gloo), not a benchmark")
    a = ap.parse_args()
    user_tblock = a.tblock
    if a.tblock <= 0:
        a.tblock = 8 if a.precision == "fp32" else 7

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
    # one physical GPU per rank? (collective; host + PCI bus id, whatever the visibility setup)
    ctx.devices_shared(device, n.device_pci_id(device) if on_gpu else "")
    if on_gpu:
        torch.cuda.set_device(device)
    bnd = 0 if a.boundary == "fixed" else 1
    prec = 0 if a.precision == "ref" else 1

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
    if user_tblock <= 0 and a.precision == "ref" and world > 1 and nx // gx <= 1024:
        # short per-rank tiles (4096^2 over >= 4 GPUs) run the persistent kernel through the direct
        # pipeline, whose fixed cost is per chunk: depth 8 is best there (512x4096 row-periodic,
        # us/step over 840 steps, K 6/7/8: 2.179/2.059/2.034; 1024 rows 2.963/2.869/2.870 —
        # profiles/pstream_r3.txt)
        a.tblock = 8

    def config(nx_, ny_, steps_, transport, pipeline, gridx, gridy, conv=False):
        c = Config(preset="heat2d", nx=nx_, ny=ny_, steps=steps_, gridx=gridx, gridy=gridy, boundary=a.boundary,
                   precision=a.precision, init="exact", output="none", device=a.device, transport=transport,
                   tblock=a.tblock, rows_per_wave=a.rows_per_wave, overlap=not a.no_overlap, pipeline=pipeline,
                   quiet=True, report="grad", text_style="grad", sync_mode=a.sync_mode, persistent=a.persistent)
        if conv:  # checks every G+1 steps that never converge (gate only)
            c.convergence, c.interval, c.sensitivity = True, a.tblock + 1, 0.0
        return c

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

    def solo_timed(e):
        """One engine alone (rank 0's in-job reference): the time-based pre-warm, the W warm-up
        steps, then the median of `repeat` timed runs of exactly --steps steps."""
        if on_gpu and a.prewarm_s > 0 and a.steps > 0:
            t0 = time.perf_counter()
            e.run(a.steps)
            e.synchronize()
            for _ in range(max(0, min(20000, math.ceil(a.prewarm_s / max(time.perf_counter() - t0, 1e-6)) - 1))):
                e.run(a.steps)
        if a.warmup > 0:
            e.run(a.warmup)
        ts = []
        for _ in range(max(1, a.repeat)):
            e.synchronize()
            t0 = time.perf_counter()
            e.run(a.steps)
            e.synchronize()
            ts.append(time.perf_counter() - t0)
        return sorted(ts)[(len(ts) - 1) // 2]

    # ---- weak-hbm: the single-GPU reference tile BEFORE the N-rank solver allocates ----------
    t1_pre = None
    if world > 1 and fill_hbm and not a.no_reference:
        if ctx.rank == 0:
            e = n.Engine(side, side, boundary=bnd, precision=prec, tblock=ref_tblock, rows_per_wave=a.rows_per_wave,
                         device=device, small_grid_lds=False, sync_mode=a.sync_mode)
            t1_pre = solo_timed(e)
            del e
        ctx.barrier()

    # ---- candidate choice: correctness gate, then the timed solver itself must verify --------
    verify_steps = 0
    cells = nx * ny
    if not a.no_verify and a.steps > 0 and cells <= VERIFY_BUDGET:
        verify_steps = max(1, min(a.steps, VERIFY_BUDGET // cells))
    holder = {}

    def build_timed(transport, pipeline):
        """Collective: the timed solver, and its first `verify_steps` steps from the initial field
        checked against the CPU oracle on rank 0.  (ok on this rank, why not)."""
        if "solver" in holder:
            holder.pop("solver").close()
        try:
            s = Solver(config(nx, ny, a.steps, "auto" if transport == "local" else transport, pipeline, gx, gy), ctx)
        except Exception as ex:  # noqa: BLE001 - e.g. a timed strip too short for the transport
            ctx.allreduce_min(0)  # pair with the agreement below on the other ranks
            return 0, f"timed solver: {type(ex).__name__}: {ex}"
        if ctx.allreduce_min(1) < 1:
            s.close()
            return 0, "timed solver failed on another rank"
        holder["solver"] = s
        holder["verified"] = None
        if verify_steps > 0:
            s.run_steps(verify_steps)
            digests = ctx.gather_objects(B.grid_digest(s.tiles()))
            ok = 1
            if ctx.rank == 0:
                ref = n.oracle_run(nx, ny, verify_steps, boundary=bnd, precision=prec)["grid"]
                ok = int(all(B.digest_of_region(ref, k) == v for d in digests for k, v in d.items()))
            ok = int(ctx.allreduce_min(ok))
            holder["verified"] = bool(ok)
            if not ok:
                return 0, f"the timed solver's first {verify_steps} steps differ from the CPU oracle"
        return 1, ""

    rows_per_rank = nx // gx
    cands = B.candidates(a.transport, a.pipeline, world, on_gpu, ctx.distinct_devices, layout,
                         rows_per_rank=rows_per_rank, depth=a.tblock, cols_per_rank=ny // gy)
    gate = None
    log = lambda m: print(m, file=sys.stderr, flush=True)  # noqa: E731
    if world > 1 and not a.no_gate:
        def make_gate_solver(transport, pipeline, gnx, gny, gsteps, conv=False):
            c = config(gnx, gny, gsteps, transport, pipeline, gx, gy, conv=conv)
            c.halo_timeout_s = 5.0
            return Solver(c, ctx)

        gate = B.run_gate(ctx, make_gate_solver,
                          lambda gnx, gny, gsteps: n.oracle_run(gnx, gny, gsteps, boundary=bnd, precision=prec)["grid"],
                          cands, gx, gy, a.tblock, log=log, accept=build_timed)
        if not gate.ok:
            if ctx.rank == 0:
                print(json.dumps({"error": "no transport passed the correctness gate", "gate": gate.tried}), flush=True)
            ctx.shutdown()
            return 3
        transport, pipeline = gate.transport, gate.pipeline
    else:
        transport, pipeline = cands[0]
        ok, why = build_timed(transport, pipeline)
        if not ok:
            if ctx.rank == 0:
                print(json.dumps({"error": why, "transport": transport, "pipeline": pipeline}), flush=True)
            ctx.shutdown()
            return 3
    s = holder["solver"]
    verified_first = holder["verified"]

    # ---- pre-warm + warm-up + timed region ----------------------------------------------------
    run = s.run_steps
    times = []
    prewarm_steps = 0
    if on_gpu and a.prewarm_s > 0 and a.steps > 0:
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
    if on_gpu:
        s.engine.reset_halo_wait()  # the halo-wait counters describe the timed runs only
    res = None
    for _ in range(max(1, a.repeat)):
        sync_barrier()
        t0 = time.perf_counter()
        res = run(a.steps)
        sync()
        times.append(ctx.allreduce_max(time.perf_counter() - t0))
    best = sorted(times)[(len(times) - 1) // 2]  # median (lower median for an even count)
    total_steps = verify_steps + prewarm_steps + max(0, a.warmup) + a.steps * max(1, a.repeat)
    if res["steps_done"] != total_steps:
        raise SystemExit(f"bench: step accounting error ({res['steps_done']} != {total_steps})")
    cups = float(nx) * float(ny) * a.steps / best
    pipeline_used = s.engine.pipeline()
    halo_depth = s.engine.halo_depth()
    path = res["path"]
    halo_wait = None
    if on_gpu and world > 1:
        hw = s.engine.halo_wait()
        chunks = max(1, int(res["chunks"]))
        chunk_us = best * 1e6 / chunks
        mine = (hw["total_us"] / max(1, hw["waits"]), hw["max_us"], hw["waits"])
        allw = ctx.gather_objects(mine)
        if ctx.rank == 0 and hw is not None:
            mean_max = max(w[0] for w in allw)
            halo_wait = {"mean_us_per_halo_unit": mean_max, "max_us": max(w[1] for w in allw),
                         "waits_per_rank": [int(w[2]) for w in allw], "chunk_us": chunk_us,
                         "share_of_chunk": mean_max / chunk_us if chunk_us > 0 else None,
                         "note": "worst rank; in-kernel flag-poll time of the halo units during the timed runs "
                                 "(Report.pdf p.34-37 MPI_Waitall analogue)"}

    # persistent launches per rank over the whole job (0: one launch per chunk)
    plaunches = ctx.gather_objects(int(s.engine.pstream_launches()))

    # ---- in-job single-GPU reference: speedup / efficiency, and bit-exact verification ------
    # (the timed solver is closed first: no two engines coexist on a rank's GPU in the bench)
    digests = None
    if world > 1 and not a.no_reference and not fill_hbm and scaling == "strong":
        digests = ctx.gather_objects(B.grid_digest(s.tiles()))
    holder.pop("solver").close()
    del s
    ctx.barrier()
    t1 = None
    verified_full = None
    ref_note = None
    if world == 1:
        t1 = best
    elif fill_hbm and not a.no_reference:
        t1 = t1_pre  # rank 0 only
        ref_note = "rank 0's GPU alone, one tile, same K/W, measured in this job before the N-rank solver"
    elif not a.no_reference and not fill_hbm:
        # strong: the same global grid on rank 0's GPU alone; weak: one GPU's tile alone
        rnx, rny = (nx, ny) if scaling == "strong" else (side, side)
        if ctx.rank == 0:
            e = n.Engine(rnx, rny, boundary=bnd, precision=prec, tblock=ref_tblock, rows_per_wave=a.rows_per_wave,
                         device=device, small_grid_lds=False)
            # the same step count as the multi-GPU run, its last pre-warm run shaped like the timed one
            if verify_steps > 0:
                e.run(verify_steps)
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
                verified_full = all(B.digest_of_region(full, k) == v for d in digests for k, v in d.items())
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
        checks = [v for v in (verified_first, verified_full) if v is not None]
        verified = all(checks) if checks else None
        how = []
        if verified_first is not None:
            how.append(f"first {verify_steps} steps of the timed solver == CPU oracle "
                       f"({'all' if verify_steps == a.steps else 'leading'} {verify_steps} of --steps {a.steps})")
        if verified_full is not None:
            how.append(f"after all {total_steps} steps every rank's tile == rank 0's single-GPU run")
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
            "verification": "; ".join(how) if how else "none (grid too large for the oracle and no in-job reference)",
            "dtype": "fp32",
            "compute": ("fp64 expression, bit-exact with the reference" if a.precision == "ref" else "fp32 FMA"),
            "data": "synthetic center-hot initial field (exact formula, generated on device)",
            "elapsed_s": best,
            "repeats_s": times,
            "timing": f"median of {len(times)} timed runs of exactly {a.steps} steps (max over ranks each)",
            "prewarm_steps": prewarm_steps,
            "gate": (gate.tried if gate is not None else None),
            "halo_wait": halo_wait,
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
                "candidate": f"{transport}/{pipeline}",
                "tblock": halo_depth,
                "path": path,
                "persistent_launches_per_rank": plaunches,
                "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
            },
        }
        print(json.dumps(out), flush=True)
    ctx.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
