"""Benchmark plumbing shared by ``bench.py`` and the tests: named configurations (the BASELINE
rows), metric labels, HBM-filling tile sizing, transport/pipeline fallback chains and the
pre-timing correctness gate.

The reference measures wall time of the step loop, max over ranks, and derives speedup
``T1/TP`` and efficiency ``S/P`` offline (``grad1612_mpi_heat.c:206-207,277-280``;
``Report.pdf`` Tables 1-3, p.21-22).  Here both are emitted by the bench itself against a
single-GPU run of the same grid measured in the same job.
"""
from __future__ import annotations

import hashlib
import math
import os
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple

from ..config import auto_grid

BASELINE_CUPS = 1.01e10  # best published throughput: 2560x2048, 160 MPI tasks (Report.pdf p.21, Table 1)


@dataclass(frozen=True)
class BenchConfig:
    """A named benchmark configuration (BASELINE.json ``configs``)."""
    name: str
    side: int            # grid side (strong: whole grid; weak: per GPU); 0 = fill HBM
    scaling: str         # "strong" | "weak"
    layout: str          # multi-GPU decomposition: "rows" (1-D strips) | "blocks" (near-square 2-D)
    note: str = ""


CONFIGS = {
    # BASELINE metric: 4096^2 grid, speedup/efficiency over GPUs (strong scaling)
    "4096-strong": BenchConfig("4096-strong", 4096, "strong", "rows", "BASELINE headline: 4096^2 split over N GPUs"),
    # BASELINE config 3: 8192^2, 2 GPUs, 1-D row decomposition
    "8192x2rows": BenchConfig("8192x2rows", 8192, "strong", "rows", "8192^2, 1-D row strips"),
    # BASELINE config 4: 16384^2, 8 GPUs, 2x4 blocks, halo exchange overlapped with the interior
    "16384x8blocks": BenchConfig("16384x8blocks", 16384, "strong", "blocks", "16384^2, 2-D blocks (2x4 at 8 GPUs)"),
    # weak scaling, 4096^2 per GPU
    "weak-4096": BenchConfig("weak-4096", 4096, "weak", "rows", "4096^2 per GPU, 1-D row strips"),
    # BASELINE config 5: per-GPU tile sized to fill HBM (fp32 double buffer)
    "weak-hbm": BenchConfig("weak-hbm", 0, "weak", "rows", "per-GPU tile filling HBM (two fp32 buffers)"),
}


def grid_for(world: int, side: int, scaling: str, layout: str) -> Tuple[int, int, int, int]:
    """(NX, NY, GRIDX, GRIDY) of a run on `world` GPUs.  Strong: one side×side grid split over
    the GPUs; weak: every GPU owns a side×side tile.  Rows: GRIDX = world (1-D strips of
    whole rows, contiguous halos); blocks: near-square (8 -> 2x4, the BASELINE layout)."""
    if world < 1 or side < 1:
        raise ValueError("world and side must be >= 1")
    gx, gy = (world, 1) if layout == "rows" else auto_grid(world)
    if scaling == "weak":
        return side * gx, side * gy, gx, gy
    if scaling != "strong":
        raise ValueError(f"scaling must be weak or strong, not {scaling!r}")
    return side, side, gx, gy


def tile_bytes(xcell: int, ycell: int, G: int) -> int:
    """Upper bound of the bytes of ONE halo-padded fp32 tile buffer (TileGeom,
    decomposition.cpp make_tile_geom: G ghost rows above/below, left pad PL = max(4,
    round_up(G, 4)), and a row pitch — a multiple of 64 floats — that also holds the last
    256-column wave window, which may reach up to 256 columns past the owned ones)."""
    PL = max(4, (G + 3) // 4 * 4)
    pitch = (PL + ycell + 256 + 63) // 64 * 64
    return (xcell + 2 * G) * pitch * 4


def fill_hbm_side(free_bytes: int, G: int = 8, headroom: float = 0.02, reserve: int = 3 << 30,
                  multiple: int = 256) -> int:
    """Largest square per-GPU tile side (a multiple of `multiple`) whose two fp32 buffers fit in
    `free_bytes` minus `reserve` and a `headroom` fraction (runtime allocations, unit lists)."""
    usable = int(free_bytes * (1.0 - headroom)) - reserve
    if usable <= 0:
        raise ValueError("not enough free device memory for a tile")
    side = int(math.isqrt(usable // 8)) // multiple * multiple
    while side > multiple and 2 * tile_bytes(side, side, G) > usable:
        side -= multiple
    if side < multiple:
        raise ValueError("not enough free device memory for a tile")
    return side


def metric_label(nx: int, ny: int, steps: int) -> str:
    """The BASELINE metric name with this run's actual grid and timed step count."""
    g = f"{nx}^2" if nx == ny else f"{nx}x{ny}"
    return f"cell-updates/sec (whole node) + speedup/efficiency, {g} grid {steps} steps"


def parallelism_label(world: int, gx: int, gy: int) -> str:
    if world == 1:
        return "single"
    return f"rows{gx}" if gy == 1 else f"blocks{gx}x{gy}"


# Engine keyword options of each halo pipeline (EngineOptions, engine.h).  "direct-sys" is the
# direct IPC pipeline with system-scope release before every flag bump and system-scope acquire
# after every halo wait: the documented-safe fences, for when the measured default (no release:
# the payload goes to the peer's uncached memory and is drained before the flag; agent acquire)
# fails between distinct devices.
PIPELINE_OPTIONS = {
    "auto": {},
    "direct-sys": dict(direct_release=0, direct_acquire=0),
    "signal": dict(signal_exchange=2),
    "serial": dict(overlap=False),
}


def candidates(transport: str, pipeline: str, world: int, on_gpu: bool, distinct_devices: bool,
               layout: str, rows_per_rank: int = 1 << 30, depth: int = 8,
               cols_per_rank: int = 1 << 30) -> List[Tuple[str, str]]:
    """(transport, pipeline) pairs to try, in order: the requested one first, then the safer
    fallbacks.  A run is only timed with a pair that passed the gate.  Between distinct devices
    (never exercised on one GPU): direct IPC with the measured fences, direct IPC with
    system-scope fences, RCCL (signalled, then serial), and host staging over gloo as the last
    resort (no device-to-device path at all).  Direct IPC needs tiles of at least 2 * depth rows
    (halo units of at least `depth` rows at both ends of every column strip) and, with west /
    east neighbours (blocks), a width that is a multiple of 4 and at least 32 columns."""
    if world == 1:
        return [("local", pipeline)]
    if not on_gpu:
        return [("torch", "serial")]
    rows = layout == "rows"
    ipc_ok = rows_per_rank >= 2 * depth and (rows or (cols_per_rank % 4 == 0 and cols_per_rank >= 32))
    ipc = [("ipc", "auto"), ("ipc", "direct-sys")] if ipc_ok else []
    if not distinct_devices:  # several ranks per GPU: RCCL refuses them; IPC and gloo host staging work
        chain = ipc if transport in ("auto", "ipc") else []
        return chain + [("host", "serial")]
    chain: List[Tuple[str, str]] = []
    if transport in ("auto", "ipc"):
        chain += ipc
    if transport in ("auto", "rccl"):
        chain += [("rccl", "signal" if pipeline == "auto" else pipeline), ("rccl", "serial")]
    elif transport not in ("ipc", "host"):
        chain += [(transport, pipeline)]
    chain += [("host", "serial")]
    out: List[Tuple[str, str]] = []
    for c in chain:
        if c not in out:
            out.append(c)
    return out


def grid_digest(tiles) -> dict:
    """{(gx0, gy0, rows, cols): blake2b hex} of the owned blocks (bit-level fingerprint)."""
    out = {}
    for gx0, gy0, b in tiles:
        out[(int(gx0), int(gy0), int(b.shape[0]), int(b.shape[1]))] = hashlib.blake2b(b.tobytes(), digest_size=16).hexdigest()
    return out


def digest_of_region(full, key) -> str:
    gx0, gy0, r, c = key
    blk = full[gx0:gx0 + r, gy0:gy0 + c].copy()
    return hashlib.blake2b(blk.tobytes(), digest_size=16).hexdigest()


@dataclass
class GateResult:
    ok: bool
    transport: str
    pipeline: str
    detail: str = ""
    tried: list = field(default_factory=list)


def gate_grid(world: int, gx: int, gy: int, G: int) -> Tuple[int, int, int]:
    """A small grid with the run's decomposition shape: several work units per column strip
    (so the halo units are the full-size signalling kind), three column strips, and a step
    count of a dozen chunks — both receive-buffer parities crossed several times — with
    balanced and ragged chunks."""
    rows = max(6 * G, 48)
    return rows * gx, 700 * gy, 12 * G + 3


def forced_failure(transport: str, pipeline: str) -> bool:
    """Test hook: HEAT2D_GATE_FAIL="ipc,rccl/signal" makes those transports (any pipeline) or
    transport/pipeline pairs fail the gate — rehearses the downgrade path on hardware where they
    would pass."""
    forced = {t for t in os.environ.get("HEAT2D_GATE_FAIL", "").split(",") if t}
    return transport in forced or f"{transport}/{pipeline}" in forced


def gate_one(ctx, make_solver, oracle, transport: str, pipeline: str, gx: int, gy: int, G: int) -> Tuple[int, str]:
    """One candidate on the gate grid, twice: a plain run, then a run with a convergence check
    every G+1 steps that never converges (sensitivity 0: the residual launches, the decision and
    the cross-rank sum all run, the grid is the plain one).  Rank 0 compares the gathered grid
    with the CPU oracle bit for bit.  Returns (ok on this rank, why not)."""
    import numpy as np

    nx, ny, steps = gate_grid(ctx.world, gx, gy, G)
    if forced_failure(transport, pipeline):
        return 0, "failure injected by HEAT2D_GATE_FAIL"
    agree = (lambda v: int(ctx.allreduce_min(v))) if hasattr(ctx, "allreduce_min") else (lambda v: v)
    ref = None
    for conv in (False, True):
        ok, why, s = 1, "", None
        try:
            s = make_solver(transport, pipeline, nx, ny, steps, conv=conv)
            s.run_steps(steps)
            s.engine.synchronize()
            full = s.gather()
            if ctx.rank == 0:
                ref = oracle(nx, ny, steps) if ref is None else ref
                if not np.array_equal(full, ref):
                    ok = 0
                    why = f"mismatch{' (with convergence checks)' if conv else ''}: {int(np.sum(full != ref))} cells differ"
        except Exception as e:  # a failing transport must not take the job down: fall back
            ok, why = 0, f"{type(e).__name__}: {e}"
        finally:
            if s is not None:
                s.close()
        if not agree(ok):  # every rank leaves together (the next phase is collective)
            return 0, why
    return 1, ""


def run_gate(ctx, make_solver: Callable[..., object], oracle: Callable[[int, int, int], object],
             cands: Sequence[Tuple[str, str]], gx: int, gy: int, G: int, log=print,
             accept: Optional[Callable[[str, str], Tuple[int, str]]] = None) -> GateResult:
    """Try each (transport, pipeline) on a small grid of the same decomposition (gate_one).
    Every rank takes part in every attempt and all agree (min over ranks) before moving on.
    `accept` (optional, collective) is a second test of a candidate that passed: e.g. building
    the timed solver and verifying its first steps; a refusal moves on to the next candidate."""
    tried = []
    for transport, pipeline in cands:
        ok, why = gate_one(ctx, make_solver, oracle, transport, pipeline, gx, gy, G)
        ok_all = int(ctx.allreduce_min(ok)) if hasattr(ctx, "allreduce_min") else ok
        if ok_all and accept is not None:
            ok, why = accept(transport, pipeline)
            ok_all = int(ctx.allreduce_min(ok)) if hasattr(ctx, "allreduce_min") else ok
            if not ok_all and not why:
                why = "refused on another rank"
        rec = {"transport": transport, "pipeline": pipeline, "ok": bool(ok_all), "detail": why}
        tried.append(rec)
        if ok_all:
            return GateResult(True, transport, pipeline, why, tried)
        if why:
            log(f"[rank {ctx.rank}] gate: {transport}/{pipeline} failed: {why}")
    return GateResult(False, "", "", "no transport passed the gate", tried)
