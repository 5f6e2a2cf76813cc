"""Runtime configuration: every compile-time ``#define`` of the reference becomes a flag.

Reference knobs: ``NXPROB NYPROB STEPS GRIDX GRIDY CONVERGENCE
INTERVAL SENSITIVITY CX CY DEBUG`` (``grad1612_mpi_heat.c:5-21``, ``mpi_heat2Dn.c:29-44``,
``grad1612_hybrid_heat.c:6-24``, ``grad1612_cuda_heat.cu:6-13``) map to ``--nx --ny --steps
--gridx --gridy --convergence --interval --sensitivity --cx --cy --debug``; ``BLOCKX/BLOCKY``
(CUDA tuning) become ``--tblock/--rows-per-wave`` (the MI355X kernel's tuning knobs);
``REORGANISATION`` is subsumed by the topology (coordinates always come from the
decomposition, B-8).  ``NUMTHREADS`` has no GPU meaning and is accepted and reported only.
"""
from __future__ import annotations

import argparse
import math
from dataclasses import asdict, dataclass, field
from typing import List, Optional, Sequence

from .models.heat2d import PRESETS, HeatModel


@dataclass
class Config:
    preset: str = "heat2d"
    nx: int = 10
    ny: int = 10
    steps: int = 100
    gridx: int = 1  # 0 = automatic from the world size
    gridy: int = 1
    convergence: bool = False
    interval: int = 20
    sensitivity: float = 0.1
    cx: float = 0.1
    cy: float = 0.1
    boundary: str = "fixed"
    init: str = "exact"
    precision: str = "ref"
    periodic: str = "none"  # none | x | y | xy  (extension: MPI_Cart_create periods)
    debug: bool = False
    numthreads: int = 4  # accepted for the hybrid preset's banner only
    output: str = "auto"  # auto | text | binary | both | none
    outdir: str = "."
    report: str = "grad"
    text_style: str = "grad"
    device: str = "auto"  # auto | gpu | cpu
    transport: str = "auto"  # auto | local | ipc | rccl | torch | host
    tblock: int = 0  # halo depth / deepest chunk; 0: measured default (7 ref, 8 fp32)
    rows_per_wave: int = 0
    overlap: bool = True
    pipeline: str = "auto"  # auto | direct-sys | signal | serial (multi-rank halo pipeline)
    sync_mode: int = 0  # end-of-run synchronisation (EngineOptions::sync_mode; the bench uses 2)
    persistent: str = "auto"  # auto | on | off: persistent stencil launches (auto: off when ranks share a GPU)
    halo_timeout_s: float = 30.0  # bounded device-side halo waits give up (and the run fails) after this
    small_grid: bool = True
    tiled: str = "auto"  # auto | on | off: LDS-tiled temporally-blocked kernel (single-tile small/medium grids)
    naive: bool = False
    tune: bool = False  # autotune K / rows-per-wave on scratch engines before the run (single GPU)
    json: bool = False
    quiet: bool = False
    load: Optional[str] = None  # resume: raw NX×NY fp32 grid (extension)
    start_step: int = 0
    save: Optional[str] = None  # checkpoint: raw grid after the run (extension)
    decomposition: str = "blocks"

    def model(self) -> HeatModel:
        m = HeatModel(boundary=self.boundary, cx=self.cx, cy=self.cy, precision=self.precision, init=self.init,
                      periodic_x="x" in self.periodic, periodic_y="y" in self.periodic)
        m.validate()
        return m

    def to_dict(self) -> dict:
        return asdict(self)

    def resolve_grid(self, world: int) -> tuple[int, int]:
        """Pick GRIDX×GRIDY for `world` ranks (0 = automatic)."""
        gx, gy = self.gridx, self.gridy
        if gx > 0 and gy > 0:
            return gx, gy
        if self.decomposition == "strips":
            return (world if gx <= 0 else gx), 1
        if gx > 0:
            if world % gx:
                raise ValueError(f"world size {world} not divisible by gridx={gx}")
            return gx, world // gx
        if gy > 0:
            if world % gy:
                raise ValueError(f"world size {world} not divisible by gridy={gy}")
            return world // gy, gy
        return auto_grid(world)


def auto_grid(world: int) -> tuple[int, int]:
    """Near-square factorisation with GRIDX <= GRIDY (8 ranks -> 2×4, the BASELINE layout)."""
    best = (1, world)
    for gx in range(1, int(math.isqrt(world)) + 1):
        if world % gx == 0:
            best = (gx, world // gx)
    return best


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="heat2d", description="MI355X-native 2-D heat equation (5-point Jacobi) solver")
    p.add_argument("--preset", choices=sorted(PRESETS), default="heat2d",
                   help="reference-program personality (defaults, banners, output format)")
    p.add_argument("--nx", type=int, help="NXPROB: rows of the grid")
    p.add_argument("--ny", type=int, help="NYPROB: columns of the grid")
    p.add_argument("--steps", type=int, help="STEPS: time steps")
    p.add_argument("--gridx", type=int, help="GRIDX: blocks along x (rows); 0 = automatic")
    p.add_argument("--gridy", type=int, help="GRIDY: blocks along y (columns); 0 = automatic")
    p.add_argument("--convergence", type=int, choices=(0, 1), help="CONVERGENCE: 1 = check every INTERVAL steps")
    p.add_argument("--interval", type=int, help="INTERVAL: steps between convergence checks")
    p.add_argument("--sensitivity", type=float, help="SENSITIVITY: stop when sum((u'-u)^2) < this")
    p.add_argument("--cx", type=float, help="CX coefficient")
    p.add_argument("--cy", type=float, help="CY coefficient")
    p.add_argument("--debug", type=int, choices=(0, 1), default=0, help="DEBUG: neighbour/device report")
    p.add_argument("--numthreads", type=int, default=4, help="NUMTHREADS (hybrid banner only)")
    p.add_argument("--boundary", choices=HeatModel.BOUNDARIES, help="fixed edges or zero ghost ring")
    p.add_argument("--init", choices=HeatModel.INITS, default=None,
                   help="exact fp64 center-hot field, the reference's int32-wrapped one, or zeros")
    p.add_argument("--precision", choices=HeatModel.PRECISIONS, default="ref",
                   help="ref = bit-exact fp64 expression; fp32 = FMA fast path")
    p.add_argument("--periodic", choices=("none", "x", "y", "xy"), default="none",
                   help="periodic dimensions (extension)")
    p.add_argument("--output", choices=("auto", "text", "binary", "both", "none"), default="auto",
                   help="initial/final dumps: text (.dat), raw binary (*_binary.dat), both or none")
    p.add_argument("--outdir", default=".", help="directory for output files")
    p.add_argument("--device", choices=("auto", "gpu", "cpu"), default="auto")
    p.add_argument("--transport", choices=("auto", "local", "ipc", "rccl", "torch", "host"), default="auto",
                   help="halo transport: in-process tiles, direct IPC peer stores (1-D row strips), native RCCL, "
                        "torch.distributed p2p (nccl backend on GPUs), or host (gloo p2p with host staging; also "
                        "allows several ranks per GPU)")
    p.add_argument("--tblock", type=int, default=0,
                   help="time steps fused per kernel (halo depth); 0: 7 for ref, 8 for fp32 (measured at 4096^2)")
    p.add_argument("--rows-per-wave", type=int, default=0, help="rows per wave work unit (0 = auto)")
    p.add_argument("--no-overlap", action="store_true", help="do not overlap halo exchange with interior compute")
    p.add_argument("--pipeline", choices=("auto", "direct-sys", "signal", "serial"), default="auto",
                   help="multi-rank halo pipeline (auto: the transport's default; direct-sys: the direct IPC "
                        "pipeline with system-scope fences; signal / serial: RCCL pipelines)")
    p.add_argument("--no-small-grid", action="store_true", help="disable the whole-grid LDS solver")
    p.add_argument("--tiled", choices=("auto", "on", "off"), default="auto",
                   help="LDS-tiled temporally-blocked kernel for single-tile small/medium grids")
    p.add_argument("--naive", action="store_true", help="validation kernel: one thread per cell, one step per launch")
    p.add_argument("--tune", action="store_true", help="autotune the temporal block / unit size before the run")
    p.add_argument("--json", action="store_true", help="print a JSON metrics line")
    p.add_argument("--quiet", action="store_true", help="no banners")
    p.add_argument("--load", default=None, help="resume from a raw NX×NY fp32 grid (extension)")
    p.add_argument("--start-step", type=int, default=0, help="step count of the --load grid")
    p.add_argument("--save", default=None, help="write the final raw grid here (checkpoint, extension)")
    return p


def config_from_args(argv: Optional[Sequence[str]] = None) -> Config:
    a = build_parser().parse_args(argv)
    pre = PRESETS[a.preset]

    def pick(v, d):
        return d if v is None else v

    c = Config(
        preset=a.preset,
        nx=pick(a.nx, pre.nx),
        ny=pick(a.ny, pre.ny),
        steps=pick(a.steps, pre.steps),
        gridx=pick(a.gridx, pre.gridx),
        gridy=pick(a.gridy, pre.gridy),
        convergence=bool(pick(a.convergence, int(pre.convergence))),
        interval=pick(a.interval, pre.interval),
        sensitivity=pick(a.sensitivity, pre.sensitivity),
        cx=pick(a.cx, pre.cx()),
        cy=pick(a.cy, pre.cx()),
        boundary=pick(a.boundary, pre.boundary),
        init=pick(a.init, "exact"),
        precision=a.precision,
        periodic=a.periodic,
        debug=bool(a.debug),
        numthreads=a.numthreads,
        output=a.output,
        outdir=a.outdir,
        report=pre.report,
        text_style=pre.text,
        device=a.device,
        transport=a.transport,
        tblock=a.tblock,
        rows_per_wave=a.rows_per_wave,
        overlap=not a.no_overlap,
        pipeline=a.pipeline,
        small_grid=not a.no_small_grid,
        tiled=a.tiled,
        naive=a.naive,
        tune=a.tune,
        json=a.json,
        quiet=a.quiet,
        load=a.load,
        start_step=a.start_step,
        save=a.save,
        decomposition=pre.decomposition,
    )
    if c.output == "auto":
        c.output = {(True, True): "both", (True, False): "text", (False, True): "binary", (False, False): "none"}[
            (pre.text != "none", pre.binary)]
    if c.text_style == "none":
        c.text_style = "grad"
    if c.nx < 1 or c.ny < 1 or c.steps < 0:
        raise SystemExit("ERROR: nx, ny must be >= 1 and steps >= 0")
    return c


def presets() -> List[str]:
    return sorted(PRESETS)


__all__ = ["Config", "config_from_args", "build_parser", "auto_grid", "presets", "field"]
