"""The heat-equation "model family": physics + program personalities of the reference.

The reference ships four programs that solve the same PDE with different semantics
(SURVEY.md §0, §2.8 B-2).  Each is a *preset* here, selected with ``--preset``:

=============  ==========================================================================
preset         reference program and its semantics
=============  ==========================================================================
``heat2dn``    ``mpi_heat2Dn.c`` — fixed (Dirichlet) edges, ``cx = cy = 0.1f`` promoted to
               double (``mpi_heat2Dn.c:41-44``), 1-D row strips (``:87-104``), transposed
               text dumps (``prtdat``, ``:253-268``), original banners.
``grad_mpi``   ``grad1612_mpi_heat.c`` — every owned cell updated against a zero ghost ring
               (``:238-259``), double ``CX = CY = 0.1`` (``:18-19``), 2-D blocks 2×2
               (``:11-12``), row-major text + raw binaries (``:177-203,282-298``).
``grad_hybrid`` ``grad1612_hybrid_heat.c`` — as grad_mpi on a 1×1 grid with convergence on
               (``:6-24``); the OpenMP team becomes the GPU's intra-device parallelism.
``cuda``       ``grad1612_cuda_heat.cu`` — fixed edges, double ``CX``, 640×1024, 10000 steps
               (``:6-13``), no output files, ``Problem size`` banner.
``heat2d``     the framework default: fixed edges (the readme's "outer elements don't
               change", ``readme.md:4``), double coefficients, exact center-hot init,
               grad-style reporting.
=============  ==========================================================================
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass, field
from typing import Dict

CX_DOUBLE = 0.1
CX_FLOAT = 0.10000000149011612  # (double)0.1f


@dataclass(frozen=True)
class Preset:
    name: str
    nx: int
    ny: int
    steps: int
    gridx: int
    gridy: int
    boundary: str  # "fixed" | "ghost-zero"
    coeff: str  # "double" | "float"
    convergence: bool
    interval: int
    sensitivity: float
    report: str  # banner style: "grad" | "hybrid" | "heat2dn" | "cuda"
    text: str  # text dump style: "grad" | "heat2dn" | "none"
    binary: bool  # write *_binary.dat
    decomposition: str = "blocks"  # "blocks" | "strips"
    notes: str = ""

    def cx(self) -> float:
        return CX_FLOAT if self.coeff == "float" else CX_DOUBLE


def _load_presets() -> Dict[str, Preset]:
    """Parse the shared preset table ``csrc/presets.def`` (also compiled into the C++ CLI)."""
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "presets.def")
    out: Dict[str, Preset] = {}
    with open(path, encoding="utf-8") as f:
        for line in f:
            m = re.match(r"\s*H2D_PRESET\((.*)\)\s*$", line)
            if not m:
                continue
            (name, nx, ny, steps, gx, gy, bnd, coeff, conv, interval, sens, report, text, binary,
             dec) = [t.strip() for t in m.group(1).split(",")]
            out[name] = Preset(name, int(nx), int(ny), int(steps), int(gx), int(gy), bnd.replace("_", "-"), coeff,
                               conv != "0", int(interval), float(sens), report, text, binary != "0",
                               decomposition=dec)
    if not out:
        raise RuntimeError(f"no presets parsed from {path}")
    return out


PRESETS: Dict[str, Preset] = _load_presets()


@dataclass
class HeatModel:
    """Physics of one run: boundary mode, coefficients, precision, initial field."""

    boundary: str = "fixed"
    cx: float = CX_DOUBLE
    cy: float = CX_DOUBLE
    precision: str = "ref"  # "ref" (bit-exact fp64 expression) | "fp32"
    init: str = "exact"  # "exact" | "ref-int32" | "zero"
    periodic_x: bool = False
    periodic_y: bool = False
    extra: dict = field(default_factory=dict)

    BOUNDARIES = ("fixed", "ghost-zero")
    PRECISIONS = ("ref", "fp32")
    INITS = ("exact", "ref-int32", "zero")

    def validate(self) -> None:
        if self.boundary not in self.BOUNDARIES:
            raise ValueError(f"boundary must be one of {self.BOUNDARIES}")
        if self.precision not in self.PRECISIONS:
            raise ValueError(f"precision must be one of {self.PRECISIONS}")
        if self.init not in self.INITS:
            raise ValueError(f"init must be one of {self.INITS}")

    # native enum values
    def boundary_id(self) -> int:
        return 0 if self.boundary == "fixed" else 1

    def precision_id(self) -> int:
        return 0 if self.precision == "ref" else 1

    def init_id(self) -> int:
        return {"exact": 0, "ref-int32": 1, "zero": 2}[self.init]

    def flops_per_cell(self) -> int:
        """Arithmetic per cell update as written in the reference expression (2 adds, 2 subs,
        2 muls by the coefficients, 2 adds, 1 mul by 2): used only for reporting."""
        return 9
