"""Topology helpers: the Cartesian decomposition seen from Python.

Parity with ``MPI_Cart_create(dims={GRIDY,GRIDX}, periods={0,0})`` + ``MPI_Cart_shift``
(``grad1612_mpi_heat.c:74-81``): rank r owns block row ``r % GRIDX`` and block column
``r // GRIDX`` (so ``xs[r] = (r % GRIDX)*xcell``, ``ys[r] = (r / GRIDX)*ycell``,
``:125-138``); neighbours outside a non-periodic grid are -1 (``MPI_PROC_NULL``).  The 1-D
strips of ``mpi_heat2Dn.c:87-104`` are ``gridy = 1`` with the same uneven split.
"""
from __future__ import annotations

from .._native import native

DIRS = ("N", "S", "W", "E", "NW", "NE", "SW", "SE")


def decomposition(nx: int, ny: int, gridx: int, gridy: int, periodic_x: bool = False, periodic_y: bool = False):
    return native().Decomposition(nx, ny, gridx, gridy, periodic_x, periodic_y)


def neighbors(dec, rank: int) -> dict:
    return {name: dec.neighbor(rank, d) for d, name in enumerate(DIRS)}


def tile_bounds(dec, rank: int) -> tuple[int, int, int, int]:
    """(x0, y0, xcell, ycell) of `rank`'s block in global coordinates."""
    px, py = dec.px_of(rank), dec.py_of(rank)
    return dec.xstart[px], dec.ystart[py], dec.xcount[px], dec.ycount[py]


def strips_table(dec) -> list[dict]:
    """Rows/offset/left/right of each 1-D strip, as the original master prints them
    (``mpi_heat2Dn.c:94-116``; workers are numbered from 1 and 0 means "no neighbour")."""
    out = []
    for i in range(dec.gridx):
        out.append({"task": i + 1, "rows": dec.xcount[i], "offset": dec.xstart[i],
                    "left": 0 if i == 0 else i, "right": 0 if i == dec.gridx - 1 else i + 2})
    return out
