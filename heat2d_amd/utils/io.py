"""Grid output: raw binaries and the two text formats, written without MPI-IO.

* ``*_binary.dat`` — native fp32, C-order NX×NY, no header; every rank ``pwrite``s its own
  tile rows at their global offsets after rank 0 created and truncated the file (fixes B-3
  and B-9 of the reference's MPI-IO, ``grad1612_mpi_heat.c:177-190,282-285``).
* ``initial.dat`` / ``final.dat`` — converted by rank 0 from the binary, in the preset's
  style: ``grad`` (row-major, ``"%6.1f "``, ``grad1612_mpi_heat.c:191-203``) or ``heat2dn``
  (transposed, ``mpi_heat2Dn.c:253-268``).  The reference rereads the binary for the same
  reason (Report.pdf p.19).
"""
from __future__ import annotations

import os
from typing import Callable, Iterable, Tuple

import numpy as np

from .._native import native

TileIter = Iterable[Tuple[int, int, np.ndarray]]  # (gx0, gy0, owned block)


def _paths(outdir: str, which: str) -> tuple[str, str]:
    return os.path.join(outdir, f"{which}_binary.dat"), os.path.join(outdir, f"{which}.dat")


def write_grid(outdir: str, which: str, nx: int, ny: int, tiles: Callable[[], TileIter], *, rank: int,
               barrier: Callable[[], None], binary: bool, text: bool, text_style: str) -> None:
    """Collective: every rank calls it with its own tiles."""
    if not (binary or text):
        return
    n = native()
    bin_path, txt_path = _paths(outdir, which)
    tmp_bin = bin_path if binary else os.path.join(outdir, f".{which}_binary.tmp")
    if rank == 0:
        os.makedirs(outdir, exist_ok=True)
        n.binary_create(tmp_bin, nx, ny)
    barrier()
    for gx0, gy0, block in tiles():
        n.binary_write_tile(tmp_bin, nx, ny, gx0, gy0, np.ascontiguousarray(block, dtype=np.float32))
    barrier()
    if rank == 0 and text:
        style = n.TEXT_HEAT2DN if text_style == "heat2dn" else n.TEXT_GRAD
        n.binary_to_text(tmp_bin, txt_path, nx, ny, style)
        if not binary:
            os.remove(tmp_bin)
    barrier()


def read_binary(path: str, nx: int, ny: int) -> np.ndarray:
    return native().binary_read(path, nx, ny)


def format_text(grid: np.ndarray, style: str = "grad") -> str:
    n = native()
    return n.format_text(np.ascontiguousarray(grid, dtype=np.float32),
                         n.TEXT_HEAT2DN if style == "heat2dn" else n.TEXT_GRAD).decode()
