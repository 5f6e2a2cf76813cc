"""Plain-PyTorch reference of the 5-point update (device-agnostic, no custom kernels).

Written op by op so that no floating-point contraction can happen: with ``precision="ref"``
it reproduces the reference's C expression bit for bit (fp32 neighbour sums, fp64
arithmetic, one rounding to fp32 — SURVEY.md §2.9); with ``precision="fp32"`` it is the
textbook fp32 stencil (no FMA), used as the tolerance oracle of the fp32 fast path.
"""
from __future__ import annotations

from typing import Tuple

import torch


def _neighbours(u: torch.Tensor, periodic: Tuple[bool, bool]):
    nx, ny = u.shape
    pad = torch.zeros((nx + 2, ny + 2), dtype=u.dtype, device=u.device)
    pad[1:-1, 1:-1] = u
    if periodic[0]:
        pad[0, 1:-1] = u[-1]
        pad[-1, 1:-1] = u[0]
    if periodic[1]:
        pad[:, 0] = pad[:, -2]
        pad[:, -1] = pad[:, 1]
    return pad[:-2, 1:-1], pad[2:, 1:-1], pad[1:-1, :-2], pad[1:-1, 2:]


def step(u: torch.Tensor, *, boundary: str = "fixed", cx: float = 0.1, cy: float = 0.1, precision: str = "ref",
         periodic: Tuple[bool, bool] = (False, False)) -> torch.Tensor:
    if u.dtype != torch.float32:
        raise ValueError("the grid is fp32")
    n_, s_, w_, e_ = _neighbours(u, periodic)
    sn = s_ + n_  # fp32
    ew = e_ + w_
    if precision == "ref":
        dc = u.double()
        r = dc + cx * (sn.double() - 2.0 * dc)
        r = r + cy * (ew.double() - 2.0 * dc)
        new = r.float()
    else:
        two_c = u + u
        new = u + cx * (sn - two_c)
        new = new + cy * (ew - two_c)
    if boundary == "fixed":
        keep = torch.zeros_like(u, dtype=torch.bool)
        if not periodic[0]:
            keep[0, :] = True
            keep[-1, :] = True
        if not periodic[1]:
            keep[:, 0] = True
            keep[:, -1] = True
        new = torch.where(keep, u, new)
    return new


def run(u: torch.Tensor, steps: int, **kw) -> torch.Tensor:
    for _ in range(steps):
        u = step(u, **kw)
    return u


def center_hot(nx: int, ny: int, device="cpu") -> torch.Tensor:
    ix = torch.arange(nx, dtype=torch.int64, device=device)[:, None]
    iy = torch.arange(ny, dtype=torch.int64, device=device)[None, :]
    return ((ix * (nx - 1 - ix)).double() * (iy * (ny - 1 - iy)).double()).float()
