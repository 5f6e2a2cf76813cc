"""Torch-tensor front end of the HIP stencil kernels.

A tile is a torch float32 tensor of shape ``(srows, pitch)`` laid out like the engine's
storage (``TileGeom``): owned cells at ``[G:G+nx, PL:PL+ny]``, a ghost ring of depth G
around them, zero elsewhere.  The ops launch the hand-written HIP kernels on the current
torch stream and fail loudly when the native extension or the GPU is missing (no silent
PyTorch fallback; ``heat2d_amd.ops.reference`` is the separate PyTorch reference).

    geom, u = alloc_tile(nx, ny, G=8, device="cuda")
    init_tile(u, geom)                         # center-hot field (exact fp64 formula)
    v = torch.zeros_like(u)
    stencil(u, v, geom, K=8)                   # 8 fused Jacobi steps: u -> v
    field = owned(v, geom)                     # (nx, ny) view
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .._native import native

BOUNDARIES = {"fixed": 0, "ghost-zero": 1}
PRECISIONS = {"ref": 0, "fp32": 1}
INITS = {"exact": 0, "ref-int32": 1, "zero": 2}


def tile_geom(nx: int, ny: int, G: int = 8) -> dict:
    """Storage geometry of an nx×ny single tile with ghost depth G."""
    return native().tile_geom(nx, ny, G)


def alloc_tile(nx: int, ny: int, G: int = 8, device="cuda") -> Tuple[dict, torch.Tensor]:
    g = tile_geom(nx, ny, G)
    return g, torch.zeros((g["srows"], g["pitch"]), dtype=torch.float32, device=device)


def owned(t: torch.Tensor, g: dict) -> torch.Tensor:
    return t[g["G"]:g["G"] + g["xcell"], g["PL"]:g["PL"] + g["ycell"]]


def _check(t: torch.Tensor, g: dict) -> None:
    if t.dtype != torch.float32 or not t.is_contiguous() or tuple(t.shape) != (g["srows"], g["pitch"]):
        raise ValueError(f"tile tensor must be contiguous float32 of shape ({g['srows']}, {g['pitch']})")
    if t.device.type != "cuda":
        raise ValueError("HIP stencil ops need a GPU tensor (see heat2d_amd.ops.reference for the PyTorch path)")


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def init_tile(t: torch.Tensor, g: dict, init: str = "exact") -> torch.Tensor:
    _check(t, g)
    native().op_init(t.data_ptr(), g, INITS[init], _stream())
    return t


def stencil(src: torch.Tensor, dst: torch.Tensor, g: dict, K: int = 1, *, precision: str = "ref",
            boundary: str = "fixed", cx: float = 0.1, cy: float = 0.1, periodic: Tuple[bool, bool] = (False, False),
            rows_per_wave: int = 0, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """K fused time steps src -> dst with the streaming kernel (owned cells of dst written).

    Asynchronous on the current torch stream: the work-unit plan (``rows_per_wave`` 0 = sized
    to the resident-wave capacity) is built once per geometry and cached on the device.
    Periodic dimensions need their ghost ring filled by the caller (``fill_periodic_ghosts``).
    ``residual``: optional float64 tensor of at least ``num_units(...)`` elements receiving
    per-wave partial sums of (u_K - u_{K-1})^2."""
    _check(src, g)
    _check(dst, g)
    if K > g["G"]:
        raise ValueError(f"K={K} exceeds the tile's ghost depth {g['G']}")
    part = 0
    if residual is not None:
        if residual.dtype != torch.float64 or residual.device != src.device:
            raise ValueError("residual must be a float64 tensor on the same device")
        need = num_units(g, K, precision=precision, boundary=boundary, periodic=periodic, rows_per_wave=rows_per_wave)
        if residual.numel() < need or not residual.is_contiguous():
            raise ValueError(f"residual needs at least {need} contiguous elements")
        part = residual.data_ptr()
    native().op_stream(src.data_ptr(), dst.data_ptr(), g, K, PRECISIONS[precision], BOUNDARIES[boundary], cx, cy,
                       periodic[0], periodic[1], rows_per_wave, part, _stream())
    return dst


def num_units(g: dict, K: int, *, precision: str = "ref", boundary: str = "fixed",
              periodic: Tuple[bool, bool] = (False, False), rows_per_wave: int = 0) -> int:
    """Waves (work units) of one ``stencil`` launch = residual partials it writes."""
    return native().op_num_units(g, K, PRECISIONS[precision], BOUNDARIES[boundary], periodic[0], periodic[1],
                                 rows_per_wave)


def naive_step(src: torch.Tensor, dst: torch.Tensor, g: dict, *, precision: str = "ref", boundary: str = "fixed",
               cx: float = 0.1, cy: float = 0.1, periodic: Tuple[bool, bool] = (False, False)) -> torch.Tensor:
    """One step with the one-thread-per-cell validation kernel."""
    _check(src, g)
    _check(dst, g)
    native().op_naive(src.data_ptr(), dst.data_ptr(), g, PRECISIONS[precision], BOUNDARIES[boundary], cx, cy,
                      periodic[0], periodic[1], _stream())
    return dst


def fill_periodic_ghosts(t: torch.Tensor, g: dict, K: int, periodic: Tuple[bool, bool]) -> None:
    """Wrap-around ghost fill of depth K for a single periodic tile (torch copies)."""
    G, PL, nx, ny = g["G"], g["PL"], g["xcell"], g["ycell"]
    if periodic[0]:
        t[G - K:G, PL:PL + ny] = t[G + nx - K:G + nx, PL:PL + ny]
        t[G + nx:G + nx + K, PL:PL + ny] = t[G:G + K, PL:PL + ny]
    if periodic[1]:
        r0, r1 = (G - K, G + nx + K) if periodic[0] else (G, G + nx)
        t[r0:r1, PL - K:PL] = t[r0:r1, PL + ny - K:PL + ny]
        t[r0:r1, PL + ny:PL + ny + K] = t[r0:r1, PL:PL + K]


def heat_steps(u: torch.Tensor, steps: int, *, K: int = 8, precision: str = "ref", boundary: str = "fixed",
               cx: float = 0.1, cy: float = 0.1, periodic: Tuple[bool, bool] = (False, False)) -> torch.Tensor:
    """Functional API: advance an (nx, ny) float32 field `steps` steps; returns a new tensor.

    GPU tensors run the HIP streaming kernel (temporal blocks of K steps); CPU tensors run
    the native bit-exact CPU oracle."""
    if u.dim() != 2:
        raise ValueError("u must be 2-D")
    nx, ny = u.shape
    if u.device.type != "cuda":
        n = native()
        r = n.oracle_run(nx, ny, steps, boundary=BOUNDARIES[boundary], precision=PRECISIONS[precision], cx=cx, cy=cy,
                         periodic_x=periodic[0], periodic_y=periodic[1],
                         initial=u.detach().to(torch.float32).contiguous().numpy())
        return torch.from_numpy(r["grid"])
    if periodic[0] or periodic[1]:
        K = max(1, min(K, nx if periodic[0] else K, ny if periodic[1] else K))
    K = max(1, K)
    while K > 1 and not native().stream_k_supported(K):
        K -= 1
    g, a = alloc_tile(nx, ny, K, u.device)
    b = torch.zeros_like(a)
    owned(a, g).copy_(u)
    done = 0
    while done < steps:
        k = min(K, steps - done)
        while k > 1 and not native().stream_k_supported(k):
            k -= 1
        fill_periodic_ghosts(a, g, k, periodic)
        stencil(a, b, g, k, precision=precision, boundary=boundary, cx=cx, cy=cy, periodic=periodic)
        a, b = b, a
        done += k
    return owned(a, g).clone()
