"""An independent numpy implementation of the reference numerics.

Written separately from the C++ oracle so the two can check each other: fp32 storage,
fp32 neighbour-pair sums, fp64 expression evaluated left to right (numpy never contracts
to FMA), one rounding to fp32.
"""
import numpy as np


def init_field(nx, ny, mode="exact"):
    ix = np.arange(nx, dtype=np.int64)[:, None]
    iy = np.arange(ny, dtype=np.int64)[None, :]
    if mode == "exact":
        a = (ix * (nx - 1 - ix)).astype(np.float64)
        b = (iy * (ny - 1 - iy)).astype(np.float64)
        return (a * b).astype(np.float32)
    if mode == "ref-int32":
        with np.errstate(over="ignore"):
            p = (ix.astype(np.uint32) * (nx - ix - 1).astype(np.uint32)).astype(np.uint32)
            p = (p * iy.astype(np.uint32)).astype(np.uint32)
            p = (p * (ny - iy - 1).astype(np.uint32)).astype(np.uint32)
        return p.view(np.int32).astype(np.float32)
    return np.zeros((nx, ny), np.float32)


def step(u, boundary="fixed", cx=0.1, cy=0.1, precision="ref", periodic=(False, False)):
    nx, ny = u.shape
    px, py = periodic
    pad = np.zeros((nx + 2, ny + 2), np.float32)
    pad[1:-1, 1:-1] = u
    if px:
        pad[0, 1:-1] = u[-1]
        pad[-1, 1:-1] = u[0]
    if py:
        pad[:, 0] = pad[:, -2]
        pad[:, -1] = pad[:, 1]
    c = pad[1:-1, 1:-1]
    n_, s_ = pad[:-2, 1:-1], pad[2:, 1:-1]
    w_, e_ = pad[1:-1, :-2], pad[1:-1, 2:]
    sn = (s_ + n_).astype(np.float32)
    ew = (e_ + w_).astype(np.float32)
    if precision == "ref":
        dc = c.astype(np.float64)
        r = dc + cx * (sn.astype(np.float64) - 2.0 * dc)
        r = r + cy * (ew.astype(np.float64) - 2.0 * dc)
        new = r.astype(np.float32)
    else:
        raise NotImplementedError("numpy oracle covers the ref precision only")
    if boundary == "fixed":
        keep = np.zeros((nx, ny), bool)
        if not px:
            keep[0, :] = keep[-1, :] = True
        if not py:
            keep[:, 0] = keep[:, -1] = True
        new = np.where(keep, u, new)
    return new


def run(nx, ny, steps, boundary="fixed", cx=0.1, cy=0.1, init="exact", periodic=(False, False), u=None):
    u = init_field(nx, ny, init) if u is None else u.copy()
    for _ in range(steps):
        u = step(u, boundary, cx, cy, "ref", periodic)
    return u
