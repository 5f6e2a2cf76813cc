"""Loader of the native runtime ``_heat2d`` (HIP kernels, engine, CPU oracle, RCCL).

``torch`` is imported first on purpose: torch's ROCm wheel ships its own ``libamdhip64`` /
``librccl`` and references them by unversioned names, while our extension links the sonames
``libamdhip64.so.7`` / ``librccl.so.1``.  Loading torch first makes both resolve to ONE HIP
runtime and ONE RCCL in the process (same device pointers, same streams).

If the extension is missing it is built in-tree (``heat2d_amd._build``) unless
``HEAT2D_NO_BUILD=1``.  On a GPU machine a missing/broken extension is an error — there is
no silent Python fallback for any device op.
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: E402,F401  (must precede the native module, see above)

_mod = None


def native():
    """Return the loaded ``_heat2d`` module.  The extension carries the hash of the native
    sources it was built from; if it is missing or stale (sources edited since), it is rebuilt
    in-tree first — or, with ``HEAT2D_NO_BUILD=1`` (GPU boxes, the driver), the import FAILS
    rather than run a binary that does not match the sources."""
    global _mod
    if _mod is not None:
        return _mod
    from . import _build

    want = _build.source_hash() if os.path.isdir(_build.CSRC) else None
    have = _build.stamped_hash(_build.EXT_PATH)
    if want is not None and have != want:
        if os.environ.get("HEAT2D_NO_BUILD") == "1":
            raise ImportError(f"heat2d_amd native extension is stale or missing (built from {have}, sources are "
                              f"{want}): run `python -m heat2d_amd._build`")
        _build.build(cli=False)
    _mod = importlib.import_module("heat2d_amd._heat2d")
    return _mod


def native_path() -> str:
    return native().__file__


def gpu_available() -> bool:
    """True when a HIP device is usable (without initialising torch's CUDA state)."""
    if os.environ.get("HEAT2D_FORCE_CPU") == "1":
        return False
    try:
        return native().device_count() > 0
    except Exception:
        return False
