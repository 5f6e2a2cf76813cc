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

# Hardware queues per process: the engine runs the compute stream and the comm stream (halo
# exchange gate, RCCL, completion counter) concurrently, and HIP maps streams onto at most
# GPU_MAX_HW_QUEUES in-order hardware queues.  With 4, streams created by other engines /
# libraries shift the round-robin map until the two share one queue, which serialises the
# exchange behind the stencil (measured: 9.5 -> 15 us/step on the multi-rank proxy,
# tools/gpu_probe_queues.sh).  8 gives every stream its own queue.  Read once at HIP init,
# so it is set here, before torch (or anything) touches the GPU.
if os.environ.get("HEAT2D_KEEP_HW_QUEUES") != "1" and int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import torch  # noqa: E402,F401  (must precede the native module, see above)

_mod = None


def native():
    """Return the loaded ``_heat2d`` module (building it first if needed)."""
    global _mod
    if _mod is not None:
        return _mod
    try:
        _mod = importlib.import_module("heat2d_amd._heat2d")
    except ImportError:
        if os.environ.get("HEAT2D_NO_BUILD") == "1":
            raise
        from . import _build

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
