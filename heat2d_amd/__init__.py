"""heat2d_amd — an MI355X-native 2-D heat-equation (5-point Jacobi) framework.

Same capabilities as patschris/Heat2D (serial, MPI strips/blocks, hybrid, CUDA programs;
see SURVEY.md), re-designed for CDNA4: register-streaming temporally-blocked HIP stencil
kernels, a native engine with halo exchange overlapped on a second HIP stream, RCCL over
xGMI between processes, a bit-exact CPU oracle.
"""
import os as _os
import sys as _sys

# Kernel arguments from host memory, not from the HIP runtime's device-memory kernel-argument pool.
# Under device-memory arguments the engine GPU tests fail in every configuration tried (round 4:
# 5-6 of 612; round 5, with device-resident argument blocks: 4-29), and pass with host-memory
# arguments (docs/ARCHITECTURE.md, "Kernel arguments (round 5)").  The stencil kernels take their
# argument-block pointer and per-launch scalars as scalar arguments that each wave reads once, so
# host-memory arguments cost nothing measurable (4096^2, K=7: 57.2 us per launch against 57.8-58.1
# with device-memory arguments).  The runtime reads the variable once, at initialisation: set before
# any GPU call; a user's own setting is kept (with a warning if it selects device memory).
KERNARG_HOST_MEMORY = _os.environ.get("HIP_FORCE_DEV_KERNARG") == "0"  # the effective state, once known
if "HIP_FORCE_DEV_KERNARG" not in _os.environ:
    _torch = _sys.modules.get("torch")
    if _torch is not None and _torch.cuda.is_initialized():
        import warnings as _w

        # too late: the runtime already chose device-memory arguments; say so, change nothing
        _w.warn("heat2d_amd imported after the GPU was initialised: kernel arguments stay in device memory "
                "(import heat2d_amd first, or export HIP_FORCE_DEV_KERNARG=0)", RuntimeWarning)
    else:
        _os.environ["HIP_FORCE_DEV_KERNARG"] = "0"
        KERNARG_HOST_MEMORY = True
elif _os.environ["HIP_FORCE_DEV_KERNARG"] != "0":
    import warnings as _w

    _w.warn("HIP_FORCE_DEV_KERNARG selects device-memory kernel arguments, which the engine GPU tests do not "
            "pass with in processes that create and destroy many engines (docs/ARCHITECTURE.md, "
            "\"Known issues\")", RuntimeWarning)

from ._native import native, gpu_available  # noqa: E402  (imports torch first: shared HIP runtime)
from .config import Config, config_from_args, auto_grid  # noqa: E402
from .models.heat2d import PRESETS, HeatModel, Preset  # noqa: E402

__all__ = ["native", "gpu_available", "Config", "config_from_args", "auto_grid", "PRESETS", "HeatModel", "Preset",
           "Solver", "KERNARG_HOST_MEMORY"]
__version__ = "0.1.0"


def __getattr__(name):
    if name == "Solver":
        from .solver import Solver

        return Solver
    raise AttributeError(name)
