"""heat2d_amd — an MI355X-native 2-D heat-equation (5-point Jacobi) framework.

Same capabilities as patschris/Heat2D (serial, MPI strips/blocks, hybrid, CUDA programs;
see SURVEY.md), re-designed for CDNA4: register-streaming temporally-blocked HIP stencil
kernels, a native engine with halo exchange overlapped on a second HIP stream, RCCL over
xGMI between processes, a bit-exact CPU oracle.
"""
import os as _os
import sys as _sys

# Kernel arguments from host memory, not from the HIP runtime's device-memory kernarg pool: in a
# process that creates many engines, launches read stale or torn arguments from that pool (the
# integrity check's torn-argument bit fired; wrong tiles and an illegal access, gone with this
# setting on the same box — docs/ARCHITECTURE.md, "Stale kernel arguments").  The HIP runtime
# reads it when it initialises, so it is set before any GPU call; set it to 1 to opt out.
if "HIP_FORCE_DEV_KERNARG" not in _os.environ:
    _torch = _sys.modules.get("torch")
    if _torch is not None and _torch.cuda.is_initialized():
        import warnings as _w

        _w.warn("heat2d_amd imported after the GPU was initialised: HIP_FORCE_DEV_KERNARG=0 cannot take effect "
                "(kernel arguments stay in device memory); import heat2d_amd first or export it", RuntimeWarning)
    _os.environ["HIP_FORCE_DEV_KERNARG"] = "0"

from ._native import native, gpu_available  # noqa: E402  (imports torch first: shared HIP runtime)
from .config import Config, config_from_args, auto_grid
from .models.heat2d import PRESETS, HeatModel, Preset

__all__ = ["native", "gpu_available", "Config", "config_from_args", "auto_grid", "PRESETS", "HeatModel", "Preset",
           "Solver"]
__version__ = "0.1.0"


def __getattr__(name):
    if name == "Solver":
        from .solver import Solver

        return Solver
    raise AttributeError(name)
