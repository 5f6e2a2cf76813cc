"""heat2d_amd — an MI355X-native 2-D heat-equation (5-point Jacobi) framework.

Same capabilities as patschris/Heat2D (serial, MPI strips/blocks, hybrid, CUDA programs;
see SURVEY.md), re-designed for CDNA4: register-streaming temporally-blocked HIP stencil
kernels, a native engine with halo exchange overlapped on a second HIP stream, RCCL over
xGMI between processes, a bit-exact CPU oracle.
"""
from ._native import native, gpu_available  # imports torch first (shared HIP runtime)
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
