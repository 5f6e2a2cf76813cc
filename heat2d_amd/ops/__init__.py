"""heat2d_amd.ops — torch-tensor entry points to the HIP kernels (``stencil``) and the
plain-PyTorch reference of the same op (``reference``)."""
from . import reference
from .stencil import (alloc_tile, fill_periodic_ghosts, heat_steps, init_tile, naive_step, num_units, owned,
                      stencil, tile_geom)

__all__ = ["reference", "alloc_tile", "fill_periodic_ghosts", "heat_steps", "init_tile", "naive_step", "num_units",
           "owned", "stencil", "tile_geom"]
