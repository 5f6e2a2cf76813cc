"""Command-line entry point: ``python -m heat2d_amd [flags]``.

Single process: ``python -m heat2d_amd --preset grad_mpi`` (all GRIDX×GRIDY tiles on one GPU).
Multi-GPU:      ``python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m heat2d_amd ...``
"""
from __future__ import annotations

import sys
from typing import Optional, Sequence


def main(argv: Optional[Sequence[str]] = None) -> int:
    # Entry-point policy (not set by the library for embedders): one hardware queue per engine
    # stream.  The engine runs compute and comm streams concurrently and HIP maps streams onto
    # at most GPU_MAX_HW_QUEUES in-order hardware queues; with 4, other libraries' streams can
    # shift the round-robin map until compute and comm share one queue, which serialises the
    # exchange behind the stencil (measured 9.5 -> 15 us/step in round 1).
    # Read once at HIP initialisation, i.e. before the first HIP call of the process.
    import os

    if os.environ.get("HEAT2D_KEEP_HW_QUEUES") != "1" and int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
        os.environ["GPU_MAX_HW_QUEUES"] = "8"
    from .config import config_from_args
    from .solver import Solver

    cfg = config_from_args(argv)
    s = Solver(cfg)
    try:
        s.main()
    finally:
        s.ctx.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
