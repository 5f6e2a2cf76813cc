"""Command-line entry point: ``python -m heat2d_amd [flags]``.

Single process: ``python -m heat2d_amd --preset grad_mpi`` (all GRIDX×GRIDY tiles on one GPU).
Multi-GPU:      ``python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m heat2d_amd ...``
"""
from __future__ import annotations

import sys
from typing import Optional, Sequence


def main(argv: Optional[Sequence[str]] = None) -> int:
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
