"""Process runtime: one process per GPU, bootstrapped with ``torch.distributed``.

Replaces ``MPI_Init / Comm_size / Comm_rank`` (``grad1612_mpi_heat.c:42-44``) and the
timing collectives ``MPI_Barrier`` + ``MPI_Reduce(MAX)`` (``:206,277-280``).

Planes:
  * control plane (bootstrap of the RCCL unique id, barriers, elapsed-time max, convergence
    sums of the external transport): a ``gloo`` process group — host-side, works with or
    without GPUs and is exercised by the CPU test-suite with world_size > 1;
  * data plane on GPUs: the engine's own RCCL communicator (ncclSend/ncclRecv over xGMI,
    ncclAllReduce for the convergence residual), created from a unique id broadcast on the
    control plane.  ``--transport torch`` instead moves halos with ``torch.distributed``
    (``nccl`` backend = RCCL on ROCm) batch_isend_irecv.

Rendezvous always uses the env:// variables set by ``torch.distributed.run``
(``MASTER_ADDR=127.0.0.1`` recommended).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    initialized_here: bool = False
    nccl_group: Optional[object] = None
    distinct_devices: bool = False  # one GPU per rank (set by the caller that maps ranks to devices)
    _shm: Optional[object] = field(default=None, repr=False)
    _shm_state: int = 0  # 0 not set up, 1 usable, -1 unavailable (ranks on several nodes)

    @property
    def is_multi(self) -> bool:
        return self.world > 1

    # ---- collectives on the control plane --------------------------------------------------
    def barrier(self) -> None:
        if self.is_multi:
            dist.barrier()

    def node_barrier(self, timeout_s: float = 60.0) -> None:
        """Tight barrier for bracketing a timed region: a gloo barrier, then a spin on a /dev/shm
        generation counter (native ``ShmBarrier``), so the ranks of one node leave within about
        a microsecond of each other instead of the gloo barrier's tens of microseconds.  The
        max-over-ranks timing (``grad1612_mpi_heat.c:277-280``) otherwise charges that exit
        skew to the run: an early rank waits for a late neighbour's halo inside its timed
        region.  Collective on first use (sets up the segment); falls back to the gloo barrier
        alone when the ranks do not share a node."""
        if not self.is_multi:
            return
        self.barrier()
        if self._shm_state == 0:
            self._shm_state = -1
            self._shm = self._make_node_barrier()
            if self._shm is not None:
                self._shm_state = 1
        if self._shm is not None:
            self._shm.wait(timeout_s)

    def _make_node_barrier(self):
        import secrets

        from heat2d_amd._native import native

        n = native()
        name = self.broadcast_bytes(
            f"/heat2d_bar_{os.getpid()}_{secrets.token_hex(6)}".encode() if self.rank == 0 else None).decode()
        b = None
        if self.rank == 0:
            try:
                b = n.ShmBarrier(name, 0, self.world, True)
            except Exception:  # noqa: BLE001 - no /dev/shm: every rank falls back together
                b = None
        self.barrier()
        if self.rank != 0:
            try:
                b = n.ShmBarrier(name, self.rank, self.world, False)
            except Exception:  # noqa: BLE001 - another node: the name does not exist there
                b = None
        ok = self.allreduce_min(1.0 if b is not None else 0.0) > 0.5
        if b is not None:
            b.unlink()  # every rank holds the mapping (or gave up): drop the name
        return b if ok else None

    def allreduce_max(self, x: float) -> float:
        if not self.is_multi:
            return float(x)
        t = torch.tensor([float(x)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def allreduce_sum(self, x: float) -> float:
        if not self.is_multi:
            return float(x)
        t = torch.tensor([float(x)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    def allreduce_min(self, x: float) -> float:
        if not self.is_multi:
            return float(x)
        t = torch.tensor([float(x)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return float(t.item())

    def device_barrier(self, device: int) -> bool:
        """Align the ranks at the device level: an RCCL all-reduce of one word on each rank's own
        GPU, then a device synchronize.  Ranks leave it within a few microseconds of each other
        (a gloo barrier's exit skew is tens of microseconds).  Only with one GPU per rank (RCCL
        refuses two ranks on one device); returns False when not applicable."""
        if not self.is_multi or not getattr(self, "distinct_devices", False):
            return False
        t = torch.ones(1, device=torch.device("cuda", device))
        dist.all_reduce(t, group=self.get_nccl_group())
        torch.cuda.synchronize(device)
        return True

    def broadcast_bytes(self, data: Optional[bytes], src: int = 0) -> bytes:
        if not self.is_multi:
            assert data is not None
            return data
        obj = [data if self.rank == src else None]
        dist.broadcast_object_list(obj, src=src)
        return obj[0]

    def all_gather_bytes(self, data: bytes) -> list:
        if not self.is_multi:
            return [data]
        out = [None] * self.world
        dist.all_gather_object(out, data)
        return out

    def gather_objects(self, obj, dst: int = 0):
        if not self.is_multi:
            return [obj]
        out = [None] * self.world if self.rank == dst else None
        dist.gather_object(obj, out, dst=dst)
        return out

    def devices_shared(self, device: int, pci_id: str) -> bool:
        """Collective: True if any two ranks run on the same physical GPU (same host and PCI bus
        id).  Ordinals and visibility masks cannot tell: two ranks may name the same device
        explicitly, or see one GPU each under different numbering.  Sets ``distinct_devices``."""
        if not self.is_multi:
            self.distinct_devices = device >= 0
            self.ranks_on_device = 1
            return False
        import socket

        ident = f"{socket.gethostname()}|{pci_id}" if device >= 0 else f"cpu|{self.rank}"
        ids = self.all_gather_bytes(ident.encode())
        shared = device >= 0 and len(set(ids)) < len(ids)
        self.distinct_devices = device >= 0 and not shared
        # ranks on this rank's GPU (itself included)
        self.ranks_on_device = sum(1 for i in ids if i == ident.encode()) if device >= 0 else 1
        return shared

    def get_nccl_group(self):
        """Lazily created RCCL-backed group for the torch p2p transport on GPUs."""
        if self.nccl_group is None:
            self.nccl_group = dist.new_group(backend="nccl")
        return self.nccl_group

    def shutdown(self) -> None:
        if self.initialized_here and dist.is_initialized():
            dist.destroy_process_group()
            self.initialized_here = False


def env_world() -> tuple[int, int, int]:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def init_distributed(timeout_s: float = 600.0) -> DistContext:
    """Initialise the control plane from the environment (no-op for a single process)."""
    rank, world, local = env_world()
    ctx = DistContext(rank=rank, world=world, local_rank=local)
    if world > 1:
        if dist.is_initialized():
            ctx.rank, ctx.world = dist.get_rank(), dist.get_world_size()
        else:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29500")
            dist.init_process_group(backend="gloo", init_method="env://", rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=timeout_s))
            ctx.initialized_here = True
    return ctx
