"""Halo transports driven from Python (the engine's "external" transport).

``TorchHaloExchanger`` moves the K-deep, 8-neighbour halo of one tile with
``torch.distributed`` point-to-point operations, using exactly the engine's exchange plan
(``decomposition.cpp: make_plan``): the engine packs its owned edges into a contiguous send
buffer, segments go to the peers, received segments are unpacked into the ghost ring.  It is
the CPU/gloo path of the multi-process test-suite and the ``--transport torch`` path on GPUs
(``nccl`` backend = RCCL).  The reference equivalent is the persistent Send/Recv set of
``grad1612_mpi_heat.c:209-235,244,274`` with its ``row``/``column`` datatypes (``:139-144``):
the pack/unpack replaces the strided ``MPI_Type_vector``.

Matching rule: a segment sent in direction d carries tag d; the receiver of ghost side
g = opp(d) posts its receive from peer[g] with that same tag, and both sides post in
direction order, so per-peer ordering is unambiguous even when one peer sits on several
sides (periodic or 2-wide grids).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .._native import native

N_DIRS = 8


class TorchHaloExchanger:
    def __init__(self, engine, tile: int = 0, device: Optional[torch.device] = None, group=None,
                 host_staging: bool = False):
        self.engine = engine
        self.tile = tile
        self.device = device or torch.device("cpu")
        self.group = group
        # host staging: a GPU engine packs into device buffers, the segments travel through
        # pinned host copies over the (gloo) group.  Fallback transport, and the way to run
        # several ranks on one GPU (RCCL refuses duplicate devices in a communicator).
        self.host_staging = host_staging and self.device.type != "cpu"
        self._bufs: dict[int, tuple[torch.Tensor, ...]] = {}
        self.opp = list(native().DIR_OPP)

    def _buffers(self, k: int):
        if k not in self._bufs:
            ns = max(1, self.engine.send_count(self.tile, k))
            nr = max(1, self.engine.recv_count(self.tile, k))
            bufs = (torch.zeros(ns, dtype=torch.float32, device=self.device),
                    torch.zeros(nr, dtype=torch.float32, device=self.device))
            if self.host_staging:
                bufs += (torch.zeros(ns, dtype=torch.float32).pin_memory(),
                         torch.zeros(nr, dtype=torch.float32).pin_memory())
            self._bufs[k] = bufs
        return self._bufs[k]

    def exchange(self, k: int) -> int:
        """Fill the tile's ghost ring to depth k.  Returns the number of messages posted."""
        info = self.engine.plan_info(self.tile, k)
        ent = [info[5 * d:5 * d + 5] for d in range(N_DIRS)]  # peer, send_off, send_n, recv_off, recv_n
        bufs = self._buffers(k)
        dsend, drecv = bufs[0], bufs[1]
        send, recv = (bufs[2], bufs[3]) if self.host_staging else (dsend, drecv)
        if self.device.type != "cpu":
            torch.cuda.synchronize(self.device)
        self.engine.pack(self.tile, k, dsend.data_ptr())
        if self.host_staging:
            torch.cuda.synchronize(self.device)
            send.copy_(dsend)
        me = dist.get_rank()
        ops = []
        for d in range(N_DIRS):
            peer, so, sn, _, _ = ent[d]
            if peer >= 0 and peer != me and sn > 0:
                ops.append(dist.P2POp(dist.isend, send[so:so + sn], peer, group=self.group, tag=d))
        for d in range(N_DIRS):
            g = self.opp[d]
            peer, _, _, ro, rn = ent[g]
            if peer == me and rn > 0:
                # periodic dimension one tile wide: this rank is its own neighbour; the ghost
                # side g receives this rank's own direction-d segment
                so, sn = ent[d][1], ent[d][2]
                assert sn == rn, (d, sn, rn)
                recv[ro:ro + rn].copy_(send[so:so + sn])
            elif peer >= 0 and rn > 0:
                ops.append(dist.P2POp(dist.irecv, recv[ro:ro + rn], peer, group=self.group, tag=d))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        if self.host_staging:
            drecv.copy_(recv)
        if self.device.type != "cpu":
            torch.cuda.synchronize(self.device)
        self.engine.unpack(self.tile, k, drecv.data_ptr())
        return len(ops)
