"""Solver: the top-level driver (one per process).

Equivalent of the reference programs' ``main()`` (``grad1612_mpi_heat.c:27-315``,
``mpi_heat2Dn.c:46-222``, ``grad1612_hybrid_heat.c:30-352``, ``grad1612_cuda_heat.cu:64-93``):
configuration, decomposition, allocation + initial field, initial output, the timed step
loop, timing reduction, final output.

Execution modes
  * one process, GPU   : every tile of the GRIDX×GRIDY decomposition lives on the one device
                         (LocalMultiTile: halos are device-to-device copies) — 1×1 is the
                         plain single-GPU run of ``grad1612_cuda_heat.cu``;
  * one process, CPU   : the same engine on host memory (test oracle path);
  * N processes, GPU   : one tile per rank, native RCCL halo exchange over xGMI (default) or
                         ``--transport torch`` (torch.distributed p2p);
  * N processes, CPU   : one tile per rank, torch.distributed (gloo) p2p — the CI path.
"""
from __future__ import annotations

import socket
import time
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

from ._native import gpu_available, native
from .config import Config
from .parallel import topology
from .parallel.dist import DistContext, init_distributed
from .parallel.exchange import TorchHaloExchanger
from .utils import io as h2io
from .utils.device import device_report
from .utils.report import Reporter, metrics


@dataclass
class RunResult:
    steps_done: int
    converged: bool
    residual: float
    elapsed_s: float  # max over ranks of the loop's wall time
    device_ms: float  # this rank's device-event time of the loop
    path: str
    chunks: int
    exchanges: int
    nranks: int
    ntiles: int
    extra: dict = field(default_factory=dict)


def autotune(cfg: Config, model, device: int, candidates_k=(2, 4, 8), candidates_h=(0, 4, 8, 16, 32),
             tile_candidates=((64, 16, 8), (64, 8, 8), (64, 8, 16), (64, 4, 8), (128, 8, 16), (128, 8, 32)),
             trial_steps: int = 0) -> dict:
    """Pick the fastest single-tile GPU path by timing candidates on scratch engines (the real
    field is untouched): the whole-grid LDS solver, the streaming kernel over (K, rows per
    wave H), and the LDS-tiled kernel over (width RY, steps per launch K, tile rows TX).
    Returns the engine keyword overrides of the winner (``engine_kw``) and the timing table."""
    n = native()
    cells = cfg.nx * cfg.ny
    steps = trial_steps or max(32, min(256, int(2e8 // max(1, cells))))
    if cfg.convergence:  # the LDS solver resumes only on a multiple of the check interval
        steps = -(-steps // cfg.interval) * cfg.interval
    base = dict(boundary=model.boundary_id(), precision=model.precision_id(), init=model.init_id(), cx=model.cx,
                cy=model.cy, device=device, convergence=cfg.convergence, interval=cfg.interval,
                sensitivity=-1.0)  # never converges: every candidate runs the same steps
    cands = []
    if n.lds_solver_fits(cfg.nx, cfg.ny) and cfg.small_grid:
        cands.append(("lds", dict(small_grid_lds=True, tiled=0)))
    for K in candidates_k:
        for H in candidates_h:
            cands.append((f"stream K={K} H={H}", dict(tblock=K, rows_per_wave=H, small_grid_lds=False, tiled=0)))
    if cfg.tiled != "off":
        for ry, k, tx in tile_candidates:
            cands.append((f"tiled RY={ry} K={k} TX={tx}",
                          dict(tiled=1, tile_width=ry, tile_k=k, tile_rows=tx, small_grid_lds=False)))
    table = []
    best = None
    for name, kw in cands:
        try:
            e = n.Engine(cfg.nx, cfg.ny, **base, **kw)
        except Exception:
            continue
        e.run(steps)  # warm
        t = min(e.run(steps)["device_ms"] for _ in range(2)) / steps
        table.append((name, t * 1e3))
        if best is None or t < best[2]:
            best = (name, kw, t)
        del e
    return {"choice": best[0], "engine_kw": best[1], "us_per_step": best[2] * 1e3, "table": table}


class Solver:
    def __init__(self, cfg: Config, ctx: Optional[DistContext] = None, device_ordinal: Optional[int] = None):
        self.cfg = cfg
        self.ctx = ctx or init_distributed()
        self.model = cfg.model()
        n = native()
        want_gpu = cfg.device in ("auto", "gpu")
        self.on_gpu = want_gpu and gpu_available()
        if cfg.device == "gpu" and not self.on_gpu:
            raise RuntimeError("--device gpu requested but no HIP device is available")
        world = self.ctx.world
        self.gridx, self.gridy = cfg.resolve_grid(world)
        self.nranks = self.gridx * self.gridy
        if world > 1 and self.nranks != world:
            raise SystemExit(f"ERROR: the number of tasks must be equal to {self.nranks}.\nQuiting...")
        self.dec = topology.decomposition(cfg.nx, cfg.ny, self.gridx, self.gridy, self.model.periodic_x,
                                          self.model.periodic_y)
        ranks = list(range(self.nranks)) if world == 1 else [self.ctx.rank]

        if self.on_gpu and cfg.transport == "ipc":
            # direct peer stores into IPC-mapped receive buffers (1-D row strips); also valid for
            # ranks sharing one GPU and for a single rank that is its own (periodic) neighbour
            transport = n.TRANSPORT_IPC
            if world == 1:
                ranks = [0]
        elif world == 1:
            transport = n.TRANSPORT_LOCAL
        elif self.on_gpu and cfg.transport in ("auto", "rccl"):
            transport = n.TRANSPORT_RCCL
        else:
            transport = n.TRANSPORT_EXTERNAL
        if self.on_gpu:
            ndev = n.device_count()
            self.device = device_ordinal if device_ordinal is not None else (self.ctx.local_rank % ndev)
            torch.cuda.set_device(self.device)
        else:
            self.device = -1
        # ranks on one physical GPU (collective; any visibility setup): persistent launches off on
        # every rank together unless forced, so all ranks' IPC handles carry the same plans
        self.shared_gpu = (world > 1 and self.on_gpu and
                           self.ctx.devices_shared(self.device, n.device_pci_id(self.device)))
        self.transport = transport
        self.tuned = None
        self.engine_kw = {}
        if cfg.tune and self.on_gpu and world == 1 and self.nranks == 1:
            self.tuned = autotune(cfg, self.model, self.device)
            self.engine_kw = dict(self.tuned["engine_kw"])
        if transport == n.TRANSPORT_IPC:
            self.engine = self._init_ipc(ranks)
        else:
            self.engine = self._make_engine(transport, ranks)
        self.exchanger = None
        if transport == n.TRANSPORT_RCCL and self.engine.has_exchange():
            ok = 1
            try:
                uid = n.Engine.rccl_unique_id() if self.ctx.rank == 0 else None
                uid = self.ctx.broadcast_bytes(uid)
                self.engine.init_rccl(uid, world, self.ctx.rank)
            except Exception as e:  # pragma: no cover - needs a broken multi-GPU setup
                ok = 0
                print(f"[rank {self.ctx.rank}] native RCCL init failed: {e}", flush=True)
            if self.ctx.allreduce_sum(ok) < world:
                # every rank falls back together to torch.distributed p2p (nccl backend = RCCL)
                transport = self.transport = n.TRANSPORT_EXTERNAL
                self.engine = self._make_engine(transport, ranks)
        if transport == n.TRANSPORT_EXTERNAL and self.engine.has_exchange():
            dev = torch.device("cuda", self.device) if self.on_gpu else torch.device("cpu")
            host = cfg.transport == "host"
            group = self.ctx.get_nccl_group() if self.on_gpu and not host else None
            self.exchanger = TorchHaloExchanger(self.engine, 0, dev, group, host_staging=self.on_gpu and host)
        if cfg.load:
            full = h2io.read_binary(cfg.load, cfg.nx, cfg.ny)
            for t in range(self.engine.num_tiles()):
                g = self.engine.geom(t)
                self.engine.upload(t, full[g["gx0"]:g["gx0"] + g["xcell"], g["gy0"]:g["gy0"] + g["ycell"]])
            self.engine.set_steps_done(cfg.start_step)
        self.reporter = Reporter(cfg.report, enabled=(self.ctx.rank == 0 and not cfg.quiet))

    def _init_ipc(self, ranks):
        """Engine with the direct IPC transport: all-gather every rank's block handle, map them,
        prime the initial halo.  Collective and failure-safe: if any rank fails (engine
        constraints, IPC mapping), every rank raises the same error (no rank is left waiting
        in a collective)."""
        n, ctx = native(), self.ctx
        eng, err = None, ""
        try:
            eng = self._make_engine(n.TRANSPORT_IPC, ranks)
            h = eng.ipc_handle() if eng.has_exchange() else b""
        except Exception as e:  # noqa: BLE001 - reported collectively below
            err, h = f"{type(e).__name__}: {e}", b""
        if ctx.allreduce_min(0 if err else 1) < 1:
            raise RuntimeError(f"IPC transport unavailable on some rank ({err or 'another rank failed'})")
        if eng.has_exchange():
            hs = ctx.all_gather_bytes(h)
            try:
                eng.ipc_open(hs)
            except Exception as e:  # noqa: BLE001
                err = f"{type(e).__name__}: {e}"
            if ctx.allreduce_min(0 if err else 1) < 1:
                raise RuntimeError(f"IPC mapping failed on some rank ({err or 'another rank failed'})")
            self._ipc_prime(eng)
        return eng

    def _ipc_prime(self, eng) -> None:
        self.ctx.barrier()  # no rank has a kernel in flight
        eng.ipc_prime()
        self.ctx.barrier()  # every receive buffer holds its initial halo

    def _make_engine(self, transport: int, ranks):
        cfg, n = self.cfg, native()
        from .utils.benchmark import PIPELINE_OPTIONS

        kw = dict(tblock=cfg.tblock if cfg.tblock > 0 else (8 if cfg.precision == "fp32" else 7), rows_per_wave=cfg.rows_per_wave, small_grid_lds=cfg.small_grid,
                  tiled={"auto": -1, "on": 1, "off": 0}[cfg.tiled], overlap=cfg.overlap)
        if cfg.pipeline not in PIPELINE_OPTIONS:
            raise ValueError(f"unknown pipeline {cfg.pipeline!r}")
        kw.update(PIPELINE_OPTIONS[cfg.pipeline])
        if cfg.persistent not in ("auto", "on", "off"):
            raise ValueError(f"unknown persistent mode {cfg.persistent!r}")
        if cfg.persistent != "auto":
            kw["persistent"] = 1 if cfg.persistent == "on" else 0
            share = getattr(self.ctx, "ranks_on_device", 1) if getattr(self, "shared_gpu", False) else 1
            if cfg.persistent == "on" and share > 1:
                # a one-GPU rehearsal: the ranks on this GPU split its wave slots, so each rank's
                # persistent launch is resident beside the others'
                kw["pstream_waves"] = 4 * n.device_props(self.device)["multiprocessor_count"] // share
        elif getattr(self, "shared_gpu", False):
            # ranks share a GPU: a persistent launch needs every one of its waves resident, which
            # another rank's persistent launch on the same GPU could prevent — launch per chunk
            # (persistent="on" keeps it: a rehearsal whose ranks' plans fit the GPU together)
            kw["persistent"] = 0
        kw.update(getattr(self, "engine_kw", {}))
        return n.Engine(
            cfg.nx, cfg.ny, gridx=self.gridx, gridy=self.gridy, periodic_x=self.model.periodic_x,
            periodic_y=self.model.periodic_y, boundary=self.model.boundary_id(), precision=self.model.precision_id(),
            init=self.model.init_id(), cx=self.model.cx, cy=self.model.cy, convergence=cfg.convergence,
            interval=cfg.interval, sensitivity=cfg.sensitivity, device=self.device, ranks=ranks,
            transport=transport, naive=cfg.naive, halo_timeout_s=cfg.halo_timeout_s,
            sync_mode=cfg.sync_mode, **kw)

    # ---- data access -------------------------------------------------------------------
    def tiles(self):
        """Yield (gx0, gy0, owned block) for every tile held by this process."""
        for t in range(self.engine.num_tiles()):
            g = self.engine.geom(t)
            yield g["gx0"], g["gy0"], self.engine.download(t)

    def gather(self) -> Optional[np.ndarray]:
        """Full NX×NY grid on rank 0 (None elsewhere).  For tests and small grids."""
        parts = self.ctx.gather_objects(list(self.tiles()))
        if self.ctx.rank != 0:
            return None
        out = np.zeros((self.cfg.nx, self.cfg.ny), dtype=np.float32)
        for plist in parts:
            for gx0, gy0, b in plist:
                out[gx0:gx0 + b.shape[0], gy0:gy0 + b.shape[1]] = b
        return out

    def write(self, which: str) -> None:
        c = self.cfg
        binary = c.output in ("binary", "both")
        text = c.output in ("text", "both")
        h2io.write_grid(c.outdir, which, c.nx, c.ny, self.tiles, rank=self.ctx.rank, barrier=self.ctx.barrier,
                        binary=binary, text=text, text_style=c.text_style)

    # ---- the run ----------------------------------------------------------------------
    def _python_loop(self, steps: int) -> dict:
        """Chunk loop for the external (torch.distributed) transport."""
        eng, c = self.engine, self.cfg
        start = eng.steps_done()
        total = start + steps
        done = start
        st = {"converged": False, "residual": -1.0, "chunks": 0, "exchanges": 0}
        while done < total:
            k, check = eng.next_chunk(done, total)
            if self.exchanger is not None:
                self.exchanger.exchange(k)
                st["exchanges"] += 1
            eng.advance(k, check)
            st["chunks"] += 1
            if check:
                r = self.ctx.allreduce_sum(eng.local_residual())
                st["residual"] = r
                if r < c.sensitivity:
                    eng.rollback()
                    st["converged"] = True
                    break
            done += k
        eng.set_steps_done(done)
        eng.synchronize()
        st["steps_done"] = done
        st["device_ms"] = 0.0
        st["path"] = "external"
        return st

    def run_steps(self, steps: int) -> dict:
        """Advance `steps` steps with whichever loop the transport needs (no barriers/timing)."""
        if self.transport == native().TRANSPORT_EXTERNAL and self.engine.has_exchange():
            return self._python_loop(steps)
        if self.transport == native().TRANSPORT_IPC and self.engine.direct() and not self.engine.ipc_primed():
            self._ipc_prime(self.engine)  # after a resume upload or a converged (rolled-back) run
        return self.engine.run(steps)

    def run(self, steps: Optional[int] = None) -> RunResult:
        steps = self.cfg.steps if steps is None else steps
        self.engine.synchronize()
        self.ctx.node_barrier()  # gloo barrier + node-local spin: ranks start within ~1 us
        t0 = time.perf_counter()
        st = self.run_steps(steps)
        self.engine.synchronize()
        local = time.perf_counter() - t0
        elapsed = self.ctx.allreduce_max(local)
        return RunResult(steps_done=int(st["steps_done"]), converged=bool(st["converged"]),
                         residual=float(st["residual"]), elapsed_s=elapsed, device_ms=float(st["device_ms"]),
                         path=str(st["path"]), chunks=int(st["chunks"]), exchanges=int(st["exchanges"]),
                         nranks=self.nranks, ntiles=self.engine.num_tiles())

    def main(self) -> RunResult:
        """Full program: banners, initial output, timed loop, final output, metrics."""
        c, rep = self.cfg, self.reporter
        g0 = self.dec.tile(0, 0)
        strips = topology.strips_table(self.dec) if c.report == "heat2dn" else None
        if c.debug and self.ctx.rank == 0 and self.on_gpu:
            rep._p(device_report())
        rep.start(nprocs=self.nranks, nx=c.nx, ny=c.ny, xcell=g0["xcell"], ycell=g0["ycell"], steps=c.steps,
                  convergence=c.convergence, interval=c.interval, numthreads=c.numthreads, strips=strips)
        if c.debug:
            host = socket.gethostname()
            for t in range(self.engine.num_tiles()):
                r = self.engine.tile_rank(t)
                Reporter(c.report, enabled=not c.quiet).debug_neighbors(r, topology.neighbors(self.dec, r), host)
        if c.output != "none":
            rep.writing_initial()
            self.write("initial")
        rep.begin_steps(strips)
        res = self.run()
        rep.finish(steps_done=res.steps_done, elapsed_s=res.elapsed_s, writes_final=c.output != "none")
        if c.output != "none":
            self.write("final")
        if c.save:
            self.save(c.save)
        if c.json and self.ctx.rank == 0:
            Reporter(c.report, enabled=True).json_line(metrics(c.nx, c.ny, res.steps_done, res.elapsed_s, ranks=self.nranks,
                                  tiles=res.ntiles, path=res.path, converged=res.converged,
                                  residual=res.residual, device="gpu" if self.on_gpu else "cpu",
                                  precision=c.precision, boundary=c.boundary, tblock=self.engine.halo_depth(),
                                  chunks=res.chunks, exchanges=res.exchanges, pipeline=self.engine.pipeline()))
        return res

    def save(self, path: str) -> None:
        """Checkpoint: the raw NX×NY grid (same layout as final_binary.dat)."""
        n = native()
        if self.ctx.rank == 0:
            n.binary_create(path, self.cfg.nx, self.cfg.ny)
        self.ctx.barrier()
        for gx0, gy0, b in self.tiles():
            n.binary_write_tile(path, self.cfg.nx, self.cfg.ny, gx0, gy0, b)
        self.ctx.barrier()

    def close(self) -> None:
        """Release the engine (device buffers, streams, RCCL communicator) now."""
        self.exchanger = None
        self.engine = None
