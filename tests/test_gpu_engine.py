"""GPU tests: the HIP kernels and the native engine against the bit-exact CPU oracle.

Every result in the ``ref`` precision must be bit-identical to ``oracle_run`` (the serial
reference semantics); fp32 results must be bit-identical to the CPU engine's fp32 path
(both use fused multiply-adds) and within tolerance of a plain PyTorch fp32 stencil.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SIZES = [(1, 1), (2, 3), (7, 5), (37, 250), (64, 256), (100, 517), (257, 241), (300, 1000), (40, 4096), (33, 4094)]


def oracle(n, nx, ny, steps, boundary=0, precision=0, init=0, per=(False, False), **kw):
    return n.oracle_run(nx, ny, steps, boundary=boundary, precision=precision, init=init, periodic_x=per[0],
                        periodic_y=per[1], **kw)


@pytest.mark.parametrize("nx,ny", SIZES)
@pytest.mark.parametrize("boundary", [0, 1])
def test_stream_single_tile_bitexact(native, gpu, nx, ny, boundary):
    steps = 23
    eng = native.Engine(nx, ny, boundary=boundary, tblock=8, device=gpu, small_grid_lds=False, tiled=0)
    st = eng.run(steps)
    assert st["path"] == "stream" and st["steps_done"] == steps
    ref = oracle(native, nx, ny, steps, boundary)["grid"]
    got = eng.download(0)
    assert np.array_equal(got, ref), np.abs(got - ref).max()


@pytest.mark.parametrize("K", [1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 16])
def test_every_compiled_K(native, gpu, K):
    nx, ny, steps = 203, 611, 2 * K + 3
    for boundary in (0, 1):
        eng = native.Engine(nx, ny, boundary=boundary, tblock=K, device=gpu, small_grid_lds=False, tiled=0,
                            rows_per_wave=max(16, 4 * K))
        assert eng.halo_depth() == K
        eng.run(steps)
        ref = oracle(native, nx, ny, steps, boundary)["grid"]
        assert np.array_equal(eng.download(0), ref), (K, boundary)


def test_bench_shape_4096_k7_writethrough(native, gpu):
    """Exactly the timed configuration of the headline bench: 4096^2, depth 7, write-through
    output stores, 20 steps = 7+7+6, capacity-fitted units (~1000, h ~ 68) — against the oracle."""
    eng = native.Engine(4096, 4096, tblock=7, device=gpu, small_grid_lds=False, tiled=0, wt_store=1)
    st = eng.run(20)
    assert st["path"] == "stream" and st["steps_done"] == 20 and st["chunks"] == 3
    assert eng.num_units(7) > 900
    assert np.array_equal(eng.download(0), oracle(native, 4096, 4096, 20)["grid"])


@pytest.mark.parametrize("rows,K", [(512, 6), (1024, 7)])
def test_strong_scaling_rank_tiles_direct(native, gpu, rows, K):
    """The per-rank tiles of 4096^2 over 8 and 4 GPUs, row-periodic through the direct IPC
    pipeline (the rank is its own neighbour): bit-exact, and the halo-wait counters see every
    halo unit's wait."""
    steps = 3 * K + 2
    e = native.Engine(rows, 4096, periodic_x=True, tblock=K, device=gpu, ranks=[0], transport=native.TRANSPORT_IPC,
                      halo_timeout_s=5.0)
    e.ipc_open([e.ipc_handle()])
    e.ipc_prime()
    e.reset_halo_wait()
    st = e.run(steps)
    assert st["steps_done"] == steps
    ref = oracle(native, rows, 4096, steps, per=(True, False))["grid"]
    assert np.array_equal(e.download(0), ref)
    hw = e.halo_wait()
    halo_units = sum(1 for u in e.unit_list(0, K, 3) if u[3] & 4) * 2  # top + bottom units per strip
    assert hw["waits"] >= halo_units and hw["max_us"] >= 0.0 and hw["total_us"] >= 0.0


def test_timeline_stamps(native, gpu):
    e = native.Engine(256, 4096, tblock=6, device=gpu, small_grid_lds=False, tiled=0, timeline=8)
    e.run(12)
    tl = e.timeline()
    assert [k for k, _ in tl] == [6, 6]
    for _k, st in tl:
        assert st.shape[1] == 4 and (st[:, 2] >= st[:, 1]).all() and (st[:, 1] >= st[:, 0]).all()
    assert tl[1][1][:, 0].min() >= tl[0][1][:, 2].min()  # the second launch starts after the first's waves


@pytest.mark.parametrize("H", [1, 5, 16, 64, 300])
def test_rows_per_wave_variants(native, gpu, H):
    nx, ny, steps = 150, 300, 17
    eng = native.Engine(nx, ny, tblock=8, rows_per_wave=H, device=gpu, small_grid_lds=False, tiled=0)
    eng.run(steps)
    assert np.array_equal(eng.download(0), oracle(native, nx, ny, steps)["grid"])


def test_int32_init_and_float_coeff(native, gpu):
    nx, ny, steps = 640, 512, 9
    cx = native.CX_FLOAT
    eng = native.Engine(nx, ny, init=native.INIT_INT32, cx=cx, cy=cx, device=gpu, small_grid_lds=False, tiled=0)
    eng.run(steps)
    ref = oracle(native, nx, ny, steps, init=1, cx=cx, cy=cx)["grid"]
    assert np.array_equal(eng.download(0), ref)


def test_fp32_matches_cpu_fp32_and_torch(native, gpu):
    nx, ny, steps = 211, 333, 30
    g = native.Engine(nx, ny, precision=native.FP32, device=gpu, small_grid_lds=False, tiled=0)
    g.run(steps)
    c = native.Engine(nx, ny, precision=native.FP32, device=-1)
    c.run(steps)
    got = g.download(0)
    assert np.array_equal(got, c.download(0))
    # plain PyTorch fp32 reference of the same op
    u = torch.from_numpy(native.init_global(nx, ny, 0)).double()
    for _ in range(steps):
        v = u.clone()
        v[1:-1, 1:-1] = u[1:-1, 1:-1] + 0.1 * (u[2:, 1:-1] + u[:-2, 1:-1] - 2 * u[1:-1, 1:-1]) + \
            0.1 * (u[1:-1, 2:] + u[1:-1, :-2] - 2 * u[1:-1, 1:-1])
        u = v.float().double()
    ref = u.float().numpy()
    rel = np.abs(got - ref).max() / np.abs(ref).max()
    assert rel < 1e-5, rel


@pytest.mark.parametrize("nx,ny", [(10, 10), (80, 64), (160, 128), (33, 7)])
def test_lds_small_grid_solver(native, gpu, nx, ny):
    steps = 1000
    for boundary in (0, 1):
        eng = native.Engine(nx, ny, boundary=boundary, device=gpu, tiled=0)
        st = eng.run(steps)
        assert st["path"] == "lds"
        assert np.array_equal(eng.download(0), oracle(native, nx, ny, steps, boundary)["grid"])


def test_naive_kernel(native, gpu):
    nx, ny, steps = 129, 257, 11
    eng = native.Engine(nx, ny, boundary=1, device=gpu, naive=True)
    st = eng.run(steps)
    assert st["path"] == "naive"
    assert np.array_equal(eng.download(0), oracle(native, nx, ny, steps, 1)["grid"])


@pytest.mark.parametrize("gx,gy", [(1, 2), (2, 1), (2, 2), (2, 4), (4, 2), (3, 3)])
@pytest.mark.parametrize("overlap", [True, False])
def test_local_multitile_decomposition_invariance(native, gpu, gx, gy, overlap):
    nx, ny, steps = 301, 599, 41
    for boundary in (0, 1):
        eng = native.Engine(nx, ny, gridx=gx, gridy=gy, boundary=boundary, tblock=8, device=gpu, overlap=overlap)
        st = eng.run(steps)
        assert st["exchanges"] > 0
        out = np.zeros((nx, ny), np.float32)
        for t in range(eng.num_tiles()):
            g = eng.geom(t)
            out[g["gx0"]:g["gx0"] + g["xcell"], g["gy0"]:g["gy0"] + g["ycell"]] = eng.download(t)
        assert np.array_equal(out, oracle(native, nx, ny, steps, boundary)["grid"]), (gx, gy, boundary)


def test_periodic_multitile(native, gpu):
    nx, ny, steps = 120, 260, 30
    eng = native.Engine(nx, ny, gridx=2, gridy=2, periodic_x=True, periodic_y=True, boundary=1, device=gpu)
    eng.run(steps)
    out = np.zeros((nx, ny), np.float32)
    for t in range(4):
        g = eng.geom(t)
        out[g["gx0"]:g["gx0"] + g["xcell"], g["gy0"]:g["gy0"] + g["ycell"]] = eng.download(t)
    assert np.array_equal(out, oracle(native, nx, ny, steps, 1, per=(True, True))["grid"])


@pytest.mark.parametrize("gx,gy", [(1, 1), (2, 2)])
def test_convergence_matches_oracle(native, gpu, gx, gy):
    nx, ny = 40, 40
    kw = dict(convergence=True, interval=20, sensitivity=0.1)
    ref = oracle(native, nx, ny, 20000, 0, **kw)
    assert ref["converged"]
    for lds in (True, False):
        eng = native.Engine(nx, ny, gridx=gx, gridy=gy, device=gpu, small_grid_lds=lds, **kw)
        st = eng.run(20000)
        assert st["converged"] and st["steps_done"] == ref["steps_done"], (st, ref["steps_done"])
        out = np.zeros((nx, ny), np.float32)
        for t in range(eng.num_tiles()):
            g = eng.geom(t)
            out[g["gx0"]:g["gx0"] + g["xcell"], g["gy0"]:g["gy0"] + g["ycell"]] = eng.download(t)
        assert np.array_equal(out, ref["grid"])


def test_rccl_self_exchange_periodic(native, gpu):
    """One rank, periodic in both dims: every halo goes through ncclSend/ncclRecv to itself."""
    nx, ny, steps = 96, 300, 25
    eng = native.Engine(nx, ny, periodic_x=True, periodic_y=True, boundary=1, device=gpu, ranks=[0],
                        transport=native.TRANSPORT_RCCL)
    eng.init_rccl(native.Engine.rccl_unique_id(), 1, 0)
    st = eng.run(steps)
    assert st["exchanges"] > 0
    assert np.array_equal(eng.download(0), oracle(native, nx, ny, steps, 1, per=(True, True))["grid"])


def test_rccl_convergence_allreduce(native, gpu):
    nx, ny = 48, 40
    kw = dict(convergence=True, interval=10, sensitivity=1e3)
    ref = oracle(native, nx, ny, 5000, 1, per=(True, False), **kw)
    eng = native.Engine(nx, ny, periodic_x=True, boundary=1, device=gpu, ranks=[0], transport=native.TRANSPORT_RCCL,
                        **kw)
    eng.init_rccl(native.Engine.rccl_unique_id(), 1, 0)
    st = eng.run(5000)
    assert st["steps_done"] == ref["steps_done"] and st["converged"] == ref["converged"]
    assert np.array_equal(eng.download(0), ref["grid"])


# pipeline: 0 serial (exchange, then the chunk), 3 signalled (one launch per chunk, exchange
# gated mid-kernel by hipStreamWaitValue64), 4 signalled with a polling-kernel gate (the
# default), 5 the same with the chunk launch waiting on a halo event instead of the in-kernel halo
# wait, 6 signalled with short boundary units instead of full-size mid-unit-signalling ones
PIPELINES = {0: dict(overlap=False), 3: dict(signal_exchange=1), 4: dict(signal_exchange=2),
             5: dict(signal_exchange=2, device_halo_wait=0), 6: dict(signal_exchange=2, signal_plan=0)}
PIPELINE_NAMES = {0: "serial", 3: "signal", 4: "signal", 5: "signal", 6: "signal"}


@pytest.mark.parametrize("gx,gy", [(2, 1), (4, 1), (2, 2), (1, 3)])
@pytest.mark.parametrize("pipeline", [0, 3, 4, 5, 6])
def test_overlap_pipelines(native, gpu, gx, gy, pipeline):
    """Serial and signalled pipelines (local multi-tile transport), with convergence."""
    nx, ny, steps = 257, 509, 45
    kw = dict(convergence=True, interval=9, sensitivity=1e-30)
    for boundary in (0, 1):
        eng = native.Engine(nx, ny, gridx=gx, gridy=gy, boundary=boundary, tblock=8, device=gpu,
                            **PIPELINES[pipeline], **kw)
        assert eng.pipeline() == PIPELINE_NAMES[pipeline]
        st = eng.run(steps)
        assert st["steps_done"] == steps
        ref = oracle(native, nx, ny, steps, boundary, **kw)
        out = np.zeros((nx, ny), np.float32)
        for t in range(eng.num_tiles()):
            g = eng.geom(t)
            out[g["gx0"]:g["gx0"] + g["xcell"], g["gy0"]:g["gy0"] + g["ycell"]] = eng.download(t)
        assert np.array_equal(out, ref["grid"]), (gx, gy, boundary, pipeline)


def test_pipeline_auto(native, gpu):
    assert native.Engine(2048, 2048, gridx=4, gridy=1, device=gpu).pipeline() == "signal"
    assert native.Engine(2048, 2048, gridx=4, gridy=1, device=gpu, signal_exchange=0).pipeline() == "serial"
    assert native.Engine(2048, 2048, gridx=2, gridy=2, device=gpu, overlap=False).pipeline() == "serial"
    assert native.Engine(2048, 2048, device=gpu).pipeline() == "none"


@pytest.mark.parametrize("pipeline", [0, 3, 4, 5, 6])
@pytest.mark.parametrize("contig,comm_cus", [(0, 0), (1, 0), (1, 8), (0, 4)])
@pytest.mark.parametrize("boundary", [0, 1])
def test_rccl_self_exchange_row_periodic(native, gpu, pipeline, contig, comm_cus, boundary):
    """Row-periodic single rank: the per-rank shape of the 1-D row-strip bench.  Covers the
    contiguous K-row halo path (no pack/unpack) and CU-partitioned comm/compute streams."""
    nx, ny, steps = 300, 701, 37
    eng = native.Engine(nx, ny, periodic_x=True, boundary=boundary, device=gpu, ranks=[0],
                        transport=native.TRANSPORT_RCCL, contiguous_halo=contig,
                        comm_cus=comm_cus, poison=True, **PIPELINES[pipeline])
    assert eng.contiguous_halo() == bool(contig) and eng.comm_cus() == comm_cus
    eng.init_rccl(native.Engine.rccl_unique_id(), 1, 0)
    eng.run(steps)
    assert np.array_equal(eng.download(0), oracle(native, nx, ny, steps, boundary, per=(True, False))["grid"])


# ---- LDS-tiled temporally-blocked path (tile_kernel.hip) --------------------------------
TILE_SIZES = [(1, 1), (3, 2), (80, 64), (97, 131), (160, 128), (257, 509), (320, 256)]


@pytest.mark.parametrize("nx,ny", TILE_SIZES)
@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("width,K", [(64, 8), (128, 16), (64, 1), (128, 5), (32, 6), (32, 14)])
@pytest.mark.parametrize("nt,cpl", [(256, 4), (1024, 4), (1024, 2), (256, 1)])
def test_tiled_bitexact(native, gpu, nx, ny, boundary, width, K, nt, cpl):
    steps = 2 * K + 5  # full chunks and a partial one
    kw = dict(boundary=boundary, device=gpu, small_grid_lds=False, tiled=1, tile_width=width, tile_k=K, tile_rows=16,
              tile_threads=nt, tile_cpl=cpl, poison=True)
    if 16 + 2 * K > 8 * nt // (width // max(cpl, width // 64)):  # a lane owns at most 8 region rows
        with pytest.raises(Exception, match="tile configuration"):
            native.Engine(nx, ny, **kw)
        return
    eng = native.Engine(nx, ny, **kw)
    st = eng.run(steps)
    assert st["path"] == "tiled" and st["steps_done"] == steps and eng.tile_config() == [16, width, K]
    assert eng.tile_threads() == nt and eng.tile_cpl() == max(cpl, width // 64)
    ref = oracle(native, nx, ny, steps, boundary)["grid"]
    got = eng.download(0)
    assert np.array_equal(got, ref), np.abs(got - ref).max()


@pytest.mark.parametrize("per", [(True, False), (False, True), (True, True)])
@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("nt,cpl,width", [(256, 4, 64), (1024, 4, 64), (1024, 1, 32), (1024, 2, 64)])
def test_tiled_periodic(native, gpu, per, boundary, nt, cpl, width):
    nx, ny, steps = 45, 70, 29
    eng = native.Engine(nx, ny, boundary=boundary, periodic_x=per[0], periodic_y=per[1], device=gpu, tiled=1,
                        tile_k=6, tile_rows=8, tile_threads=nt, tile_cpl=cpl, tile_width=width)
    assert eng.run(steps)["path"] == "tiled"
    assert np.array_equal(eng.download(0), oracle(native, nx, ny, steps, boundary, per=per)["grid"])


@pytest.mark.parametrize("precision", [0, 1])
@pytest.mark.parametrize("nt,cpl", [(256, 4), (1024, 4), (1024, 2), (1024, 1)])
def test_tiled_convergence_and_fp32(native, gpu, precision, nt, cpl):
    nx, ny = 120, 200
    kw = dict(convergence=True, interval=7, sensitivity=5e3)
    ref = oracle(native, nx, ny, 3000, 0, precision=precision, **kw)
    eng = native.Engine(nx, ny, precision=precision, device=gpu, tiled=1, tile_k=8, tile_threads=nt, tile_cpl=cpl,
                        small_grid_lds=False, **kw)
    st = eng.run(3000)
    assert st["path"] == "tiled"
    assert st["steps_done"] == ref["steps_done"] and st["converged"] == ref["converged"]
    assert np.array_equal(eng.download(0), ref["grid"])


def test_tiled_auto_selection(native, gpu):
    assert native.Engine(640, 512, device=gpu).tiled()
    assert not native.Engine(4096, 4096, device=gpu).tiled()
    assert not native.Engine(640, 512, gridx=2, device=gpu).tiled()  # several tiles
    assert not native.Engine(640, 512, device=gpu, tiled=0).tiled()


# ---- direct IPC transport (halo units push rows into the neighbour's receive buffers) -----
def _ipc_engine(native, **kw):
    eng = native.Engine(ranks=[0], transport=native.TRANSPORT_IPC, halo_timeout_s=5.0, **kw)
    eng.ipc_open([eng.ipc_handle()])  # one rank: its own block (it is its own periodic neighbour)
    eng.ipc_prime()
    return eng


@pytest.mark.parametrize("nx,ny", [(96, 300), (300, 701), (257, 4096), (64, 40)])
@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("tblock", [8, 5, 16])
def test_ipc_direct_self_exchange_row_periodic(native, gpu, nx, ny, boundary, tblock):
    """Row-periodic single rank over the direct pipeline: every halo goes through the push /
    flag / receive-buffer protocol (its own block), with balanced, ragged and K-changing chunks."""
    steps = 3 * tblock + 11
    eng = _ipc_engine(native, nx=nx, ny=ny, periodic_x=True, boundary=boundary, tblock=tblock, device=gpu,
                      poison=True)
    assert eng.pipeline() == "direct" and eng.direct()
    st = eng.run(steps)
    assert st["steps_done"] == steps and st["exchanges"] > 0
    ref = oracle(native, nx, ny, steps, boundary, per=(True, False))["grid"]
    assert np.array_equal(eng.download(0), ref)
    # a second run continues the push/flag sequence (no re-prime), odd length
    eng.run(7)
    ref = oracle(native, nx, ny, steps + 7, boundary, per=(True, False))["grid"]
    assert np.array_equal(eng.download(0), ref)


@pytest.mark.parametrize("nx,ny", [(96, 300), (300, 704), (257, 4096), (64, 64)])
@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("tblock", [8, 5, 16])
def test_ipc_direct_2d_self_exchange(native, gpu, nx, ny, boundary, tblock):
    """Periodic in both dimensions, one rank: all eight neighbours are the rank itself, so every
    halo — rows, W/E ghost columns and the four corners — goes through the 2-D direct protocol
    (pushes into the ghost-column groups, per-direction flags and counts, K-changing chunks)."""
    steps = 3 * tblock + 11
    eng = _ipc_engine(native, nx=nx, ny=ny, periodic_x=True, periodic_y=True, boundary=boundary, tblock=tblock,
                      device=gpu, poison=True)
    assert eng.pipeline() == "direct"
    K = eng.halo_depth()
    units = eng.unit_list(0, K, 3)
    assert any(u[7] & 0x3f for u in units)  # side-linked units exist
    eng.reset_halo_wait()
    st = eng.run(steps)
    assert st["steps_done"] == steps
    ref = oracle(native, nx, ny, steps, boundary, per=(True, True))["grid"]
    got = eng.download(0)
    assert np.array_equal(got, ref), np.argwhere(got != ref)[:5]
    assert eng.halo_wait()["waits"] > 0
    eng.run(7)  # continues the flag sequence (no re-prime)
    assert np.array_equal(eng.download(0), oracle(native, nx, ny, steps + 7, boundary, per=(True, True))["grid"])


def test_ipc_direct_2d_convergence(native, gpu):
    nx, ny = 96, 300
    kw = dict(convergence=True, interval=10, sensitivity=1e12)
    ref = oracle(native, nx, ny, 5000, 1, per=(True, True), **kw)
    assert ref["converged"]
    eng = _ipc_engine(native, nx=nx, ny=ny, periodic_x=True, periodic_y=True, boundary=1, device=gpu, **kw)
    st = eng.run(5000)
    assert st["converged"] and st["steps_done"] == ref["steps_done"]
    assert np.array_equal(eng.download(0), ref["grid"])


def test_ipc_direct_2d_rejects_unaligned_width(native, gpu):
    with pytest.raises(Exception, match="multiple of 4"):
        native.Engine(96, 302, periodic_x=True, periodic_y=True, ranks=[0], transport=native.TRANSPORT_IPC,
                      device=gpu)


@pytest.mark.parametrize("wt", [0, 1])
@pytest.mark.parametrize("path", ["single", "tiles", "ipc"])
def test_output_store_policy_bitexact(native, gpu, wt, path):
    """Plain and write-through (buffer_store sc1, scalar row offsets incl. bottom-up units)
    output stores give the same grid as the oracle on every streaming path."""
    nx, ny, steps, boundary = 300, 701, 29, 1
    kw = dict(boundary=boundary, tblock=8, device=gpu, poison=True, wt_store=wt, small_grid_lds=False, tiled=0)
    if path == "ipc":
        eng = _ipc_engine(native, nx=nx, ny=ny, periodic_x=True, **kw)
        per = (True, False)
    else:
        eng = native.Engine(nx, ny, gridx=3 if path == "tiles" else 1, **kw)
        per = (False, False)
    eng.run(steps)
    got = eng.download(0) if path != "tiles" else _gather(eng, nx, ny)
    assert np.array_equal(got, oracle(native, nx, ny, steps, boundary, per=per)["grid"])


def test_ipc_direct_convergence_and_reprime(native, gpu):
    nx, ny = 96, 300
    kw = dict(convergence=True, interval=10, sensitivity=1e12)
    ref = oracle(native, nx, ny, 5000, 1, per=(True, False), **kw)
    assert ref["converged"] and ref["steps_done"] == 219
    eng = _ipc_engine(native, nx=nx, ny=ny, periodic_x=True, boundary=1, device=gpu, **kw)
    st = eng.run(5000)
    assert st["converged"] and st["steps_done"] == ref["steps_done"]
    assert np.array_equal(eng.download(0), ref["grid"])
    assert not eng.ipc_primed()  # the rollback invalidated the pushed halos
    with pytest.raises(RuntimeError):
        eng.run(5)
    eng.ipc_prime()
    eng.run(5)


def test_ipc_direct_rejects_unsupported(native, gpu):
    with pytest.raises(Exception):  # two tiles in one process
        native.Engine(96, 300, gridx=1, gridy=2, transport=native.TRANSPORT_IPC, device=gpu)
    with pytest.raises(Exception):  # tile too short for full-size halo units
        native.Engine(12, 300, periodic_x=True, ranks=[0], transport=native.TRANSPORT_IPC, device=gpu)


# ---- fused (device-side) convergence: checks end a chunk, no host round trip --------------
CONV = dict(convergence=True, interval=9, sensitivity=1.93e13)  # ghost-zero 257x509: converges at 98 steps


def _gather(eng, nx, ny):
    out = np.zeros((nx, ny), np.float32)
    for t in range(eng.num_tiles()):
        g = eng.geom(t)
        out[g["gx0"]:g["gx0"] + g["xcell"], g["gy0"]:g["gy0"] + g["ycell"]] = eng.download(t)
    return out


def _ranges(v):
    v = sorted(set(int(x) for x in v))
    out, a = [], None
    for i, x in enumerate(v):
        if a is None:
            a = x
        if i + 1 == len(v) or v[i + 1] != x + 1:
            out.append(f"{a}-{x}" if a != x else f"{a}")
            a = None
    return ",".join(out[:12]) + ("..." if len(out) > 12 else "")


@pytest.mark.parametrize("gx,gy", [(1, 1), (2, 1), (1, 2)])
@pytest.mark.parametrize("pipeline", [0, 3, 4, 5, 6])
def test_fused_convergence_matches_oracle(native, gpu, gx, gy, pipeline):
    """Convergence (check every 9 steps) on every pipeline, fused (device-side) and host-synchronised
    checks: the converged step, residual and grid of the oracle.  The run advances in 9-step pieces
    (one check each, the same chunks as one long run) in lockstep with the CPU engine of the same
    decomposition, so a divergence is caught at the piece where it happens."""
    nx, ny = 257, 509
    ref = oracle(native, nx, ny, 3000, 1, **CONV)
    assert ref["converged"] and ref["steps_done"] == 98
    for fused in (-1, 0):
        eng = native.Engine(nx, ny, gridx=gx, gridy=gy, boundary=1, tblock=8, device=gpu, fused_check=fused,
                            small_grid_lds=False, tiled=0, **PIPELINES[pipeline], **CONV)
        cpu = native.Engine(nx, ny, gridx=gx, gridy=gy, boundary=1, tblock=8, device=-1, **CONV)
        for piece in range(1, 40):
            st, sc = eng.run(9), cpu.run(9)
            got, want = _gather(eng, nx, ny), _gather(cpu, nx, ny)
            if not np.array_equal(got, want) or st["converged"] != sc["converged"]:
                bad = got != want
                r, c = np.nonzero(bad)
                per_tile = []
                for t in range(eng.num_tiles()):
                    g = eng.geom(t)
                    bt = bad[g["gx0"]:g["gx0"] + g["xcell"], g["gy0"]:g["gy0"] + g["ycell"]]
                    per_tile.append(int(bt.sum()))
                pytest.fail(f"fused={fused}: piece {piece} (steps {9 * (piece - 1)}-{9 * piece}): wrong cells "
                            f"{int(bad.sum())} per tile {per_tile} rows {_ranges(r)} cols {_ranges(c)}"
                            + (f" max|d| {float(np.abs(got - want)[bad].max()):.4g}" if bad.any() else "")
                            + f"; converged {st['converged']} vs {sc['converged']}, residual {st['residual']!r} "
                              f"vs {sc['residual']!r}; path {st['path']} chunks {st['chunks']}")
            if st["converged"]:
                break
        assert st["converged"] and st["steps_done"] == ref["steps_done"]
        assert abs(st["residual"] - ref["residual"]) <= 1e-9 * ref["residual"]
        assert np.array_equal(_gather(eng, nx, ny), ref["grid"]), (gx, gy, pipeline, fused)
        # continuing re-checks at step 99 against the converged state: converged again, same state
        st2 = eng.run(5)
        assert st2["converged"] and st2["steps_done"] == ref["steps_done"]
        assert np.array_equal(_gather(eng, nx, ny), ref["grid"])
        del eng, cpu


def _outside_nonzero(eng, t, b):
    """Cells of buffer b of tile t that lie outside the global grid (ghost-zero: must stay 0)."""
    g = eng.geom(t)
    st = eng.storage(t, b)
    G, PL = g["G"], g["PL"]
    rows = np.arange(st.shape[0])[:, None] - G + g["gx0"]
    cols = np.arange(st.shape[1])[None, :] - PL + g["gy0"]
    out = (rows < 0) | (rows >= g["NX"]) | (cols < 0) | (cols >= g["NY"])
    # only the ghost ring the stencil can read (G rows / PL columns around the owned block)
    ring = (np.arange(st.shape[1])[None, :] < PL + g["ycell"] + G) & (np.arange(st.shape[1])[None, :] >= PL - G)
    r, c = np.nonzero(out & ring & (st != 0))
    return len(r), (_ranges(r - G), _ranges(c - PL)) if len(r) else None


# Engine orders: the previous engine released before the next is built (release-first), the
# next built while the previous is alive and the previous released right before the run
# (create-first: the plain `eng = Engine(...)` in a loop), and the previous kept alive through the
# run (create-keep).  With the HIP runtime's kernel arguments in device memory these orders
# computed wrong tiles in the long GPU test process and sometimes faulted (rounds 3-5); the
# library's default (host-memory arguments, free since round 5's preloaded kernel arguments) is
# what this test runs (docs/ARCHITECTURE.md, "Kernel arguments and metadata memory").
_SERIAL_ORDERS = ["release-first", "create-first", "create-keep"] + [o for o in os.environ.get("H2D_SERIAL_ORDERS", "").split(",") if o]


@pytest.mark.parametrize("order", _SERIAL_ORDERS)
@pytest.mark.parametrize("gx,gy", [(2, 1), (1, 2)])
def test_serial_tiles_long_convergence_run(native, gpu, gx, gy, order):
    """The local two-tile serial pipeline with checks every 9 steps, as ONE run of up to 3000 steps
    (fused and host-synchronised checks): converges at the oracle's step with its grid.  On a
    mismatch it reports the wrong owned cells per tile and any non-zero cell of the zero ghost
    ring in either buffer (a stray writer)."""
    nx, ny = 257, 509
    ref = oracle(native, nx, ny, 3000, 1, **CONV)
    eng = None
    kept = []
    for fused in (-1, 0):
        if order == "release-first":
            eng = None  # the previous engine is released before the next one is built
        elif order == "create-keep":
            kept.append(eng)  # the previous engine stays alive through the next run
        # canary (create-keep): every byte of the kept engines' storage, before the next run
        canary = [(k, t, b, k.storage(t, b)) for k in kept if k is not None for t in range(k.num_tiles())
                  for b in (0, 1)]
        eng = native.Engine(nx, ny, gridx=gx, gridy=gy, boundary=1, tblock=8, device=gpu, fused_check=fused,
                            small_grid_lds=False, tiled=0, overlap=False, **CONV)
        st = eng.run(3000)
        for k, t, b, before in canary:  # an idle engine's memory: no stray writer touched it
            after = k.storage(t, b)
            assert np.array_equal(before.view(np.uint32), after.view(np.uint32)), \
                f"kept engine tile {t} buffer {b}: {int((before.view(np.uint32) != after.view(np.uint32)).sum())} words changed"
        got = _gather(eng, nx, ny)
        if not (st["converged"] and st["steps_done"] == ref["steps_done"] and np.array_equal(got, ref["grid"])):
            want = oracle(native, nx, ny, int(st["steps_done"]), 1)["grid"]
            bad = got != want
            lines = [f"fused={fused}: converged {st['converged']} steps {st['steps_done']} residual {st['residual']!r}"]
            for t in range(eng.num_tiles()):
                g = eng.geom(t)
                bt = bad[g["gx0"]:g["gx0"] + g["xcell"], g["gy0"]:g["gy0"] + g["ycell"]]
                r, c = np.nonzero(bt)
                lines.append(f"tile {t} (cur {eng.current_buffer(t)}): wrong {int(bt.sum())} rows {_ranges(r)} cols "
                             f"{_ranges(c)}; ring non-zero buf0 {_outside_nonzero(eng, t, 0)} buf1 "
                             f"{_outside_nonzero(eng, t, 1)}")
            eng = None
            pytest.fail("\n".join(lines))
        # create-first: the next engine is built while this one is alive and this one is released
        # right before the next run (the engine order of the round-3 failures)


@pytest.mark.parametrize("interval", [1, 4, 8, 9, 20])
@pytest.mark.parametrize("tblock", [8, 5])
def test_fused_convergence_intervals(native, gpu, interval, tblock):
    nx, ny = 257, 509
    kw = dict(convergence=True, interval=interval, sensitivity=2.68e13)
    ref = oracle(native, nx, ny, 3000, 1, **kw)
    assert ref["converged"]
    eng = native.Engine(nx, ny, boundary=1, tblock=tblock, device=gpu, small_grid_lds=False, tiled=0, poison=True,
                        **kw)
    st = eng.run(3000)
    assert st["converged"] and st["steps_done"] == ref["steps_done"]
    assert np.array_equal(eng.download(0), ref["grid"])


@pytest.mark.parametrize("interval,tile_k", [(20, 16), (9, 16), (7, 6), (1, 8), (16, 16), (33, 16)])
def test_tiled_chunks_run_through_checks(native, gpu, interval, tile_k):
    """Tiled lone tile with the fused check: chunks span check steps (the residual is summed at
    the check's level inside the launch), a converged check is rolled back by recomputation —
    same converged step and grid as the oracle, and fewer launches than one-chunk-per-check."""
    nx, ny = 257, 509
    for sens in (2.68e13, 0.0):  # converges (after a few checks) / never converges
        kw = dict(convergence=True, interval=interval, sensitivity=sens)
        ref = oracle(native, nx, ny, 400, 1, **kw)
        eng = native.Engine(nx, ny, boundary=1, device=gpu, tiled=1, tile_k=tile_k, small_grid_lds=False, **kw)
        st = eng.run(400)
        assert st["path"] == "tiled" and st["converged"] == ref["converged"]
        assert st["steps_done"] == ref["steps_done"], (st, ref["steps_done"])
        assert np.array_equal(eng.download(0), ref["grid"])
        if not ref["converged"]:
            # one check per launch: intervals shorter than tile_k launch once per check
            assert st["chunks"] <= -(-400 // tile_k) + 400 // interval + 1
            if interval >= tile_k:
                assert st["chunks"] <= -(-400 // tile_k) + 400 // tile_k + 1


def test_fused_convergence_tiled_and_split_runs(native, gpu):
    nx, ny = 257, 509
    ref = oracle(native, nx, ny, 3000, 1, **CONV)
    eng = native.Engine(nx, ny, boundary=1, device=gpu, tiled=1, tile_k=8, small_grid_lds=False, **CONV)
    st = eng.run(3000)
    assert st["path"] == "tiled" and st["converged"] and st["steps_done"] == 98
    assert np.array_equal(eng.download(0), ref["grid"])
    # a run split into pieces that end between checks converges at the same step
    eng = native.Engine(nx, ny, boundary=1, device=gpu, tiled=0, small_grid_lds=False, **CONV)
    done = 0
    for piece in (13, 22, 31, 3000):
        st = eng.run(piece)
        done = st["steps_done"]
        if st["converged"]:
            break
    assert st["converged"] and done == 98 and np.array_equal(eng.download(0), ref["grid"])


def test_fused_convergence_rccl_and_ipc_self(native, gpu):
    nx, ny = 96, 300
    kw = dict(convergence=True, interval=10, sensitivity=1e12)
    ref = oracle(native, nx, ny, 5000, 1, per=(True, False), **kw)
    eng = native.Engine(nx, ny, periodic_x=True, boundary=1, device=gpu, ranks=[0], transport=native.TRANSPORT_RCCL,
                        **kw)
    eng.init_rccl(native.Engine.rccl_unique_id(), 1, 0)
    st = eng.run(5000)
    assert st["converged"] and st["steps_done"] == ref["steps_done"] == 219
    assert np.array_equal(eng.download(0), ref["grid"])


# ---- persistent pipelined stencil (pstream_kernel.hpp) -------------------------------------
@pytest.mark.parametrize("cols", [256, 128])
@pytest.mark.parametrize("nx,ny,K,steps,boundary", [(300, 517, 7, 37, 0), (257, 1000, 4, 41, 1), (203, 611, 1, 5, 0),
                                                    (203, 611, 3, 9, 1), (512, 4096, 8, 40, 0), (96, 300, 5, 26, 1)])
def test_persistent_kernel_bitexact(native, gpu, cols, nx, ny, K, steps, boundary):
    """Runs of equal chunks in ONE persistent launch (forced on a lone tile), both strip widths,
    NaN-poisoned ghost ring: bit-exact with the oracle, and a second run continues the progress
    words of the same plan."""
    e = native.Engine(nx, ny, tblock=K, device=gpu, small_grid_lds=False, tiled=0, persistent=1, pstream_cols=cols,
                      boundary=boundary, poison=True, halo_timeout_s=5.0)
    assert e.pstream_units(K), "no persistent plan"
    e.run(steps)
    assert e.pstream_launches() >= 1
    assert np.array_equal(e.download(0), oracle(native, nx, ny, steps, boundary)["grid"])
    e.run(steps)
    assert np.array_equal(e.download(0), oracle(native, nx, ny, 2 * steps, boundary)["grid"])


@pytest.mark.parametrize("rows,K,cols", [(512, 8, 128), (512, 8, 256), (1024, 8, 256), (300, 6, 128)])
def test_persistent_direct_row_periodic(native, gpu, rows, K, cols):
    """The per-rank shape of strong scaling through the direct pipeline with the persistent
    kernel (the auto choice for short strips): bit-exact, halo waits counted, and the chunk
    sequence continues across runs and across a convergence-free re-run."""
    steps = 5 * K + 3
    e = native.Engine(rows, 4096, periodic_x=True, tblock=K, device=gpu, ranks=[0], transport=native.TRANSPORT_IPC,
                      halo_timeout_s=5.0, pstream_cols=cols)
    e.ipc_open([e.ipc_handle()])
    e.ipc_prime()
    e.reset_halo_wait()
    e.run(steps)
    assert e.pstream_launches() >= 1
    assert np.array_equal(e.download(0), oracle(native, rows, 4096, steps, per=(True, False))["grid"])
    assert e.halo_wait()["waits"] > 0
    e.run(2 * K)
    assert np.array_equal(e.download(0), oracle(native, rows, 4096, steps + 2 * K, per=(True, False))["grid"])


def _converging_at_60(native, nx, ny, boundary=0, per=(False, False)):
    """A sensitivity between the residuals of the checks at steps 40 and 60 (check every 20)."""
    r = [oracle(native, nx, ny, s, boundary, per=per, convergence=True, interval=20, sensitivity=0.0)["residual"]
         for s in (40, 60)]
    return 0.5 * (r[0] + r[1])


@pytest.mark.parametrize("K,cols", [(6, 256), (5, 128)])
def test_persistent_fused_convergence_lone(native, gpu, K, cols):
    """The fused check with the persistent kernel forced on a lone tile: the chunks between checks
    are persistent launches (no-ops once a check converged), the pending decision is made before
    each of them; converged step and grid equal the oracle's, and so does a run that never
    converges."""
    nx, ny = 256, 1000
    for sens in (_converging_at_60(native, nx, ny, 1), 0.0):
        kw = dict(convergence=True, interval=20, sensitivity=sens)
        ref = oracle(native, nx, ny, 200, 1, **kw)
        e = native.Engine(nx, ny, boundary=1, tblock=K, device=gpu, small_grid_lds=False, tiled=0, persistent=1,
                          pstream_cols=cols, halo_timeout_s=5.0, **kw)
        st = e.run(200)
        assert e.pstream_launches() >= 1
        assert st["converged"] == ref["converged"] and st["steps_done"] == ref["steps_done"], (st, ref["steps_done"])
        assert np.array_equal(e.download(0), ref["grid"])


def test_persistent_direct_fused_convergence(native, gpu):
    """Strong scaling's per-rank shape (direct pipeline, row-periodic self-exchange) with the fused
    check every 20 steps: persistent launches between the checks, the decision through the IPC
    all-reduce; stops at the oracle's step with its grid.  After a re-prime the next run starts
    on the converged check's step and converges there again (same step, same grid)."""
    rows, K = 512, 8
    per = (True, False)
    kw = dict(convergence=True, interval=20, sensitivity=_converging_at_60(native, rows, 4096, 0, per))
    e = native.Engine(rows, 4096, periodic_x=True, tblock=K, device=gpu, ranks=[0], transport=native.TRANSPORT_IPC,
                      halo_timeout_s=5.0, pstream_cols=128, **kw)
    e.ipc_open([e.ipc_handle()])
    e.ipc_prime()
    ref = oracle(native, rows, 4096, 200, per=per, **kw)
    st = e.run(200)
    assert e.pstream_launches() >= 1
    assert st["converged"] and ref["converged"] and st["steps_done"] == ref["steps_done"], (st, ref["steps_done"])
    assert np.array_equal(e.download(0), ref["grid"])
    e.ipc_prime()
    st = e.run(2 * K)
    assert st["converged"] and st["steps_done"] == ref["steps_done"]
    assert np.array_equal(e.download(0), ref["grid"])


def test_persistent_auto_policy(native, gpu):
    """Auto: the persistent kernel only for the direct pipeline's short strips, never for a lone
    tile (there launch per chunk is faster)."""
    e = native.Engine(512, 4096, tblock=8, device=gpu, small_grid_lds=False, tiled=0)
    e.run(40)
    assert e.pstream_launches() == 0
    d = native.Engine(512, 4096, periodic_x=True, tblock=8, device=gpu, ranks=[0], transport=native.TRANSPORT_IPC,
                      halo_timeout_s=5.0)
    d.ipc_open([d.ipc_handle()])
    d.ipc_prime()
    d.run(40)
    assert d.pstream_launches() >= 1
