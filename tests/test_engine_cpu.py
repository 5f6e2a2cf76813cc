"""CPU tests of the native runtime: oracle vs an independent numpy implementation, the
decomposition / exchange plan, and the engine (temporal blocking + deep halos) vs the oracle
for many decompositions — decomposition invariance is the strongest oracle."""
import numpy as np
import pytest

from tests import oracle_numpy as onp


def test_update_ref_matches_numpy(native):
    rng = np.random.default_rng(0)
    v = rng.standard_normal((1000, 5)).astype(np.float32) * np.float32(1e3)
    for c, n_, s, w, e in v[:200]:
        sn = np.float32(s + n_)
        ew = np.float32(e + w)
        r = np.float64(c) + 0.1 * (np.float64(sn) - 2.0 * np.float64(c))
        r = r + 0.1 * (np.float64(ew) - 2.0 * np.float64(c))
        assert native.update_ref(float(c), float(n_), float(s), float(w), float(e), 0.1, 0.1) == np.float32(r)


@pytest.mark.parametrize("mode", ["exact", "ref-int32"])
@pytest.mark.parametrize("nx,ny", [(10, 10), (640, 512), (97, 1031)])
def test_init_matches_numpy(native, mode, nx, ny):
    m = {"exact": 0, "ref-int32": 1}[mode]
    assert np.array_equal(native.init_global(nx, ny, m), onp.init_field(nx, ny, mode))


def test_int32_center_value_4096(native):
    # the wrapped centre at 4096^2 is 4 194 304, the exact one 1.7575e13.
    assert native.init_value(1, 2048, 2048, 4096, 4096) == 4194304.0
    assert abs(native.init_value(0, 2048, 2048, 4096, 4096) - 1.7575e13) / 1.7575e13 < 1e-3


@pytest.mark.parametrize("boundary", ["fixed", "ghost-zero"])
@pytest.mark.parametrize("per", [(False, False), (True, False), (False, True), (True, True)])
def test_oracle_vs_numpy(native, boundary, per):
    nx, ny, steps = 23, 31, 40
    b = 0 if boundary == "fixed" else 1
    r = native.oracle_run(nx, ny, steps, boundary=b, periodic_x=per[0], periodic_y=per[1])
    assert np.array_equal(r["grid"], onp.run(nx, ny, steps, boundary, periodic=per))


def test_decomposition_uneven_split(native):
    d = native.Decomposition(10, 7, 3, 2)
    assert d.xcount == [4, 3, 3] and d.xstart == [0, 4, 7]
    assert d.ycount == [4, 3]
    # grad1612_mpi_heat.c:125-138 / MPI_Cart_shift: rank = py*GRIDX + px
    assert d.px_of(4) == 1 and d.py_of(4) == 1
    assert d.neighbor(0, 0) == -1 and d.neighbor(0, 1) == 1 and d.neighbor(0, 3) == 3


def test_plans_match_pairwise(native):
    for gx, gy, px, py in [(2, 2, False, False), (3, 4, True, False), (2, 1, True, True), (1, 1, True, True)]:
        d = native.Decomposition(50, 61, gx, gy, px, py)
        G = 4
        plans = [d.plan(r, G, 3) for r in range(d.nranks())]
        opp = native.DIR_OPP
        for r in range(d.nranks()):
            for k, e in enumerate(plans[r]):
                if e["peer"] < 0:
                    continue
                q = plans[e["peer"]][opp[k]]
                assert q["peer"] == r
                assert e["send"][2:] == q["recv"][2:], (gx, gy, r, k)


def test_auto_grid():
    from heat2d_amd.config import auto_grid

    assert auto_grid(1) == (1, 1) and auto_grid(2) == (1, 2) and auto_grid(4) == (2, 2) and auto_grid(8) == (2, 4)


def gather(eng, nx, ny):
    out = np.zeros((nx, ny), np.float32)
    for t in range(eng.num_tiles()):
        g = eng.geom(t)
        out[g["gx0"]:g["gx0"] + g["xcell"], g["gy0"]:g["gy0"] + g["ycell"]] = eng.download(t)
    return out


@pytest.mark.parametrize("gx,gy", [(1, 1), (1, 2), (2, 1), (2, 2), (2, 4), (4, 2), (3, 3)])
@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("tblock", [1, 3, 8])
def test_cpu_engine_decomposition_invariance(native, gx, gy, boundary, tblock):
    nx, ny, steps = 37, 45, 29
    eng = native.Engine(nx, ny, gridx=gx, gridy=gy, boundary=boundary, tblock=tblock, device=-1)
    st = eng.run(steps)
    assert st["steps_done"] == steps
    assert np.array_equal(gather(eng, nx, ny), native.oracle_run(nx, ny, steps, boundary=boundary)["grid"])


def test_cpu_engine_periodic(native):
    nx, ny, steps = 30, 22, 33
    eng = native.Engine(nx, ny, gridx=2, gridy=3, periodic_x=True, periodic_y=True, boundary=1, device=-1)
    eng.run(steps)
    ref = native.oracle_run(nx, ny, steps, boundary=1, periodic_x=True, periodic_y=True)["grid"]
    assert np.array_equal(gather(eng, nx, ny), ref)


@pytest.mark.parametrize("interval", [1, 7, 20])
def test_cpu_convergence_semantics(native, interval):
    nx, ny = 20, 20
    kw = dict(convergence=True, interval=interval, sensitivity=0.5)
    ref = native.oracle_run(nx, ny, 100000, **kw)
    assert ref["converged"]
    # committed count is a multiple of the interval minus one (the checked step is discarded)
    assert (ref["steps_done"] + 1) % interval == 0
    plain = native.oracle_run(nx, ny, ref["steps_done"])["grid"]
    assert np.array_equal(plain, ref["grid"])
    eng = native.Engine(nx, ny, gridx=2, gridy=2, device=-1, **kw)
    st = eng.run(100000)
    assert st["converged"] and st["steps_done"] == ref["steps_done"]
    assert np.array_equal(gather(eng, nx, ny), ref["grid"])


def test_resume_equals_uninterrupted(native):
    nx, ny = 33, 40
    e1 = native.Engine(nx, ny, device=-1)
    e1.run(17)
    e1.run(13)
    assert np.array_equal(e1.download(0), native.oracle_run(nx, ny, 30)["grid"])
    mid = native.oracle_run(nx, ny, 17)["grid"]
    e2 = native.Engine(nx, ny, init=native.INIT_ZERO, device=-1)
    e2.upload(0, mid)
    e2.run(13)
    assert np.array_equal(e2.download(0), native.oracle_run(nx, ny, 30)["grid"])


@pytest.mark.parametrize("n,cap", [(37, 1024), (4096, 1024), (4096, 2048), (16384, 1024), (180000, 1024)])
def test_unit_planner_covers_rows_and_packs_rounds(native, n, cap):
    K = 8
    units = native.unit_plan(n, n, K, 0, True, False, False, 1.2, cap)
    strips = native.strip_layout(n, n, K, True, False)
    nstrips = len(strips)
    # output columns tile [0, n) without overlap; windows stay inside the padded row
    R, pos = native.lead_cols(K), 0
    for cb, lo, hi in strips:
        assert lo == pos and hi > lo and cb % 4 == 0
        assert cb + R <= lo or cb == 0  # left cone inside the window (or edge-aligned)
        assert hi <= cb + 256 - R or cb + 256 >= n  # right cone inside the window (or edge-aligned)
        pos = hi
    assert pos == n
    if n == 4096:
        assert nstrips == 17  # 248 + 15 x 240 + 248
    rows = {}
    for s, x0, h, flags in units:
        rows.setdefault(s, []).append((x0, h))
    assert sorted(rows) == list(range(nstrips))
    for s, segs in rows.items():
        segs.sort()
        pos = 0
        for x0, h in segs:
            assert x0 == pos and h >= 1
            pos += h
        assert pos == n
    # one full round when possible, otherwise nearly-full rounds
    rounds = -(-len(units) // cap)
    assert len(units) <= cap or len(units) / (rounds * cap) > 0.9


def test_unit_planner_sizes_corner_units_by_their_cost(native):
    """A corner unit (row- and column-masked body) costs more per row than a column-edge unit
    (profiles/unit_balance_r5.md: it was the launch's last wave when sized like one): the planner
    gives it fewer rows, and every unit class stays within one resident round."""
    for n in (4096, 2048):
        units = native.unit_plan(n, 4096, 7, 0, True, False, False, 1.16, 1024)
        assert len(units) <= 1024
        by = {}
        for _s, _x0, h, flags in units:
            by.setdefault(flags & 3, []).append(h)
        assert set(by) == {0, 1, 2, 3}, sorted(by)
        assert max(by[3]) < min(by[1]) < min(by[0])  # corner < column edge < plain
        assert max(by[2]) < min(by[0])  # row edge < plain
