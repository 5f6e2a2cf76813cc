"""Debug / race-detection subsystems:

* halo canary — every storage cell that no valid update may read (padding, fixed-mode ghost
  cells outside the grid, and ghost cells inside the grid before the first exchange) is
  NaN-poisoned; results must stay bit-identical.  This checks the dependency-cone argument
  of the temporally-blocked kernel and the completeness of the halo exchange.
* host sanitizers — the CPU runtime built with -fsanitize=address,undefined runs the oracle,
  the decomposition/plans and the CPU engine without a report.
* phase tracing — per-phase hipEvent timers.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def gather(eng, nx, ny):
    out = np.zeros((nx, ny), np.float32)
    for t in range(eng.num_tiles()):
        g = eng.geom(t)
        out[g["gx0"]:g["gx0"] + g["xcell"], g["gy0"]:g["gy0"] + g["ycell"]] = eng.download(t)
    return out


@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("gx,gy", [(1, 1), (2, 3)])
def test_poison_canary_cpu(native, boundary, gx, gy):
    nx, ny, steps = 29, 38, 23
    eng = native.Engine(nx, ny, gridx=gx, gridy=gy, boundary=boundary, tblock=5, device=-1, poison=True)
    eng.run(steps)
    assert np.array_equal(gather(eng, nx, ny), native.oracle_run(nx, ny, steps, boundary=boundary)["grid"])


@pytest.mark.gpu
@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("gx,gy,K", [(1, 1, 8), (1, 1, 3), (2, 1, 8), (2, 2, 6), (3, 2, 4)])
def test_poison_canary_gpu(native, gpu, boundary, gx, gy, K):
    nx, ny, steps = 301, 517, 37  # ny % 4 != 0: partial-lane stores at the east edge
    eng = native.Engine(nx, ny, gridx=gx, gridy=gy, boundary=boundary, tblock=K, device=gpu, poison=True,
                        small_grid_lds=False, tiled=0)
    eng.run(steps)
    assert np.array_equal(gather(eng, nx, ny), native.oracle_run(nx, ny, steps, boundary=boundary)["grid"])


@pytest.mark.gpu
def test_poison_canary_rccl_self(native, gpu):
    nx, ny, steps = 200, 300, 29
    eng = native.Engine(nx, ny, periodic_x=True, periodic_y=True, boundary=1, device=gpu, ranks=[0],
                        transport=native.TRANSPORT_RCCL, poison=True)
    eng.init_rccl(native.Engine.rccl_unique_id(), 1, 0)
    eng.run(steps)
    ref = native.oracle_run(nx, ny, steps, boundary=1, periodic_x=True, periodic_y=True)["grid"]
    assert np.array_equal(eng.download(0), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("signal_exchange", [-1, 0])
def test_phase_trace(native, gpu, signal_exchange):
    eng = native.Engine(512, 1024, gridx=2, device=gpu, trace=True, signal_exchange=signal_exchange)
    st = eng.run(40)
    ph = st["phase_ms"]
    # signalled pipeline: one launch per chunk; split pipelines: interior + boundary launches
    main = "chunk" if eng.pipeline() == "signal" else "interior"
    assert ({"chunk", "exchange"} if main == "chunk" else {"boundary", "interior", "exchange"}) <= set(ph), ph
    assert all(v >= 0 for v in ph.values())
    assert st["phase_count"][main] == st["chunks"]


SAN_DRIVER = r"""
#include <cstdio>
#include <vector>
#include "cpu_reference.h"
#include "decomposition.h"
#include "io.h"
using namespace h2d;
int main() {
  Physics ph;
  OracleResult r = oracle_run(33, 21, 40, ph, kInitInt32, true, 7, 0.5);
  ph.boundary = kGhostZero; ph.periodic_x = true;
  r = oracle_run(17, 45, 25, ph, kInitExact, false, 20, 0.1);
  Decomposition d(50, 61, 3, 4, true, false);
  for (int rank = 0; rank < d.nranks(); ++rank) {
    TileGeom g = d.tile(rank, 4);
    ExchangePlan p = make_plan(d, rank, g, 3);
    std::vector<float> a(g.elems()), b(g.elems()), s0(g.elems()), s1(g.elems()), sb(p.send_total + 1);
    cpu_tile_init(g, a.data(), kInitExact);
    std::vector<CopyDesc> v;
    plan_pack_descs(p, g, a.data(), sb.data(), v);
    cpu_copy_rects(v);
    cpu_tile_advance(g, ph, a.data(), b.data(), 3, s0.data(), s1.data(), true);
  }
  std::string t = format_text(r.grid.data(), 17, 45, kTextHeat2dn);
  std::printf("ok %zu\n", t.size());
  return 0;
}
"""


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_host_sanitizers(tmp_path):
    src = tmp_path / "san.cpp"
    src.write_text(SAN_DRIVER)
    csrc = os.path.join(ROOT, "heat2d_amd", "csrc")
    exe = tmp_path / "san"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-ffp-contract=off", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", f"-I{csrc}", str(src), os.path.join(csrc, "cpu_reference.cpp"),
           os.path.join(csrc, "decomposition.cpp"), os.path.join(csrc, "io.cpp"), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
