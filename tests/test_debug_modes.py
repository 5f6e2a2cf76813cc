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
    # signalled pipeline: one launch per chunk; serial pipeline: exchange, then the chunk's step
    main = "chunk" if eng.pipeline() == "signal" else "step"
    assert {main, "exchange"} <= set(ph), ph
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


ENGINE_SAN_DRIVER = r"""
#include <cstdio>
#include <cstring>
#include <vector>
#include "cpu_reference.h"
#include "decomposition.h"
#include "engine.h"
#include "kernels.h"
using namespace h2d;
static int check_engine(int64_t nx, int64_t ny, int gx, int gy, int K, int boundary, bool px, bool py, bool conv) {
  EngineOptions o;
  o.nx = nx; o.ny = ny; o.gridx = gx; o.gridy = gy; o.tblock = K; o.boundary = boundary;
  o.periodic_x = px; o.periodic_y = py; o.device = -1; o.convergence = conv; o.interval = 6; o.sensitivity = 1e-30;
  o.poison = true;
  Engine e(o);
  RunStats st = e.run(29);
  st = e.run(8);  // a second run continues the chunk schedule
  Physics ph; ph.boundary = boundary; ph.periodic_x = px; ph.periodic_y = py;
  OracleResult r = oracle_run(nx, ny, 37, ph, kInitExact, conv, 6, 1e-30, nullptr);
  for (int t = 0; t < e.num_tiles(); ++t) {
    const TileGeom g = e.geom(t);
    std::vector<float> b = e.download(t);
    for (int64_t i = 0; i < g.xcell; ++i)
      if (std::memcmp(&b[i * g.ycell], &r.grid[(g.gx0 + i) * ny + g.gy0], g.ycell * sizeof(float))) return 1;
  }
  return st.steps_done == 37 ? 0 : 2;
}
int main() {
  int bad = 0;
  bad += check_engine(41, 37, 3, 2, 5, kFixed, false, false, false);
  bad += check_engine(30, 44, 2, 2, 4, kGhostZero, true, true, true);
  bad += check_engine(25, 19, 1, 3, 3, kGhostZero, false, true, false);
  // the unit planner (host code shared with the GPU path)
  for (int K : {1, 4, 8, 16}) {
    for (int64_t nx : {1, 9, 100, 513}) for (int64_t ny : {1, 255, 256, 700, 4096}) {
      TileGeom g = make_tile_geom(nx, ny, 0, 0, nx, ny, K);
      bool peer[kNumDirs] = {true, true, false, false, false, false, false, false};
      for (int64_t cap : {1, 64, 1024}) {
        UnitPlan p = plan_units(g, K, 0, true, false, false, 1.2, cap, peer, 8);
        std::vector<Unit> u = build_units(g, K, 0, false, true, false, 1.0, cap);
        int64_t rows = 0;
        for (const Unit& x : u) rows += x.h;
        std::vector<Strip> s = strip_layout(g, K, true, false);
        if (rows != nx * (int64_t)strip_layout(g, K, false, false).size()) bad += 100;
        (void)p; (void)s;
      }
    }
  }
  std::printf("ok %d\n", bad);
  return bad;
}
"""


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
def test_host_sanitizers_engine_cpu_path(native, tmp_path):
    """The engine's CPU path (chunk scheduler, local halo plans, poison canary, convergence) and
    the work-unit planner under ASan + UBSan, with every -fsanitize= behind -Xarch_host (host
    code only; nothing runs on a GPU: the engine is created with device = -1).  The heavy
    stencil translation units (device code only, unchanged) are linked from the regular build."""
    import concurrent.futures as cf

    from heat2d_amd import _build

    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    csrc = os.path.join(ROOT, "heat2d_amd", "csrc")
    drv = tmp_path / "engine_san.cpp"
    drv.write_text(ENGINE_SAN_DRIVER)
    srcs = [str(drv)] + [os.path.join(csrc, f) for f in ("engine.cpp", "decomposition.cpp", "cpu_reference.cpp",
                                                          "kernels.hip")]
    prebuilt = [_build._obj_for(f) for f in ["tile_kernel.hip"] + list(_build.GEN_TUS)]
    assert all(os.path.exists(o) for o in prebuilt)
    flags = ["-x", "hip", "--offload-arch=gfx950", "-std=c++17", "-O1", "-ffp-contract=off", f"-I{csrc}",
             "-Xarch_host", "-g", "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
             "-Xarch_host", "-fno-sanitize-recover=all", "-Xarch_host", "-fno-omit-frame-pointer"]

    def compile_one(src):
        obj = str(tmp_path / (os.path.basename(src) + ".o"))
        r = subprocess.run([hipcc, *flags, "-c", src, "-o", obj], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-3000:]
        return obj

    with cf.ThreadPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, srcs))
    exe = str(tmp_path / "engine_san")
    r = subprocess.run([hipcc, "--offload-arch=gfx950", "-fno-gpu-sanitize", "-fsanitize=address,undefined", *objs, *prebuilt, "-o", exe,
                        "-L/opt/rocm/lib", "-lrccl", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and r.stdout.startswith("ok 0"), r.stdout[-2000:] + r.stderr[-4000:]


def test_kernel_arguments_default_to_host_memory():
    """Importing heat2d_amd selects host-memory kernel arguments for the HIP runtime unless the
    user chose (docs/ARCHITECTURE.md, "Kernel arguments (round 5)"), and records the
    effective state; the CLI does the same, and bench.py runs the library default (no override of
    its own), so the bench times what the tests run.  A fresh interpreter, so the setting is seen
    before anything initialises the GPU."""
    import subprocess
    import sys

    code = "import os, heat2d_amd; print(os.environ['HIP_FORCE_DEV_KERNARG'], heat2d_amd.KERNARG_HOST_MEMORY)"
    env = {k: v for k, v in os.environ.items() if k != "HIP_FORCE_DEV_KERNARG"}
    env["HEAT2D_NO_BUILD"] = "1"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True, check=True)
    assert out.stdout.split()[-2:] == ["0", "True"]
    env["HIP_FORCE_DEV_KERNARG"] = "1"  # the user's choice is kept
    out = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True, check=True)
    assert out.stdout.split()[-2:] == ["1", "False"]
    assert "device-memory kernel arguments" in out.stderr  # ... with a warning
    with open(os.path.join(root, "bench.py")) as fh:
        assert "HIP_FORCE_DEV_KERNARG" not in fh.read()
    with open(os.path.join(root, "heat2d_amd", "csrc", "heat2d_main.cpp")) as fh:
        assert 'setenv("HIP_FORCE_DEV_KERNARG", "0", 0)' in fh.read()
