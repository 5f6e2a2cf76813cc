"""Golden tests against the reference programs themselves.

The reference C sources are compiled into a private temp directory by a fixture (MPICH from
/opt/conda, the recipe of SURVEY.md Appendix A) — never vendored, never modified in place —
and run as an external oracle.  Our CLI must reproduce their outputs byte for byte:
  * grad1612_mpi_heat.c  (ghost-zero boundary, double CX, row-major text, raw binaries)
  * mpi_heat2Dn.c        (fixed boundary, float cx, transposed text)
Skipped when no MPI toolchain is present.
"""
import os
import re
import shutil
import subprocess
import sys

import numpy as np
import pytest

REF = "/root/reference"
CONDA = "/opt/conda/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(
    not (os.path.exists(os.path.join(CONDA, "mpicc")) and os.path.isdir(REF)), reason="no MPI toolchain / reference")


def _env():
    e = dict(os.environ)
    e["PATH"] = CONDA + ":" + e.get("PATH", "")
    e["MPICH_CC"] = "gcc"
    return e


_WORKER_MSG = re.compile(r"Task \d+ received work\. Beginning time steps\.\.\.")


def _banner_signature(text):
    from collections import Counter

    text = _strip_elapsed(text)
    workers = Counter(_WORKER_MSG.findall(text))
    return workers, Counter(_WORKER_MSG.sub(" ", text).split())


def _variant(src, dst, defs):
    text = open(os.path.join(REF, src)).read()
    for k, v in defs.items():
        text, n = re.subn(r"^#define %s\s+.*$" % k, "#define %s %s" % (k, v), text, flags=re.M)
        assert n == 1, k
    open(dst, "w").write(text)


@pytest.fixture(scope="module")
def refdir(tmp_path_factory):
    return tmp_path_factory.mktemp("refbuild")


def build_and_run(refdir, src, name, defs, nproc, extra_flags=()):
    d = os.path.join(str(refdir), name)
    os.makedirs(d, exist_ok=True)
    c = os.path.join(d, name + ".c")
    _variant(src, c, defs)
    exe = os.path.join(d, name)
    subprocess.run([os.path.join(CONDA, "mpicc"), "-g", "-Wall", *extra_flags, "-o", exe, c], check=True, env=_env(),
                   capture_output=True)
    r = subprocess.run([os.path.join(CONDA, "mpiexec"), "-n", str(nproc), exe], cwd=d, env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return d, r.stdout


def run_ours(outdir, *args):
    r = subprocess.run([sys.executable, "-m", "heat2d_amd", "--device", "cpu", "--outdir", outdir, *args], cwd=ROOT,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    return r.stdout


def _strip_elapsed(s):
    return re.sub(r"Elapsed time: \S+ sec", "Elapsed time: X sec", s)


def _read(p):
    return open(p, "rb").read()


@pytest.mark.parametrize("nx,ny,steps", [(10, 10, 100), (16, 8, 100), (80, 64, 50)])
def test_grad_mpi_single_rank_bitexact(refdir, tmp_path, nx, ny, steps):
    d, out = build_and_run(refdir, "grad1612_mpi_heat.c", f"grad_{nx}x{ny}",
                           {"NXPROB": nx, "NYPROB": ny, "STEPS": steps, "GRIDX": 1, "GRIDY": 1}, 1)
    ours = run_ours(str(tmp_path), "--preset", "grad_mpi", "--nx", str(nx), "--ny", str(ny), "--steps", str(steps),
                    "--gridx", "1", "--gridy", "1", "--init", "ref-int32")
    for f in ("initial_binary.dat", "final_binary.dat", "initial.dat", "final.dat"):
        assert _read(os.path.join(d, f)) == _read(os.path.join(str(tmp_path), f)), f
    assert _strip_elapsed(out) == _strip_elapsed(ours)


def test_grad_mpi_multirank_matches_single_rank_reference(refdir, tmp_path):
    """Reference 4×2 ranks: its initial binary is right, its final binary is corrupt (B-3);
    ours (4×2 tiles) must equal the reference's *single-rank* final state."""
    nx, ny, steps = 16, 8, 100
    d1, _ = build_and_run(refdir, "grad1612_mpi_heat.c", "grad_16x8_1",
                          {"NXPROB": nx, "NYPROB": ny, "STEPS": steps, "GRIDX": 1, "GRIDY": 1}, 1)
    d8, out8 = build_and_run(refdir, "grad1612_mpi_heat.c", "grad_16x8_8",
                             {"NXPROB": nx, "NYPROB": ny, "STEPS": steps, "GRIDX": 4, "GRIDY": 2}, 8)
    ours = run_ours(str(tmp_path), "--preset", "grad_mpi", "--nx", str(nx), "--ny", str(ny), "--steps", str(steps),
                    "--gridx", "4", "--gridy", "2", "--init", "ref-int32")
    assert _read(os.path.join(d8, "initial_binary.dat")) == _read(os.path.join(str(tmp_path), "initial_binary.dat"))
    assert _read(os.path.join(d1, "final_binary.dat")) == _read(os.path.join(str(tmp_path), "final_binary.dat"))
    assert _read(os.path.join(d8, "final_binary.dat")) != _read(os.path.join(str(tmp_path), "final_binary.dat"))
    assert _strip_elapsed(out8) == _strip_elapsed(ours)


def test_grad_int32_overflow_init(refdir, tmp_path):
    """640×512: the reference's int32 product wraps (B-1); --init ref-int32 reproduces it."""
    nx, ny, steps = 640, 512, 3
    d, _ = build_and_run(refdir, "grad1612_mpi_heat.c", "grad_640x512",
                         {"NXPROB": nx, "NYPROB": ny, "STEPS": steps, "GRIDX": 1, "GRIDY": 1}, 1)
    run_ours(str(tmp_path), "--preset", "grad_mpi", "--nx", str(nx), "--ny", str(ny), "--steps", str(steps),
             "--gridx", "1", "--gridy", "1", "--init", "ref-int32", "--output", "binary")
    a = np.fromfile(os.path.join(d, "initial_binary.dat"), np.float32)
    b = np.fromfile(os.path.join(str(tmp_path), "initial_binary.dat"), np.float32)
    assert (a < 0).any(), "reference field should contain wrapped (negative) cells"
    assert np.array_equal(a, b)
    assert _read(os.path.join(d, "final_binary.dat")) == _read(os.path.join(str(tmp_path), "final_binary.dat"))


@pytest.mark.parametrize("nx,ny,nproc", [(10, 10, 4), (16, 8, 4), (80, 64, 5)])
def test_original_heat2dn_text_exact(refdir, tmp_path, nx, ny, nproc):
    d, out = build_and_run(refdir, "mpi_heat2Dn.c", f"orig_{nx}x{ny}", {"NXPROB": nx, "NYPROB": ny, "STEPS": 100},
                           nproc)
    workers = nproc - 1
    ours = run_ours(str(tmp_path), "--preset", "heat2dn", "--nx", str(nx), "--ny", str(ny), "--gridx", str(workers),
                    "--init", "ref-int32")
    for f in ("initial.dat", "final.dat"):
        assert _read(os.path.join(d, f)) == _read(os.path.join(str(tmp_path), f)), f
    # Banner text.  The reference's workers print concurrently with the master, and a worker
    # message can land in the middle of a master line, so compare the worker messages as a
    # multiset and the remaining text as a multiset of tokens.
    assert _banner_signature(out) == _banner_signature(ours)
