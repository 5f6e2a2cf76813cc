"""Command-line programs: the Python CLI (``python -m heat2d_amd``) and the native ``heat2d``
executable must produce byte-identical outputs and banners (elapsed time aside), for every
preset; checkpoint/resume must equal an uninterrupted run."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "heat2d_amd", "bin", "heat2d")


def py_cli(outdir, *args):
    r = subprocess.run([sys.executable, "-m", "heat2d_amd", "--device", "cpu", "--outdir", str(outdir), *args],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout


def native_cli(outdir, *args):
    r = subprocess.run([NATIVE, "--device", "cpu", "--outdir", str(outdir), *args], cwd=ROOT, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout


def strip_elapsed(s):
    return re.sub(r"Elapsed time: \S+ sec", "Elapsed time: X sec", s)


CASES = [
    ("grad_mpi",),
    ("heat2dn", "--gridx", "3", "--nx", "16", "--ny", "8"),
    ("grad_hybrid", "--nx", "24", "--ny", "30", "--steps", "5000", "--sensitivity", "0.5", "--interval", "7"),
    ("heat2d", "--nx", "33", "--ny", "47", "--steps", "60", "--gridx", "2", "--gridy", "3", "--init", "ref-int32"),
    ("cuda", "--nx", "64", "--ny", "96", "--steps", "50"),
]


@pytest.mark.skipif(not os.path.exists(NATIVE), reason="native CLI not built")
@pytest.mark.parametrize("case", CASES, ids=lambda c: c[0])
def test_native_equals_python_cli(tmp_path, case):
    a, b = tmp_path / "native", tmp_path / "py"
    args = ["--preset", *case]
    out_n = native_cli(a, *args)
    out_p = py_cli(b, *args)
    assert strip_elapsed(out_n) == strip_elapsed(out_p)
    files_n = sorted(os.listdir(a)) if a.exists() else []
    files_p = sorted(os.listdir(b)) if b.exists() else []
    assert files_n == files_p
    for f in files_n:
        assert (a / f).read_bytes() == (b / f).read_bytes(), f


def test_hybrid_and_cuda_banners(tmp_path):
    out = py_cli(tmp_path, "--preset", "grad_hybrid", "--steps", "10", "--output", "none")
    assert out.startswith("Starting with 1 processes and 4 threads\nProblem size:10x10\n")
    assert "Check for convergence every 20 iterations\n" in out
    out = py_cli(tmp_path, "--preset", "cuda", "--nx", "16", "--ny", "32", "--steps", "4")
    assert re.fullmatch(r"Problem size: 16x32\nAmount of iterations: 4\nElapsed time: \S+ sec\n", out)


def test_checkpoint_resume(native, tmp_path):
    nx, ny = 40, 56
    ck = tmp_path / "ck.bin"
    py_cli(tmp_path / "a", "--nx", str(nx), "--ny", str(ny), "--steps", "30", "--output", "none", "--save", str(ck))
    py_cli(tmp_path / "b", "--nx", str(nx), "--ny", str(ny), "--steps", "25", "--load", str(ck), "--start-step", "30",
           "--output", "binary", "--gridx", "2")
    got = np.fromfile(tmp_path / "b" / "final_binary.dat", np.float32).reshape(nx, ny)
    assert np.array_equal(got, native.oracle_run(nx, ny, 55)["grid"])


def test_json_metrics_line(tmp_path):
    import json

    out = py_cli(tmp_path, "--nx", "30", "--ny", "30", "--steps", "20", "--output", "none", "--json", "--quiet")
    d = json.loads(out.strip().splitlines()[-1])
    assert d["grid"] == [30, 30] and d["steps"] == 20 and d["cell_updates_per_s"] > 0


MULTI = [
    (4, ("--preset", "grad_mpi", "--nx", "41", "--ny", "37", "--steps", "29")),
    (3, ("--preset", "heat2dn", "--gridx", "3", "--nx", "16", "--ny", "8")),
    (3, ("--nx", "53", "--ny", "47", "--steps", "37", "--gridx", "3", "--gridy", "1", "--tblock", "5")),
    (4, ("--nx", "40", "--ny", "36", "--steps", "21", "--gridx", "2", "--gridy", "2", "--periodic", "xy",
         "--boundary", "ghost-zero")),
    (2, ("--preset", "grad_hybrid", "--gridx", "1", "--gridy", "2", "--nx", "24", "--ny", "30", "--steps", "5000",
         "--sensitivity", "0.5", "--interval", "7")),
]


@pytest.mark.skipif(not os.path.exists(NATIVE), reason="native CLI not built")
@pytest.mark.parametrize("np_,args", MULTI, ids=lambda x: str(x) if isinstance(x, int) else x[1])
def test_native_multirank_equals_single_process(tmp_path, np_, args):
    """`heat2d --np P` (the native mpiexec: P forked ranks, TCP bootstrap, per-rank binary
    writes, max-over-ranks timing) gives the same outputs and banners as one process with all
    tiles, byte for byte."""
    a, b = tmp_path / "multi", tmp_path / "single"
    a.mkdir()
    b.mkdir()
    out_m = native_cli(a, "--np", str(np_), *args)
    out_s = native_cli(b, *args)
    assert strip_elapsed(out_m) == strip_elapsed(out_s)
    files = sorted(os.listdir(b))
    assert files and files == sorted(os.listdir(a))
    for f in files:
        assert (a / f).read_bytes() == (b / f).read_bytes(), f


@pytest.mark.skipif(not os.path.exists(NATIVE), reason="native CLI not built")
def test_native_under_torchrun_no_python(tmp_path):
    """The native executable launched like the reference (`mpiexec -n P ./binary`) by
    torch.distributed.run --no-python: ranks from RANK / WORLD_SIZE / MASTER_ADDR."""
    from tests.test_multiprocess_cpu import free_port

    args = ["--device", "cpu", "--nx", "45", "--ny", "33", "--steps", "23", "--gridx", "3", "--gridy", "1",
            "--output", "binary", "--outdir", str(tmp_path), "--json"]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "--no-python", NATIVE, *args],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert '"ranks": 3' in r.stdout
    from heat2d_amd._native import native

    ref = native().oracle_run(45, 33, 23)["grid"]
    got = np.fromfile(tmp_path / "final_binary.dat", dtype=np.float32).reshape(45, 33)
    assert np.array_equal(got, ref)
