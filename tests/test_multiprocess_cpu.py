"""Multi-process runs on the CPU: torch.distributed (gloo) with world_size > 1.

Each rank owns one tile and exchanges its K-deep, 8-neighbour halo through
``TorchHaloExchanger`` (the engine's exchange plan); the global binary written with per-rank
pwrite must equal the single-process oracle bit for bit — the decomposition-invariance
oracle of SURVEY.md §2.9.  Launched exactly like the driver launches the bench
(``python -m torch.distributed.run --master-addr 127.0.0.1``).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def torchrun(n, args, cwd, timeout=300):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "-m", "heat2d_amd", "--device", "cpu",
           *args]
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["OMP_NUM_THREADS"] = "1"
    env["HEAT2D_NO_BUILD"] = "1"
    for _attempt in range(3):  # retry only a launcher port collision, with a fresh port
        r = subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)
        if r.returncode != 0 and "EADDRINUSE" in r.stderr:
            cmd[cmd.index("--master-port") + 1] = str(free_port())
            continue
        break
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def read_grid(path, nx, ny):
    return np.fromfile(path, dtype=np.float32).reshape(nx, ny)


@pytest.mark.parametrize("n,gx,gy,boundary", [(2, 2, 1, "fixed"), (2, 1, 2, "ghost-zero"), (4, 2, 2, "fixed"),
                                              (3, 3, 1, "ghost-zero")])
def test_gloo_ranks_match_oracle(native, tmp_path, n, gx, gy, boundary):
    nx, ny, steps = 53, 47, 37
    out = torchrun(n, ["--nx", str(nx), "--ny", str(ny), "--steps", str(steps), "--gridx", str(gx), "--gridy", str(gy),
                       "--boundary", boundary, "--output", "binary", "--outdir", str(tmp_path), "--tblock", "5"],
                   str(tmp_path))
    assert f"Starting with {n} processes" in out
    b = 0 if boundary == "fixed" else 1
    ref = native.oracle_run(nx, ny, steps, boundary=b)["grid"]
    assert np.array_equal(read_grid(tmp_path / "final_binary.dat", nx, ny), ref)
    assert np.array_equal(read_grid(tmp_path / "initial_binary.dat", nx, ny), native.init_global(nx, ny, 0))


def test_gloo_convergence_allreduce(native, tmp_path):
    nx, ny = 24, 30
    out = torchrun(2, ["--nx", str(nx), "--ny", str(ny), "--steps", "100000", "--gridx", "1", "--gridy", "2",
                       "--convergence", "1", "--interval", "7", "--sensitivity", "0.5", "--output", "binary",
                       "--outdir", str(tmp_path)], str(tmp_path))
    ref = native.oracle_run(nx, ny, 100000, convergence=True, interval=7, sensitivity=0.5)
    assert ref["converged"]
    assert f"Exiting after {ref['steps_done']} iterations" in out
    assert np.array_equal(read_grid(tmp_path / "final_binary.dat", nx, ny), ref["grid"])


@pytest.mark.parametrize("n,gx,gy", [(4, 2, 2), (2, 1, 2), (2, 2, 1)])
def test_gloo_periodic_blocks(native, tmp_path, n, gx, gy):
    """Periodic dims; a dimension one tile wide makes a rank its own neighbour."""
    nx, ny, steps = 40, 36, 21
    torchrun(n, ["--nx", str(nx), "--ny", str(ny), "--steps", str(steps), "--gridx", str(gx), "--gridy", str(gy),
                 "--periodic", "xy", "--boundary", "ghost-zero", "--output", "binary", "--outdir", str(tmp_path)],
             str(tmp_path))
    ref = native.oracle_run(nx, ny, steps, boundary=1, periodic_x=True, periodic_y=True)["grid"]
    assert np.array_equal(read_grid(tmp_path / "final_binary.dat", nx, ny), ref)


def test_gloo_heat2dn_strips_text(native, tmp_path):
    """Original-program personality on 3 ranks: 1-D strips, transposed text dump."""
    nx, ny = 16, 8
    torchrun(3, ["--preset", "heat2dn", "--nx", str(nx), "--ny", str(ny), "--outdir", str(tmp_path)], str(tmp_path))
    from heat2d_amd.utils.io import format_text

    ref = native.oracle_run(nx, ny, 100, cx=native.CX_FLOAT, cy=native.CX_FLOAT)["grid"]
    assert (tmp_path / "final.dat").read_text() == format_text(ref, "heat2dn")


def _bench(n, args, cwd):
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["HEAT2D_NO_BUILD"] = "1"
    if n == 1:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), *args]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
               "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"), *args]
    for _attempt in range(3):  # retry only a launcher port collision, with a fresh port
        r = subprocess.run(cmd, cwd=str(cwd), env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0 and "EADDRINUSE" in r.stderr and "--master-port" in cmd:
            cmd[cmd.index("--master-port") + 1] = str(free_port())
            continue
        break
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    import json

    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2, 4])
def test_bench_contract_cpu_rehearsal(tmp_path, n):
    """bench.py under torch.distributed.run: one JSON line from rank 0, whole-job value, the
    default strong-scaling config (one grid split over N), label from the actual run, the
    correctness gate and the in-job single-rank reference (speedup/efficiency, verified)."""
    d = _bench(n, ["--gpus", str(n), "--steps", "6", "--warmup", "2", "--side", "48", "--device", "cpu"], tmp_path)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "speedup", "efficiency"):
        assert k in d
    assert d["n_gpus"] == n and d["steps"] == 6 and d["scaling"] == "strong"
    assert d["config"]["grid"] == [48, 48] and d["config"]["grid_per_gpu"] == [48 // n, 48]
    assert d["metric"] == "cell-updates/sec (whole node) + speedup/efficiency, 48^2 grid 6 steps"
    assert d["config"]["parallelism"] == ("single" if n == 1 else f"rows{n}")
    # short per-rank tiles (<= 1024 rows) at N > 1: depth 8 (the persistent kernel's best), else 7
    assert d["config"]["tblock"] == (8 if n > 1 else 7)
    assert abs(d["value"] - 48 * 48 * 6 / d["elapsed_s"]) / d["value"] < 1e-9
    assert abs(d["efficiency"] - d["speedup"] / n) < 1e-12
    if n > 1:
        assert d["verified"] is True  # every rank's tile == the single-rank grid, bit for bit
        assert d["gate"][0]["ok"] and d["config"]["transport"] == "torch"
    else:
        assert d["speedup"] == 1.0 and d["gate"] is None


def test_bench_weak_and_blocks_cpu_rehearsal(tmp_path):
    d = _bench(4, ["--gpus", "4", "--steps", "5", "--warmup", "1", "--config", "weak-4096", "--side", "40",
                   "--layout", "blocks", "--device", "cpu"], tmp_path)
    assert d["scaling"] == "weak" and d["config"]["grid"] == [80, 80] and d["config"]["grid_per_gpu"] == [40, 40]
    assert d["config"]["parallelism"] == "blocks2x2"
    # the timed solver's first 5 steps were checked against the CPU oracle on the whole 80x80 grid
    assert d["verified"] is True and "CPU oracle" in d["verification"]
    assert abs(d["speedup"] - 4 * d["efficiency"]) < 1e-12


def test_bench_weak_hbm_efficiency_cpu_rehearsal(tmp_path):
    """weak-hbm at N=4: the single-rank reference tile is timed before the N-rank solver
    allocates (on a GPU both would not fit), so speedup and efficiency are reported."""
    d = _bench(4, ["--gpus", "4", "--steps", "4", "--warmup", "1", "--config", "weak-hbm", "--device", "cpu"], tmp_path)
    assert d["scaling"] == "weak" and d["config"]["grid_per_gpu"] == [64, 64]
    assert d["efficiency"] is not None and d["efficiency"] > 0 and abs(d["speedup"] - 4 * d["efficiency"]) < 1e-12
    assert "before the N-rank solver" in d["speedup_reference"]


def test_bench_gate_all_candidates_fail_cpu(tmp_path):
    """Every transport fails the gate: rank 0 prints an error record naming what was tried and
    the job exits non-zero instead of timing an unverified configuration."""
    env = dict(os.environ, HEAT2D_NO_BUILD="1", HEAT2D_GATE_FAIL="torch")
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
           "4", "--warmup", "1", "--side", "32", "--device", "cpu"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    import json

    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["error"] == "no transport passed the correctness gate"
    assert rec["gate"][0]["transport"] == "torch" and not rec["gate"][0]["ok"]
    assert "HEAT2D_GATE_FAIL" in rec["gate"][0]["detail"]


@pytest.mark.parametrize("config,label", [("4096-strong", "rows8"), ("16384x8blocks", "blocks2x4")])
def test_bench_eight_ranks_cpu_rehearsal(tmp_path, config, label):
    """The driver's N=8 SCALE run, rehearsed on the host: 8 ranks under torch.distributed.run
    (gloo), the BASELINE headline (4096^2 as 1-D row strips) and config 4 (2x4 blocks) at a small
    side — one JSON line, the gate passed, every rank's tile == the single-rank grid."""
    d = _bench(8, ["--gpus", "8", "--steps", "4", "--warmup", "1", "--side", "64", "--config", config,
                   "--device", "cpu"], tmp_path)
    assert d["n_gpus"] == 8 and d["steps"] == 4 and d["scaling"] == "strong"
    assert d["config"]["parallelism"] == label and d["config"]["grid"] == [64, 64]
    assert d["verified"] is True and d["gate"][0]["ok"]
    assert abs(d["efficiency"] - d["speedup"] / 8) < 1e-12
