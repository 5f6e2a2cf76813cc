"""Multi-process runs on one MI355X: several ranks share the card through the ``host``
transport (gloo point-to-point with pinned host staging; RCCL refuses two ranks on one
device).  This rehearses the one-process-per-GPU path the bench uses at N > 1 — rank
device selection, per-rank tiles, timed loop with barrier + max over ranks, collective
binary output, JSON contract — everything except the RCCL wire itself (covered by the
RCCL self-exchange tests in ``test_gpu_engine.py``).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from tests.test_multiprocess_cpu import ROOT, free_port, read_grid

pytestmark = pytest.mark.gpu


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["OMP_NUM_THREADS"] = "1"
    env["HEAT2D_NO_BUILD"] = "1"
    return env


def _torchrun(n, script_args, cwd, timeout=400):
    # a port from free_port() can be taken again before the launcher binds it: retry on that
    # (and only that) with a fresh port
    for _attempt in range(3):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
               "127.0.0.1", "--master-port", str(free_port()), *script_args]
        r = subprocess.run(cmd, cwd=cwd, env=_env(), capture_output=True, text=True, timeout=timeout)
        if r.returncode != 0 and "EADDRINUSE" in r.stderr:
            continue
        break
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    return r.stdout


@pytest.mark.parametrize("n,gx,gy,boundary,periodic", [(2, 2, 1, "fixed", "none"), (4, 2, 2, "ghost-zero", "none"),
                                                       (2, 1, 2, "ghost-zero", "xy")])
def test_gpu_ranks_host_transport_match_oracle(native, gpu, tmp_path, n, gx, gy, boundary, periodic):
    nx, ny, steps = 301, 517, 37
    out = _torchrun(n, ["-m", "heat2d_amd", "--device", "gpu", "--transport", "host", "--nx", str(nx), "--ny", str(ny),
                        "--steps", str(steps), "--gridx", str(gx), "--gridy", str(gy), "--boundary", boundary,
                        "--periodic", periodic, "--output", "binary", "--outdir", str(tmp_path)], str(tmp_path))
    assert f"Starting with {n} processes" in out
    b = 0 if boundary == "fixed" else 1
    ref = native.oracle_run(nx, ny, steps, boundary=b, periodic_x="x" in periodic, periodic_y="y" in periodic)["grid"]
    assert np.array_equal(read_grid(tmp_path / "final_binary.dat", nx, ny), ref)


@pytest.mark.parametrize("n,boundary,conv", [(2, "fixed", 0), (3, "ghost-zero", 0), (4, "fixed", 1)])
def test_gpu_ranks_ipc_direct_match_oracle(native, gpu, tmp_path, n, boundary, conv):
    """Ranks sharing the GPU through real IPC handles: direct halo pushes between processes,
    the device all-reduce of the convergence residual, uneven row split."""
    nx, ny, steps = 67 * n + 1, 517, 61
    args = ["-m", "heat2d_amd", "--device", "gpu", "--transport", "ipc", "--nx", str(nx), "--ny", str(ny),
            "--steps", str(steps), "--gridx", str(n), "--gridy", "1", "--boundary", boundary, "--output", "binary",
            "--outdir", str(tmp_path)]
    kw = {}
    if conv:
        args += ["--convergence", "1", "--interval", "6", "--sensitivity", "1e-30"]
        kw = dict(convergence=True, interval=6, sensitivity=1e-30)
    out = _torchrun(n, args, str(tmp_path))
    assert f"Starting with {n} processes" in out
    b = 0 if boundary == "fixed" else 1
    ref = native.oracle_run(nx, ny, steps, boundary=b, **kw)["grid"]
    assert np.array_equal(read_grid(tmp_path / "final_binary.dat", nx, ny), ref)


@pytest.mark.parametrize("n,gx,gy,boundary,periodic,conv", [(4, 2, 2, "fixed", "none", 0),
                                                             (8, 2, 4, "ghost-zero", "none", 0),
                                                             (4, 2, 2, "fixed", "none", 1),
                                                             (4, 2, 2, "ghost-zero", "xy", 0),
                                                             (2, 1, 2, "fixed", "none", 0)])
def test_gpu_ranks_ipc_blocks_match_oracle(native, gpu, tmp_path, n, gx, gy, boundary, periodic, conv):
    """2-D blocks through the direct pipeline between processes sharing the GPU: row, column and
    corner halos pushed into the neighbours' IPC-mapped receive buffers, uneven row split,
    convergence all-reduce."""
    # tiles of 600 columns: a strip that pushes to a W/E neighbour must not also hold a global
    # edge column (the engine refuses narrower tiles at a global edge)
    nx, ny, steps = 61 * gx + 1, 600 * gy, 43
    args = ["-m", "heat2d_amd", "--device", "gpu", "--transport", "ipc", "--nx", str(nx), "--ny", str(ny),
            "--steps", str(steps), "--gridx", str(gx), "--gridy", str(gy), "--boundary", boundary, "--periodic",
            periodic, "--output", "binary", "--outdir", str(tmp_path), "--json"]
    kw = {}
    if conv:
        args += ["--convergence", "1", "--interval", "6", "--sensitivity", "1e-30"]
        kw = dict(convergence=True, interval=6, sensitivity=1e-30)
    out = _torchrun(n, args, str(tmp_path))
    assert '"pipeline": "direct"' in out
    b = 0 if boundary == "fixed" else 1
    ref = native.oracle_run(nx, ny, steps, boundary=b, periodic_x="x" in periodic, periodic_y="y" in periodic,
                            **kw)["grid"]
    assert np.array_equal(read_grid(tmp_path / "final_binary.dat", nx, ny), ref)


def test_gpu_bench_four_ranks_blocks_ipc(tmp_path):
    """The bench with the 2-D block layout at N=4 on one GPU: the gate picks the 2-D direct
    pipeline, the timed solver verifies against the oracle and the in-job reference."""
    out = _torchrun(4, [os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "20", "--warmup", "5", "--side",
                        "1024", "--layout", "blocks", "--prewarm-s", "0"], str(tmp_path))
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert d["config"]["parallelism"] == "blocks2x2" and d["config"]["candidate"] == "ipc/auto"
    assert d["config"]["pipeline"] == "direct" and d["verified"] is True
    assert min(d["halo_wait"]["waits_per_rank"]) > 0


@pytest.mark.parametrize("n", [4, 8])
def test_gpu_bench_persistent_rehearsal(tmp_path, n):
    """The driver's N=4 / N=8 strong-scaling command (4096^2, row strips) with every rank on one
    GPU and the persistent kernel forced on: the ranks split the GPU's wave slots
    (pstream_waves), every rank runs persistent launches through the direct pipeline, and the
    timed result is bit-exact (CPU oracle on the leading steps, rank 0's single-GPU run after all
    of them)."""
    out = _torchrun(n, [os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "42", "--warmup", "14",
                        "--persistent", "on", "--prewarm-s", "0"], str(tmp_path))
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert d["config"]["parallelism"] == f"rows{n}" and d["config"]["grid_per_gpu"] == [4096 // n, 4096]
    assert d["config"]["pipeline"] == "direct" and d["verified"] is True
    pl = d["config"]["persistent_launches_per_rank"]
    assert len(pl) == n and min(pl) > 0, pl


def test_gpu_bench_two_ranks_driver_environment(tmp_path):
    """The driver's own command at N=2 (default grid, pre-warm and flags) in the driver's environment:
    no HIP_FORCE_DEV_KERNARG inherited from this test process — bench.py's import of the library
    picks the kernel-argument setting itself, exactly as in the driver's run."""
    env = _env()
    env.pop("HIP_FORCE_DEV_KERNARG", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20",
           "--warmup", "5"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 2 and d["steps"] == 20 and d["warmup"] == 5 and d["verified"] is True
    assert d["config"]["grid"] == [4096, 4096]


def test_gpu_bench_two_ranks_ipc(tmp_path):
    """The bench at N=2 on one GPU: the gate picks the direct IPC transport first."""
    out = _torchrun(2, [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "40", "--warmup", "8", "--side",
                        "1024", "--prewarm-s", "0"], str(tmp_path))
    lines = [l for l in out.splitlines() if l.startswith("{")]
    d = json.loads(lines[-1])
    assert d["config"]["transport"] == "ipc" and d["config"]["pipeline"] == "direct"
    assert d["gate"][0]["ok"] and d["verified"] is True and "CPU oracle" in d["verification"]
    hw = d["halo_wait"]
    assert min(hw["waits_per_rank"]) > 0 and 0.0 <= hw["share_of_chunk"] and hw["max_us"] >= hw["mean_us_per_halo_unit"]


def test_gpu_bench_two_ranks_gate_downgrade(tmp_path, monkeypatch):
    """Both direct IPC flavours fail the gate (injected per transport/pipeline): every rank falls
    back together to the third candidate, the run is timed with it, verified, and the JSON says
    what failed and which candidate was used."""
    monkeypatch.setenv("HEAT2D_GATE_FAIL", "ipc/auto,ipc/direct-sys")
    out = _torchrun(2, [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20", "--warmup", "5", "--side",
                        "512", "--prewarm-s", "0"], str(tmp_path))
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert [(g["transport"], g["pipeline"], g["ok"]) for g in d["gate"]] == [
        ("ipc", "auto", False), ("ipc", "direct-sys", False), ("host", "serial", True)]
    assert d["config"]["transport"] == "host" and d["config"]["candidate"] == "host/serial"
    assert d["verified"] is True


def test_gpu_bench_two_ranks_direct_sys(tmp_path, monkeypatch):
    """Only the measured-fence flavour fails: the system-scope-fence direct pipeline is timed."""
    monkeypatch.setenv("HEAT2D_GATE_FAIL", "ipc/auto")
    out = _torchrun(2, [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20", "--warmup", "5", "--side",
                        "512", "--prewarm-s", "0"], str(tmp_path))
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert not d["gate"][0]["ok"] and d["gate"][1]["ok"]
    assert d["config"]["candidate"] == "ipc/direct-sys" and d["config"]["pipeline"] == "direct"
    assert d["verified"] is True and d["halo_wait"]["waits_per_rank"][0] > 0


def test_gpu_bench_two_ranks_host_transport(tmp_path):
    """Two ranks on the one GPU: the gate, the strong-scaling default and the in-job
    single-GPU reference with bit-exact verification of the timed run."""
    out = _torchrun(2, [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "40", "--warmup", "8", "--side",
                        "1024", "--prewarm-s", "0", "--transport", "host"], str(tmp_path))
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 40 and d["config"]["grid"] == [1024, 1024]
    assert d["value"] > 0 and d["config"]["transport"] == "host" and d["scaling"] == "strong"
    assert d["gate"][0]["ok"] and d["verified"] is True and d["speedup"] > 0


@pytest.mark.parametrize("n,gx,conv", [(2, 2, 0), (3, 3, 1), (4, 2, 0)])
def test_native_cli_ranks_ipc_on_gpu(native, gpu, tmp_path, n, gx, conv):
    """The native executable's own launcher (`heat2d --np P`, fork without exec) on the GPU:
    ranks share the card through the direct IPC halo pipeline (rows, and 2x2 blocks);
    bit-exact against the oracle."""
    exe = os.path.join(ROOT, "heat2d_amd", "bin", "heat2d")
    gy = n // gx
    nx, ny, steps = 70 * gx + 3, 520 if gy > 1 else 517, 41
    args = [exe, "--np", str(n), "--device", "gpu", "--nx", str(nx), "--ny", str(ny), "--steps", str(steps),
            "--gridx", str(gx), "--gridy", str(gy), "--output", "binary", "--outdir", str(tmp_path), "--json"]
    kw = {}
    if conv:
        args += ["--convergence", "1", "--interval", "6", "--sensitivity", "1e-30"]
        kw = dict(convergence=True, interval=6, sensitivity=1e-30)
    r = subprocess.run(args, cwd=str(tmp_path), env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert '"pipeline": "direct"' in r.stdout and f'"ranks": {n}' in r.stdout
    ref = native.oracle_run(nx, ny, steps, **kw)["grid"]
    assert np.array_equal(read_grid(tmp_path / "final_binary.dat", nx, ny), ref)


def test_gpu_halo_wait_sees_a_late_neighbour(tmp_path):
    """The exposed halo wait (the MPI_Waitall analogue, Report.pdf p.34-37): a neighbour that
    starts 50 ms late shows up in the waiting rank's in-kernel halo-wait counters, not in the
    late rank's."""
    out = _torchrun(2, [os.path.join(ROOT, "tests", "_halo_delay_worker.py")], str(tmp_path))
    # the two ranks' lines can interleave on the launcher's stdout: pick the JSON objects out
    import re

    recs = {d["rank"]: d for d in (json.loads(m) for m in re.findall(r'\{"rank"[^{}]*\}', out))}
    assert set(recs) == {0, 1}
    # loose bounds: gloo barrier skew and launch latency can eat into the 50 ms delay,
    # but not most of it
    assert recs[0]["max_us"] > 5000.0, recs
    assert recs[1]["max_us"] < recs[0]["max_us"], recs
    assert recs[0]["waits"] > 0 and recs[1]["waits"] > 0


@pytest.mark.parametrize("mode", ["plain", "conv"])
def test_gpu_persistent_two_processes(tmp_path, mode):
    """The persistent kernel on two ranks of the direct pipeline (separate processes, IPC handles
    carrying each rank's persistent push counts): bit-exact on both ranks, across two runs.
    conv: with the fused convergence check — persistent launches between the checks, stop at the
    oracle's step (the decision through the IPC all-reduce), then continue after a re-prime."""
    import re

    out = _torchrun(2, [os.path.join(ROOT, "tests", "_pstream_ranks_worker.py")] + (["conv"] if mode == "conv" else []),
                    str(tmp_path))
    recs = {d["rank"]: d for d in (json.loads(m) for m in re.findall(r'\{"rank"[^{}]*\}', out))}
    assert set(recs) == {0, 1}, out[-2000:]
    if any("skip" in r for r in recs.values()):
        pytest.skip(recs[0].get("skip") or recs[1].get("skip"))
    for r in recs.values():
        assert r["ok"] and r["ok2"] and r["launches"] >= 1, recs
