"""Node-local spin barrier (csrc/shm_barrier.cpp, ``DistContext.node_barrier``) that brackets
the bench's timed region: barrier semantics under uneven arrival, every rank on the shm path,
and no segment left behind in /dev/shm."""
import json
import os
import subprocess
import sys

from tests.test_multiprocess_cpu import ROOT, free_port


def _segments():
    try:
        return {f for f in os.listdir("/dev/shm") if f.startswith("heat2d_bar_")}
    except OSError:
        return set()


def test_node_barrier_semantics(tmp_path):
    before = _segments()
    out = tmp_path / "rec.json"
    n, rounds = 4, 40
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "tests", "_node_barrier_worker.py"),
           str(out), str(rounds)]
    env = dict(os.environ, OMP_NUM_THREADS="1", HEAT2D_NO_BUILD="1")
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    recs = json.loads(out.read_text())
    assert sorted(x["rank"] for x in recs) == list(range(n))
    assert all(x["shm"] == 1 for x in recs), "every rank must use the shm barrier on one node"
    for i in range(rounds):
        last_arrival = max(x["arr"][i] for x in recs)
        first_exit = min(x["dep"][i] for x in recs)
        assert first_exit >= last_arrival, f"round {i}: a rank left before the last one arrived"
    assert _segments() <= before, "the barrier segment must be unlinked after setup"


def test_shm_barrier_single_process(native):
    b = native.ShmBarrier(f"/heat2d_bar_test_{os.getpid()}", 0, 1, True)
    for _ in range(3):
        assert b.wait(1.0) >= 0.0
    b.unlink()
    assert f"heat2d_bar_test_{os.getpid()}" not in _segments()


def test_shm_barrier_rejects_bad_arguments(native):
    import pytest

    name = f"/heat2d_bar_args_{os.getpid()}"
    with pytest.raises(Exception):
        native.ShmBarrier("no_leading_slash", 0, 2, True)
    with pytest.raises(Exception):
        native.ShmBarrier(name, 2, 2, True)  # rank out of range
    owner = native.ShmBarrier(name, 0, 2, True)
    with pytest.raises(Exception):
        native.ShmBarrier(name, 1, 3, False)  # world size differs from the creator's
    with pytest.raises(Exception):
        native.ShmBarrier(name, 0, 2, True)  # exclusive create: the name exists
    with pytest.raises(Exception):
        owner.wait(0.05)  # rank 1 never arrives: bounded wait
    owner.unlink()
    with pytest.raises(Exception):
        native.ShmBarrier(name, 1, 2, False)  # unlinked: nothing to open
