"""Bench plumbing on the CPU: named BASELINE configurations, labels, HBM sizing, fallback chains."""
import pytest

from heat2d_amd.utils import benchmark as B


def test_grid_for_strong_weak_rows_blocks():
    assert B.grid_for(1, 4096, "strong", "rows") == (4096, 4096, 1, 1)
    assert B.grid_for(8, 4096, "strong", "rows") == (4096, 4096, 8, 1)
    assert B.grid_for(8, 16384, "strong", "blocks") == (16384, 16384, 2, 4)
    assert B.grid_for(2, 8192, "strong", "rows") == (8192, 8192, 2, 1)
    assert B.grid_for(8, 4096, "weak", "rows") == (8 * 4096, 4096, 8, 1)
    assert B.grid_for(8, 100, "weak", "blocks") == (200, 400, 2, 4)
    with pytest.raises(ValueError):
        B.grid_for(2, 10, "sideways", "rows")


def test_configs_cover_baseline_rows():
    c = B.CONFIGS
    assert c["4096-strong"].side == 4096 and c["4096-strong"].scaling == "strong"
    assert c["8192x2rows"].layout == "rows" and c["16384x8blocks"].layout == "blocks"
    assert c["weak-hbm"].side == 0 and c["weak-hbm"].scaling == "weak"


def test_metric_label_tracks_the_run():
    assert B.metric_label(4096, 4096, 1000) == "cell-updates/sec (whole node) + speedup/efficiency, 4096^2 grid 1000 steps"
    assert B.metric_label(32768, 4096, 20).endswith("32768x4096 grid 20 steps")


def test_fill_hbm_side_fits_two_buffers():
    free = 288 * 10**9
    side = B.fill_hbm_side(free, G=8)
    assert side % 256 == 0
    assert 2 * B.tile_bytes(side, side, 8) <= free * 0.98 - (3 << 30)
    assert 2 * B.tile_bytes(side + 256, side + 256, 8) > free * 0.98 - (3 << 30)
    assert 2 * side * side * 4 > 250 * 10**9  # ~259 GB of the 288 GB card
    with pytest.raises(ValueError):
        B.fill_hbm_side(1 << 20)


def test_tile_bytes_matches_engine_geometry(native):
    for nx, ny, G in [(100, 517, 8), (4096, 4096, 8), (33, 7, 3)]:
        g = native.tile_geom(nx, ny, G)
        actual = g["srows"] * g["pitch"] * 4
        assert actual <= B.tile_bytes(nx, ny, G) <= actual + g["srows"] * 320 * 4


def test_candidate_chains():
    assert B.candidates("auto", "auto", 1, True, True, "rows") == [("local", "auto")]
    assert B.candidates("auto", "auto", 4, False, False, "rows") == [("torch", "serial")]
    # ranks sharing one GPU: both direct flavours, then host staging
    assert B.candidates("auto", "auto", 2, True, False, "rows") == [("ipc", "auto"), ("ipc", "direct-sys"),
                                                                    ("host", "serial")]
    assert B.candidates("auto", "auto", 4, True, False, "blocks") == [("ipc", "auto"), ("ipc", "direct-sys"),
                                                                      ("host", "serial")]
    assert B.candidates("auto", "auto", 4, True, False, "blocks", cols_per_rank=30) == [("host", "serial")]
    # distinct devices (the first cross-device run must fail safe): measured fences, system-scope
    # fences, RCCL signalled, RCCL serial, host staging
    ch = B.candidates("auto", "auto", 8, True, True, "rows")
    assert ch == [("ipc", "auto"), ("ipc", "direct-sys"), ("rccl", "signal"), ("rccl", "serial"), ("host", "serial")]
    assert B.candidates("auto", "auto", 8, True, True, "blocks") == ch  # 2-D direct IPC too
    assert B.candidates("auto", "auto", 8, True, True, "blocks", cols_per_rank=4094)[0] == ("rccl", "signal")
    # strips too short for halo units of the depth: no direct IPC candidate
    assert B.candidates("auto", "auto", 8, True, True, "rows", rows_per_rank=10, depth=7)[0] == ("rccl", "signal")
    assert B.candidates("rccl", "serial", 8, True, True, "rows") == [("rccl", "serial"), ("host", "serial")]
    assert len(ch) == len(set(ch))


def test_forced_gate_failures(monkeypatch):
    monkeypatch.setenv("HEAT2D_GATE_FAIL", "ipc/auto,rccl")
    assert B.forced_failure("ipc", "auto") and not B.forced_failure("ipc", "direct-sys")
    assert B.forced_failure("rccl", "signal") and B.forced_failure("rccl", "serial")
    assert not B.forced_failure("host", "serial")
