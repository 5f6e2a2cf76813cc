"""The analytic cost models (heat2d_amd/utils/model.py) and the scaling-table tool."""
import json
import os
import subprocess
import sys

from heat2d_amd.utils import model as M

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_report_blocks_model_reproduces_table_17_19():
    # Report.pdf p.31-32: blocks, 2560x2048, P = 160 -> 0.119 s, efficiency 0.997
    t = M.report_time_blocks(2560, 2048, 160)
    assert round(t * 1e-6, 3) == 0.119
    e = M.report_time_blocks(2560, 2048, 1) / t / 160
    assert round(e, 3) == 0.997


def test_report_strips_formula_terms():
    tc, ts, tw = M.REPORT_TC_US, M.REPORT_TS_US, M.REPORT_TW_US
    assert M.report_time_strips(1000, 1000, 100) == tc * 1000 * (1000 // 100 + 1) + 2 * ts + 4 * 1000 * tw
    # orientation: M >= N is the long side
    assert M.report_time_strips(1000, 500, 10) == M.report_time_strips(500, 1000, 10)


def test_report_tables_shape_and_p1():
    tab = M.report_tables(M.REPORT_GRIDS, M.REPORT_PROCS, "strips")
    assert set(tab) == set(M.REPORT_GRIDS)
    for rows in tab.values():
        assert rows[0][0] == 1 and abs(rows[0][2] - 1.0) < 1e-12 and abs(rows[0][3] - 1.0) < 1e-12


def test_mi355x_model_shapes():
    # fitted to the measured single-GPU 4096^2 run (7.8 us/step) within 10 %
    assert abs(M.step_time_us(4096, 4096, 8) - 7.81) / 7.81 < 0.1
    rows = M.strong_scaling(4096, [1, 2, 4, 8], "rows", 1000)
    assert rows[0]["speedup"] == 1.0
    assert all(a["speedup"] < b["speedup"] for a, b in zip(rows, rows[1:]))
    assert all(0 < r["efficiency"] <= 1.0 for r in rows)
    assert M.strips(4096, 8) == 17  # edge-aligned fixed-edge layout (kernels.hip strip_layout)


def test_mi355x_strips_matches_engine(native):
    for ny, K in [(4096, 8), (4096, 4), (1000, 6), (700, 8)]:
        assert M.strips(ny, K) == len(native.strip_layout(64, ny, K, True, False)), (ny, K)


def test_scaling_table_tool(tmp_path):
    recs = []
    for n, ms in [(1, 8.0), (2, 4.5), (8, 1.9)]:
        recs.append({"n_gpus": n, "value": 4096 * 4096 / (ms * 1e-3), "ms_per_step": ms, "scaling": "strong",
                     "speedup": None, "efficiency": None, "config": {"grid": [4096, 4096], "transport": "ipc",
                                                                      "pipeline": "direct"}})
    p = tmp_path / "b.jsonl"
    p.write_text("\n".join(json.dumps(r) for r in recs))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scaling_table.py"), str(p)],
                         capture_output=True, text=True, check=True).stdout
    assert "4.21" in out  # 8 GPUs: 8.0 / 1.9
