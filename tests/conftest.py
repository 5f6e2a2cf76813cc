"""Test configuration.

* ``gpu`` marker: needs a real MI355X (run with ``-m gpu``); everything else runs on CPU.
* The native extension is built in-tree once per session if missing or stale.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X)")
    config.addinivalue_line("markers", "slow: long-running test")
    if os.environ.get("HEAT2D_NO_BUILD") != "1":
        from heat2d_amd import _build

        # binaries stamped with the current source hash are up to date: no compile step (a GPU
        # box receives the built extension and CLI but not build/obj, so an object-level
        # incremental build there would recompile everything)
        want = _build.source_hash()
        if _build.stamped_hash(_build.EXT_PATH) != want or _build.stamped_hash(_build.CLI_PATH) != want:
            _build.build(cli=True)


@pytest.fixture(scope="session")
def native():
    from heat2d_amd import native as _n

    return _n()


@pytest.fixture(scope="session")
def gpu(native):
    if native.device_count() < 1:
        pytest.fail("GPU test selected but no HIP device is visible")
    return 0
