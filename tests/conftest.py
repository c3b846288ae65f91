"""Test configuration.

* ``gpu`` marker: needs a real MI355X (run with ``-m gpu``); everything else runs on CPU.
* The native extension is (re)built in-tree once per session if missing or stale, so the
  CPU tier exercises the same compiled C++ core as the GPU tier.
"""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X / gfx950)")
    config.addinivalue_line("markers", "slow: long-running test")
    if os.environ.get("PKD_SKIP_BUILD") != "1":
        from parallel_kd_tree_amd import _build
        _build.build(verbose=False)


@pytest.fixture(scope="session")
def native():
    from parallel_kd_tree_amd.ops import native as _n
    return _n()


@pytest.fixture(scope="session")
def bin_dir():
    return ROOT / "bin"


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but torch.cuda.is_available() is False")
    return torch.device("cuda:0")
