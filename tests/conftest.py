import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# tests tune kernels per process (isolation); tests of the persistent autotuner table point it at a temp dir
os.environ.setdefault("PVA_TUNE_CACHE", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built _C extension")
    config.addinivalue_line("markers", "slow: long-running test")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU on this host")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
