import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "leak-det-gnn_amd"
GOLD = REPO / "tests" / "golden"
LTA_INP = PKG / "data" / "L-TOWN-A.inp"

for p in (str(REPO), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); runs the HIP kernels")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no ROCm GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
