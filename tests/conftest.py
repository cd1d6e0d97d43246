"""Test configuration: markers, import paths and shared fixtures.

`-m "not gpu"` tests run on CPU (oracle vs golden vectors, host logic, C-ABI loading and
argument validation, gloo multi-process paths).  `-m gpu` tests are the parity tests proper:
they call the HIP kernels through the C ABI and compare with the oracle.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "two-tower-model-v2_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests")
    config.addinivalue_line("markers", "slow: long-running (full-size) case")
    config.addinivalue_line("markers", "perf: wall-clock guard on a GPU (not part of -m gpu)")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        have_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        have_gpu = False
    if have_gpu:
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for item in items:
        if "gpu" in item.keywords or "perf" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def golden():
    d = os.path.join(ROOT, "tests", "golden")

    def load(name):
        return np.load(os.path.join(d, name), allow_pickle=False)

    return load


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle

    oracle.lib()
    return oracle
