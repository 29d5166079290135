"""pytest setup: import paths and the `gpu` marker.

`-m "not gpu"` runs the oracle-vs-golden, host-logic, drop-in API and C-ABI symbol
tests on CPU; `-m gpu` runs the parity tests through libmivs.so on an MI355X.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cuvs-rag_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) GPU and the built libmivs.so")
    config.addinivalue_line("markers", "slow: large-size property tests")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no ROCm GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def mivs_lib():
    import mivs

    mivs.load()  # fails loudly if libmivs.so is missing: no fallback path exists
    return mivs
