import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REF = "/root/reference"
# reference example CSVs (Example_*.csv, data only), shipped as tracked fixtures
DATA = os.path.join(ROOT, "tests", "data")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running statistical test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def example(name):
    """Path of an example CSV of the reference (tracked copy in tests/data/)."""
    for d in (DATA, os.path.join(ROOT, ".refdata"), REF):
        p = os.path.join(d, name)
        if os.path.exists(p):
            return p
    return os.path.join(DATA, name)


def have_example(name):
    return os.path.exists(example(name))
