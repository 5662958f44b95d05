import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


def pytest_collection_modifyitems(config, items):
    # the per-config GPU parity tests run first (tests/test_gpu_configs.py)
    items.sort(key=lambda it: 0 if it.nodeid.startswith("tests/test_gpu_configs.py") or
               os.path.basename(str(it.fspath)) == "test_gpu_configs.py" else 1)
    have_gpu = False
    try:
        import torch
        have_gpu = torch.cuda.is_available()
    except Exception:
        pass
    if not have_gpu:
        skip = pytest.mark.skip(reason="no GPU in this container")
        for it in items:
            if "gpu" in it.keywords:
                it.add_marker(skip)


def golden(name):
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


@pytest.fixture(scope="session")
def oracle():
    from oracle_py import Oracle, build
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        build(ref=False)
    return Oracle()
