import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) HIP device; runs the HIP path")


def _gpu_count():
    # torch's device count does not initialise HIP on this image, so the pytest process has not used the GPU when
    # tests/test_dist_gpu.py (the first GPU module) starts its torch.distributed child
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:
        return 0


def pytest_collection_modifyitems(config, items):
    if any(item.get_closest_marker("gpu") for item in items) and _gpu_count() < 1:
        skip = pytest.mark.skip(reason="no HIP device visible")
        for item in items:
            if item.get_closest_marker("gpu"):
                item.add_marker(skip)


@pytest.fixture(scope="session")
def meshes():
    return dict(np.load(os.path.join(GOLDEN, "meshes.npz")))


@pytest.fixture(scope="session")
def ref_tests():
    with open(os.path.join(GOLDEN, "ref_tests.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O
