import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "ska-sdp-idg-bench_amd")
ORACLE = os.path.join(REPO, "oracle")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, ORACLE, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

# Parity bar of the reference harness (tests/test_util.hpp:84).
TOLERANCE = 1e-5


def pytest_configure(config):
    config.addinivalue_line(
        "markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    # -m gpu on a box without a GPU must fail loudly, not skip: the product
    # path has no fallback.  Without -m gpu the gpu tests are deselected by
    # the driver's -m "not gpu".
    pass


def load_manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


CASES = sorted(load_manifest()["cases"].keys())


def load_case(name):
    man = load_manifest()["cases"][name]
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    arrays = {k: np.ascontiguousarray(z[k]) for k in z.files}
    return man["params"], arrays


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle as _o
    return _o.Oracle()
