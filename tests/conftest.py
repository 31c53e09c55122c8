import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running (large inputs)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build_oracle()
    return O


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np
    d = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(d, "golden.json")) as f:
        meta = json.load(f)
    arr = np.load(os.path.join(d, "golden.npz"), allow_pickle=False)
    cases = {}
    for name, info in meta["cases"].items():
        cases[name] = dict(info, text=arr[f"{name}__text"], sa=arr[f"{name}__sa"], lcp=arr[f"{name}__lcp"])
    return {"cases": cases, "known": meta["known_answers"]}


@pytest.fixture(scope="session")
def sa_lib():
    """libsa_hip built in-tree (hipcc cross-compiles here without a GPU)."""
    from hpc_suffix_array_amd import _native as N
    N.build_library()
    return N


@pytest.fixture(scope="session")
def gpu(sa_lib):
    import torch  # noqa: F401  (binds the HIP runtime torch ships before the library's)
    if sa_lib.device_count() <= 0:
        pytest.fail("gpu test selected but no HIP device is visible")
    return sa_lib
