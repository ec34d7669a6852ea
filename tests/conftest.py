import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def native():
    from fastapriori_amd.ops import build
    build.build_host()
    return True


@pytest.fixture
def tune():
    """tune(name=value, ...) sets fastapriori_amd.tuning.TUNING knobs for one test and
    restores them afterwards (the config object, not module globals)."""
    from fastapriori_amd.tuning import TUNING
    saved = {}

    def set_(**kw):
        for k, v in kw.items():
            if not hasattr(TUNING, k):
                raise AttributeError(f"unknown tuning knob {k}")
            saved.setdefault(k, getattr(TUNING, k))
            setattr(TUNING, k, v)
        return TUNING

    yield set_
    for k, v in saved.items():
        setattr(TUNING, k, v)
