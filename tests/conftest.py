import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")
    config.addinivalue_line(
        "markers", "ablation: checks a measured-slower, non-shipped code path kept for A/B "
        "timing; skipped unless GSPLAT_TEST_ABLATION=1")


def pytest_collection_modifyitems(config, items):
    if os.environ.get("GSPLAT_TEST_ABLATION") == "1":
        return
    skip = pytest.mark.skip(reason="ablation path (set GSPLAT_TEST_ABLATION=1 to run)")
    for item in items:
        if "ablation" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


@pytest.fixture
def quirk_mask(request, oracle_lib):
    """Run a test under GSPLAT_QUIRK_* mask request.param (default all) in both the HIP library
    and the oracle, restoring the previous mask afterwards."""
    from gaussctrl_exp_amd import quirks
    mask = getattr(request, "param", quirks.ALL)
    prev, prev_o = quirks.get(), oracle_lib.get_quirks()
    quirks.set(mask)
    oracle_lib.set_quirks(mask)
    yield mask
    quirks.set(prev)
    oracle_lib.set_quirks(prev_o)


@pytest.fixture
def hooks():
    """The test's C-ABI calls go to the test library (libgsplat_mi355x_hooks.so: the shipped
    kernels plus the gsplat_debug_* switches, include/gsplat_mi355x.h "test hooks")."""
    from gaussctrl_exp_amd import _lib
    with _lib.hooks() as L:
        yield L
