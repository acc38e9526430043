import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device; runs the HIP path")


@pytest.fixture(scope="session")
def oracle():
    from oracle import kq_oracle
    kq_oracle.lib()
    return kq_oracle


@pytest.fixture(scope="session")
def npo():
    from oracle import kq_oracle_np
    return kq_oracle_np


@pytest.fixture(scope="session")
def dev():
    """GPU tests: the HIP library and a gfx950 device must be present (no skip, no fallback)."""
    import torch
    import ggml_mi355x as g
    assert g.device_available(), "gfx950 device / libggml_mi355x.so required for -m gpu tests"
    assert torch.cuda.is_available()
    return torch.device("cuda:0")


@pytest.fixture(params=[(0, 0), (1, 0), (0, 12), (0, 6)], ids=["rows", "tasks", "rows12", "rows6"])
def impl(request):
    """Runs a decode-GEMV test on both kernels, kq_rows (default) and kq_gemv, and kq_rows
    at both launch shapes: waves per workgroup by launch size (default), 12 and 6."""
    import ggml_mi355x as g
    which, waves = request.param
    prev = g.gemv_impl(which)
    prev_w = g.gemv_waves(waves)
    yield which
    g.gemv_impl(prev)
    g.gemv_waves(prev_w)
