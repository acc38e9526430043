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


@pytest.fixture(params=[(0, 0), (1, 0), (0, 12), (0, 6), (3, 0), (3, 6)],
                ids=["rows", "tasks", "rows12", "rows6", "dyn", "dyn6"])
def impl(request):
    """Runs a decode-GEMV test on every kernel: kq_rows (default), kq_gemv, kq_rows at both
    launch shapes (waves per workgroup by launch size, 12 and 6), and the claimed-row
    kq_rows_dyn forced on every one-type launch (by size, and at 6 waves)."""
    import ggml_mi355x as g
    which, waves = request.param
    prev = g.gemv_impl(which)
    prev_w = g.gemv_waves(waves)
    yield which
    g.gemv_impl(prev)
    g.gemv_waves(prev_w)
