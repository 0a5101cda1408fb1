import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (os.path.join(ROOT, "phase-vocoder_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def cuda():
    if not gpu_available():
        pytest.skip("no GPU")
    import torch
    from pvamd import _lib
    # the GPU tests check the product: a diagnostic build (timing-only ablations,
    # instrumentation; pv_diagnostic_build() = 1) is refused loudly
    assert not _lib.diagnostic_build(), f"{_lib.LIB_PATH} is a diagnostic build (PV_DIAGNOSTIC_BUILD)"
    return torch.device("cuda:0")
