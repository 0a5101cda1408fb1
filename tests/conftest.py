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
def device_asm(tmp_path_factory):
    """gfx950 assembly of the kernel sources (the Makefile's device flags) and the compiler's
    kernel-resource-usage remarks, one parallel compile per source, shared by the tests that
    read them: {source: (asm path, remarks text)}"""
    import subprocess
    d = tmp_path_factory.mktemp("asm")
    csrc = os.path.join(ROOT, "phase-vocoder_amd", "csrc")
    flags = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
             "-fhip-fp32-correctly-rounded-divide-sqrt", "--cuda-device-only", "-S",
             "-Rpass-analysis=kernel-resource-usage"]
    procs = {}
    for src in ("pv_analysis", "pv_kernels", "pv_fused", "pv_rt"):
        extra = ["-fno-slp-vectorize"] if src == "pv_analysis" else []
        out = str(d / f"{src}.s")
        procs[src] = (out, subprocess.Popen(["/opt/rocm/bin/hipcc", *flags, *extra, "-I", os.path.join(ROOT, "include"),
                                             "-o", out, os.path.join(csrc, f"{src}.hip")],
                                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    res = {}
    for src, (out, pr) in procs.items():
        so, se = pr.communicate(timeout=900)
        assert pr.returncode == 0, se[-2000:]
        res[src] = (out, so + se)
    return res


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
