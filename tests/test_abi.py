"""CPU checks of the C-ABI library: it loads, exports every symbol include/pv.h declares,
and its host-only helpers behave (no compute calls: there is no GPU here)."""
import ctypes
import os
import subprocess

import pytest

from conftest import ROOT
from pvamd import _lib


def test_library_loads_and_exports_every_declared_symbol():
    L = _lib.lib()
    declared = _lib.declared_symbols()
    assert len(declared) >= 14
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in nm.splitlines() if " T " in ln}
    assert set(declared) <= exported


def test_library_is_built_from_this_tree():
    """libpv.so carries the hash of the sources it was built from (the Makefile's SRC_SHA);
    it must be the tree's, the hash bench.py records, and the Makefile's own computation."""
    L = _lib.lib()  # refuses a mismatch itself
    built = L.pv_sources_sha().decode()
    assert built == _lib.sources_sha()
    import bench
    assert bench.kernel_sources_sha() == built
    mk = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "phase-vocoder_amd", "csrc"), "sources-sha"],
                        capture_output=True, text=True, check=True).stdout.strip()
    assert mk == built


def test_stale_library_is_refused(tmp_path, monkeypatch):
    """A library whose compiled-in hash differs from the tree's is not loaded."""
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "sources_sha", lambda: "0000000000000000")
    with pytest.raises(_lib.PVError, match="built from sources"):
        _lib.lib()
    monkeypatch.setattr(_lib, "_lib", None)


def test_library_is_gfx950_code_object():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob


def test_abi_version_and_status_strings():
    L = _lib.lib()
    assert L.pv_abi_version() == _lib.ABI_VERSION == 5
    assert L.pv_status_string(0) == b"PV_OK"
    assert L.pv_status_string(2) == b"PV_ERR_UNSUPPORTED"


def test_contract_version_matches_oracle():
    """The GPU's fp32 analysis contract and the oracle's restatement are versioned together
    (DESIGN.md §3.2): a library and an oracle of different versions would disagree in the
    last bits of the phases and hence in unwrap decisions."""
    import pvref
    assert _lib.lib().pv_contract_version() == pvref.contract_version() == 4


def test_frame_count_is_main_cpp_loop():
    # main.cpp:231  for (i = 0; i < numSamples - hopSize; i += hopSize)
    def loop(n, hop):
        c, i = 0, 0
        while i < n - hop:
            c += 1
            i += hop
        return c
    for n in (0, 1, 255, 256, 257, 1000, 441000, 2646000):
        for hop in (64, 128, 256, 512):
            assert _lib.frame_count(n, hop) == loop(n, hop)


def test_create_rejects_bad_configs_without_touching_gpu():
    L = _lib.lib()
    h = ctypes.c_void_p()
    for cfg in (_lib.config(1000, 4, ord("t"), 1.0, 1, 1, 10, 0),   # N not a power of 2
                _lib.config(1024, 0, ord("t"), 1.0, 1, 1, 10, 0),   # hop_div 0
                _lib.config(1024, 4, ord("x"), 1.0, 1, 1, 10, 0),   # bad effect
                _lib.config(1024, 4, ord("t"), -1.0, 1, 1, 10, 0),  # bad scale
                _lib.config(1024, 4, ord("p"), 2.0, 0, 1, 10, 0),   # compat has no pitch
                _lib.config(1024, 4, ord("t"), 1.0, 0, 1, 10, 0, 7),  # unknown window
                _lib.config(1024, 4, ord("t"), 1.0, 1, 1, 10, 0, 2)):  # STANDARD: Hann only
        st = L.pv_create(ctypes.byref(cfg), ctypes.byref(h))
        assert st in (_lib.PV_ERR_ARG, _lib.PV_ERR_UNSUPPORTED)
        assert len(L.pv_last_error()) > 0


def test_product_does_not_reference_oracle():
    root = _lib.ROOT
    for dirpath, _, files in os.walk(os.path.join(root, "phase-vocoder_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".hpp", ".h")):
                code = [ln for ln in open(os.path.join(dirpath, f)).read().splitlines()
                        if not ln.lstrip().startswith(("//", "#", "*", "/*")) or ln.lstrip().startswith("#include")]
                txt = "\n".join(code)
                for bad in ("import pvref", "from pvref", "libpvref", "oracle/", "pvr_"):
                    assert bad not in txt, (f, bad)


@pytest.mark.slow
def test_prefetch_kernels_have_no_spills(device_asm):
    """The self-tracked prefetch (gload_pairs / vm_wait, pv_device.hpp) is only sound when
    the registers it loads are never spilled or moved to AGPRs while in flight: the
    kernels that use it (analysis L <= 1024, register-OLA synthesis L <= 512) must compile
    without spills or AGPR use."""
    import re
    remarks = "\n".join(txt for _, txt in device_asm.values())
    rows, cur = {}, None
    for line in remarks.splitlines():
        m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
        if not m:
            continue
        body = m.group(1)
        if body.startswith("Function Name:"):
            cur = body.split(":", 1)[1].strip()
            rows[cur] = {}
        elif cur and ":" in body:
            k, v = body.split(":", 1)
            rows[cur][k.strip()] = v.strip()
    assert rows, remarks[-2000:]
    checked = 0
    for name, info in rows.items():
        m = re.match(r"_ZN2pv14k_std_analysisILi(\d+)E", name)
        n = re.match(r"_ZN2pv11k_synthesisILi(\d+)ELi\dELi([124])E", name)
        f = re.match(r"_ZN2pv7k_fusedILi512E", name)
        if (m and int(m.group(1)) <= 1024) or (n and int(n.group(1)) <= 512) or f:
            checked += 1
            assert info.get("VGPRs Spill") == "0" and info.get("AGPRs") == "0", (name, info)
    assert checked >= 4 + 3 * 3 * 3
    # the occupancy the hot kernels are sized for (the config-2 single
    # launch holds 3 workgroups per CU (balanced runs) at 3 waves/SIMD with no spills, the
    # analyses run at 3 or more, the config-4 synthesis at the 2 its LDS allows)
    floors = {r"_ZN2pv11k_synthesisILi512ELi0ELi1ELb1ELb1": 3, r"_ZN2pv11k_synthesisILi1024ELi[02]ELi4ELb1": 2,
              r"_ZN2pv14k_std_analysisILi1024ELb0ELi[124]ELb1": 3,
              r"_ZN2pv14k_std_analysisILi512ELb0ELi2ELb1": 3, r"_ZN2pv7k_fusedILi512ELi[23]ELi2E": 3}
    for pat, floor in floors.items():
        hits = [(n, i) for n, i in rows.items() if re.match(pat, n)]
        assert hits, pat
        for name, info in hits:
            assert int(info["Occupancy [waves/SIMD]"]) >= floor and info.get("AGPRs") == "0", (name, info)


def test_create_rejects_a_config_built_against_another_header():
    """pv_config / pv_info lead with abi_version: a caller compiled against an
    older pv.h is refused with PV_ERR_ARG instead of having its struct misread."""
    L = _lib.lib()
    h = ctypes.c_void_p()
    cfg = _lib.config(1024, 4, ord("t"), 1.0, 1, 1, 10, 0)
    for bad in (3, 0, 1024):  # an ABI-3 caller's first field is n_samps
        cfg.abi_version = bad
        assert L.pv_create(ctypes.byref(cfg), ctypes.byref(h)) == _lib.PV_ERR_ARG
        assert b"abi_version" in L.pv_last_error()
        assert not h.value


def test_create_rejects_bad_spec_layouts():
    L = _lib.lib()
    h = ctypes.c_void_p()
    for cfg in (_lib.config(1024, 4, ord("t"), 1.0, 1, 1, 10, 0, spec_layout=2),     # unknown
                _lib.config(1024, 4, ord("t"), 1.0, 0, 1, 10, 0, spec_layout=1)):    # REF_COMPAT
        assert L.pv_create(ctypes.byref(cfg), ctypes.byref(h)) != _lib.PV_OK
        assert not h.value


def test_static_inline_helpers_are_not_abi_symbols():
    assert "pv_unpack_bins" not in _lib.declared_symbols()
    assert "pv_process" in _lib.declared_symbols()


def test_fused_stamps_diagnostic_compiles():
    """The diagnostic build configurations (PV_FUSED_STAMPS: per-wave phase stamps of the
    config-2 single launch, scripts/fused_stamps.py; the PV_ABL_* timing-only ablations)
    compile only together with PV_DIAGNOSTIC_BUILD, which the library then reports."""
    import subprocess
    csrc = os.path.join(_lib.ROOT, "phase-vocoder_amd", "csrc")
    for src in ("pv_fused.hip", "pv_api.cpp"):
        cmd = ["/opt/rocm/bin/hipcc", "-O1", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
               "-DPV_FUSED_STAMPS", "-DPV_DIAGNOSTIC_BUILD", "-fPIC", "-c", os.path.join(csrc, src), "-o", os.devnull]
        if src.endswith(".cpp"):
            cmd[1:1] = ["-x", "hip"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
    # without PV_DIAGNOSTIC_BUILD an ablation switch is a compile error
    cmd = ["/opt/rocm/bin/hipcc", "-x", "hip", "-O0", "-std=c++17", "--offload-arch=gfx950", "-DPV_ABL_NOSTORE",
           "-fsyntax-only", os.path.join(csrc, "pv_api.cpp")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode != 0 and "PV_DIAGNOSTIC_BUILD" in r.stderr


def test_product_library_is_not_diagnostic():
    assert _lib.diagnostic_build() is False


def test_device_asm_has_no_prefetch_or_scc_hazards(device_asm):
    """The self-tracked prefetch loads (inline asm, invisible to the compiler's waits) must not
    have their registers read, written or copied before the vmcnt that retires them, and no
    inline asm that writes SCC may sit between an SCC writer and its reader
    (scripts/prefetch_hazards.py; both once produced wrong results and a GPU fault)."""
    import subprocess
    import sys
    outs = [out for out, _ in device_asm.values()]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "prefetch_hazards.py"), *outs],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.strip().endswith("0 hazard(s)"), r.stdout[-3000:]


def test_rt_and_harmonizer_create_reject_bad_configs_without_touching_gpu():
    """pv_rt_create / pv_harmonizer_create check the ABI version before any other field
    (ADVICE r5), then their own limits, all before a device call (pv_api.cpp)."""
    L = _lib.lib()
    h = ctypes.c_void_p()
    ratios = (ctypes.c_float * 2)(1.5, 0.5)
    good = _lib.config(1024, 4, ord("p"), 1.5, 1, 1, 10, 0)
    bad_abi = _lib.config(1024, 4, ord("p"), 1.5, 1, 1, 10, 0)
    bad_abi.abi_version = 4
    assert L.pv_rt_create(ctypes.byref(bad_abi), 2, ctypes.byref(h)) == _lib.PV_ERR_ARG
    assert b"abi_version" in L.pv_last_error()
    assert L.pv_harmonizer_create(ctypes.byref(bad_abi), ratios, 2, ctypes.byref(h)) == _lib.PV_ERR_ARG
    assert b"abi_version" in L.pv_last_error()
    # voice count outside [1, 64]
    for k in (0, -1, 65):
        assert L.pv_harmonizer_create(ctypes.byref(good), ratios, k, ctypes.byref(h)) == _lib.PV_ERR_ARG
        assert not h.value
    # both run the STANDARD pipeline only; neither takes external tables
    compat = _lib.config(1024, 4, ord("t"), 1.0, 0, 1, 10, 0)
    assert L.pv_harmonizer_create(ctypes.byref(compat), ratios, 2, ctypes.byref(h)) == _lib.PV_ERR_UNSUPPORTED
    assert L.pv_rt_create(ctypes.byref(compat), 2, ctypes.byref(h)) == _lib.PV_ERR_UNSUPPORTED
    ext = _lib.config(1024, 4, ord("p"), 1.5, 1, 1, 10, 0, tables_external=1)
    assert L.pv_harmonizer_create(ctypes.byref(ext), ratios, 2, ctypes.byref(h)) == _lib.PV_ERR_UNSUPPORTED
    assert L.pv_rt_create(ctypes.byref(ext), 2, ctypes.byref(h)) == _lib.PV_ERR_UNSUPPORTED
    # real time: natural rows only, at least one channel
    packed = _lib.config(1024, 4, ord("p"), 1.5, 1, 1, 10, 0, spec_layout=1)
    assert L.pv_rt_create(ctypes.byref(packed), 2, ctypes.byref(h)) == _lib.PV_ERR_UNSUPPORTED
    assert L.pv_rt_create(ctypes.byref(good), 0, ctypes.byref(h)) == _lib.PV_ERR_ARG
    assert not h.value
    # null harmoniser
    assert L.pv_harmonize(None, None, 0, 0, 1, 1, None, 0, None, 0, 0, None, None, 0, None) == _lib.PV_ERR_ARG
