"""CPU-side checks of the C-ABI library (no GPU compute): it loads, exports every entry point
include/ggml-mi355x.h declares, and its ggml plugin symbols are the ones the reference loader
dlsym()s (src/ggml-backend-reg.cpp:248, :256)."""
import ctypes
import os
import subprocess

import pytest

import mi355x_qmm as M


@pytest.fixture(scope="module")
def lib():
    M.build()
    return M.lib()


def test_header_declares_boundary():
    names = M.exported_api()
    for must in ("ggml_backend_init", "ggml_backend_score", "ggml_backend_mi355x_reg",
                 "ggml_mi355x_mul_mat", "ggml_mi355x_mul_mat_id", "ggml_mi355x_dequantize"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    for name in M.exported_api():
        assert hasattr(lib, name), f"{name} declared in include/ggml-mi355x.h but not exported"


def test_dynamic_symbol_table():
    out = subprocess.run(["nm", "-D", "--defined-only", M.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(M.exported_api()) <= exported
    # the library must not leak internal C++ symbols into the loader's namespace
    assert not any(s.startswith("_ZN6mi355x") for s in exported)


def test_no_unresolved_internal_symbols():
    """every kernel launch stub and internal function is defined inside the library (a template
    kernel whose host stub the compiler dropped would only fail at dlopen on the GPU box)"""
    out = subprocess.run(["nm", "-D", "--undefined-only", M.LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert "mi355x" not in out, [l for l in out.splitlines() if "mi355x" in l]


def test_code_object_targets_gfx950_only():
    """every embedded device code object is for gfx950 (no other arch, no dual paths)"""
    import re
    blob = open(M.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa-[-a-z0-9:+]*", blob))
    assert targets, "no device code embedded"
    assert all(t.endswith(b"gfx950") for t in targets), targets


def test_strerror_and_no_device_score(lib):
    assert lib.ggml_mi355x_strerror(0) == b"ok"
    assert b"shape" in lib.ggml_mi355x_strerror(-1)
    if not os.path.exists("/dev/kfd"):
        assert lib.ggml_backend_score() == 0
        assert lib.ggml_mi355x_device_count() == 0
