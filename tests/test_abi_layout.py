"""The plugin's restatement of the ggml backend ABI (ggml-gfx906_amd/csrc/ggml_abi.h) against the
reference's headers: oracle/abi_check.cpp is compiled once per side and both listings of struct
sizes, field offsets and enum values must be identical (CPU-only; needs /root/reference, which
exists in the build container, not on the GPU box)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
SRC = os.path.join(ROOT, "oracle", "abi_check.cpp")


def _listing(tmp_path, side: str, incs) -> str:
    exe = str(tmp_path / f"abi_{side}")
    cmd = ["g++", "-std=c++17", f"-DSIDE_{side}", SRC, "-o", exe] + [f"-I{i}" for i in incs]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return subprocess.run([exe], check=True, capture_output=True, text=True).stdout


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src")), reason="reference sources not present")
def test_abi_restatement_matches_reference(tmp_path):
    ref = _listing(tmp_path, "REF", [os.path.join(REF, "include"), os.path.join(REF, "src")])
    ours = _listing(tmp_path, "OURS", [os.path.join(ROOT, "ggml-gfx906_amd", "csrc")])
    assert ref.count("\n") > 100
    diff = [(a, b) for a, b in zip(ref.splitlines(), ours.splitlines()) if a != b]
    assert not diff, diff[:10]
    assert ref == ours
