"""The key setup's fast GF(2^128) forms (hsig-picotls_amd/csrc/gf128.h: multiply by x^s with one fold, squaring by bit
spreading, 4-bit window products from the basis plane) against the SP 800-38D bit-serial product, compiled for the host
(no GPU).  3 000 random pairs plus edge values."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_gf128_forms_match_bit_serial(tmp_path):
    exe = tmp_path / "gf128_check"
    subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "hsig-picotls_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "gf128_check.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr
