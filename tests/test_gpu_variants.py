"""Parity of the measurement switches DESIGN.md §4.7 keeps off by default (batch_kernel.h VALU_TREE, HYBRID).

Each switch is built into a TEST-ONLY alternate library (`make -C hsig-picotls_amd alts`, part of
__graft_entry__.build()); tests/variant_case.py runs the golden length sweep, the cross-chunk dealing case and a
long-record case on it in a fresh process (PTLS_HIP_LIB) and every record must match lib/fusion.c / the oracle.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ALT = os.path.join(os.path.dirname(HERE), "hsig-picotls_amd", "alt")


@pytest.mark.parametrize("variant", ["valutree", "hybrid4"])
def test_alternate_build_parity(variant):
    lib = os.path.join(ALT, f"libptls_hip_{variant}.so")
    if not os.path.exists(lib):
        pytest.fail(f"{lib} missing: build it with `make -C hsig-picotls_amd alts` (part of __graft_entry__.build())")
    env = dict(os.environ, PTLS_HIP_LIB=lib)
    out = subprocess.run([sys.executable, os.path.join(HERE, "variant_case.py")], env=env, capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("MISMATCHES")]
    assert len(lines) == 16 and f"DONE lib={lib}" in out.stdout, out.stdout[-2000:]
    bad = [ln for ln in lines if not ln.endswith("seal=0 open=0")]
    assert not bad, bad
