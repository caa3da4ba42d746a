"""Parity of the batch kernel's cross-chunk dynamic dealing (batch_kernel.h `g` / `have_g` / `cbase`).

A workgroup that takes several chunks of one key run keeps drawing wave tasks from one LDS counter and carries
a drawn task into the next chunk.  With the grid capped at 2 workgroups (tests/dealing_case.py) every
workgroup takes 2-3 same-key chunks of each of 3 key runs; every record must still equal the oracle and open
back.  The same case run on the two TEST-ONLY mutant builds (hsig-picotls_amd/mutants/, DEAL_MUTANT 1: the
carried task is dropped; 2: cbase is not advanced) must FAIL, so this test is known to see that path break.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import dealing_case  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
MUTANTS = os.path.join(os.path.dirname(HERE), "hsig-picotls_amd", "mutants")


@pytest.mark.parametrize("key_len", [16, 32])
@pytest.mark.parametrize("lanes", [4, 8, 16, 32])
def test_cross_chunk_dealing_parity(engine, oracle, lanes, key_len):
    assert dealing_case.mismatches(engine, oracle, key_len, lanes) == (0, 0)


@pytest.mark.parametrize("lanes", [8, 16, 32])
@pytest.mark.parametrize("mutant", [1, 2])
def test_dealing_mutants_are_caught(mutant, lanes):
    lib = os.path.join(MUTANTS, f"libptls_hip_deal{mutant}.so")
    if not os.path.exists(lib):
        pytest.fail(f"{lib} missing: build it with `make -C hsig-picotls_amd mutants` (part of __graft_entry__.build())")
    env = dict(os.environ, PTLS_HIP_LIB=lib)
    out = subprocess.run([sys.executable, os.path.join(HERE, "dealing_case.py"), str(lanes), "16"], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    line = next(ln for ln in out.stdout.splitlines() if ln.startswith("MISMATCHES"))
    seal = int(line.split("seal=")[1].split()[0])
    assert lib in line and seal > 0, line
