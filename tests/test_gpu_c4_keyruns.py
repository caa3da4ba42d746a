"""configs[3]'s own execution path pinned against lib/fusion.c (VERDICT r04 "next round" item 1a).

tests/c4_keyruns_case.py seals whole key runs of configs[3] (keys 0..255 x 64 records, AES-256, mixed lengths) in
key-run order, as the full config is laid out: the planner must pick the 32-lane batch kernel (not the sparse kernel
the config samples of test_gpu_parity.py take), every digest must equal lib/fusion.c's (tests/golden/c4_keyruns.npy),
every record must open back, and one flipped tag per key run must fail exactly there.

Each key run is ONE chunk here (64 records = 32 wave tasks = the chunk cap), exactly as in the full config: configs[3]'s
path is the key switch (table rebuild + task-counter reset between two barriers), not the cross-chunk task carry that
tests/test_gpu_dealing.py pins.  So on the TEST-ONLY mutants (hsig-picotls_amd/mutants/, rebuilt at 8, 16 and 32 lanes)
the case must FAIL with DEAL_MUTANT 3 (the task counter not reset at a key switch after
the workgroup's first key) and is expected to PASS with 1 and 2
(cross-chunk carry broken: a path configs[3] never takes), which the test asserts too, so a planner change that starts
splitting c4's key runs shows up here.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import c4_keyruns_case  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
MUTANTS = os.path.join(os.path.dirname(HERE), "hsig-picotls_amd", "mutants")


@pytest.fixture(scope="module")
def c4_records(oracle):
    return c4_keyruns_case.records(oracle)


@pytest.mark.parametrize("max_wg", [0, 1, 3])
def test_c4_key_runs_match_fusion(engine, oracle, c4_records, max_wg):
    """max_wg 0: the planner's own grid (one workgroup per CU, chunks from the device-wide queue), as bench.py runs
    configs[3]; 1 and 3: every workgroup takes many key runs in turn (a key switch at every chunk)"""
    r = c4_keyruns_case.run(engine, oracle, max_wg, c4_records)
    assert r["lanes"] == 32 and r["chunks"] == 256, r  # one chunk per key run
    assert (r["seal"], r["open"], r["tamper"]) == (0, 0, 0), r


@pytest.mark.parametrize("mutant", [1, 2, 3])
def test_c4_key_runs_dealing_mutants(mutant):
    lib = os.path.join(MUTANTS, f"libptls_hip_deal{mutant}.so")
    if not os.path.exists(lib):
        pytest.fail(f"{lib} missing: build it with `make -C hsig-picotls_amd mutants` (part of __graft_entry__.build())")
    env = dict(os.environ, PTLS_HIP_LIB=lib)
    out = subprocess.run([sys.executable, os.path.join(HERE, "c4_keyruns_case.py"), "1"], env=env, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    line = next(ln for ln in out.stdout.splitlines() if ln.startswith("MISMATCHES"))
    seal = int(line.split("seal=")[1].split()[0])
    assert lib in line and "lanes=32" in line and "chunks=256" in line, line
    assert (seal > 0) == (mutant == 3), line
