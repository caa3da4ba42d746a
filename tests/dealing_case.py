"""The batch kernel's cross-chunk task dealing under parity (used by tests/test_gpu_dealing.py).

The batch kernel's waves draw wave tasks from a workgroup counter that runs across all chunks of one key run
that the workgroup takes (batch_kernel.h: `g`, `have_g`, `cbase`).  That carry only happens when a workgroup
gets two or more chunks of the same key, which a full-device launch of a small test batch never does.  Here the
grid is capped at 2 workgroups (ptls_hip_batch_set_max_workgroups), so with key runs of 300-1200 records each
workgroup takes 2-3 consecutive chunks of every run.

Run as a script (`python dealing_case.py LANES KEY_LEN`) it prints the number of records whose sealed bytes or
open result differ from the oracle, for whichever libptls_hip.so PTLS_HIP_LIB names: the test runs it on the
TEST-ONLY mutant builds (hsig-picotls_amd/mutants/) and expects a non-zero count.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(ROOT, "hsig-picotls_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

RUNS = (1200, 300, 800)  # records per key run, in this order in the batch
MAX_WG = 2


def records(oracle, key_len, seed=0):
    rng = np.random.default_rng(1000 + key_len + seed)
    from oracle_lib import tls_aad
    recs = []
    for k, n in enumerate(RUNS):
        key, iv = oracle.gen_key(700 + k, key_len)
        for i in range(n):
            L = int(rng.integers(0, 3000))
            recs.append((key, iv, 5000 * k + i, tls_aad(L), oracle.stream(31 * k + i + 17 * seed, L)))
    return recs


def mismatches(engine, oracle, key_len, lanes):
    """(sealed records != oracle, opened records with a wrong result or plaintext), grid capped at MAX_WG"""
    from hip_helpers import HostBatch
    recs = records(oracle, key_len)
    hb = HostBatch(engine, recs)
    hb.batch.set_max_workgroups(MAX_WG)
    outs = hb.seal(lanes)
    expect = [oracle.seal(*r) for r in recs]
    bad_seal = sum(1 for o, e in zip(outs, expect) if o != e)
    res, pts = hb.open(expect, lanes)
    bad_open = sum(1 for r, x, p in zip(recs, res, pts) if x != len(r[4]) or p != r[4])
    hb.close()
    return bad_seal, bad_open


def main():
    lanes, key_len = int(sys.argv[1]), int(sys.argv[2])
    import torch
    # torch first: its HIP runtime must be the process's one before libptls_hip.so loads (the same order as
    # tests/conftest.py's engine fixture and bench.py; the other order leaves torch with "No HIP GPUs")
    assert torch.cuda.is_available()
    import ptls_hip
    from oracle_lib import Oracle
    eng = ptls_hip.Engine(0)
    bad_seal, bad_open = mismatches(eng, Oracle(), key_len, lanes)
    eng.close()
    print(f"MISMATCHES seal={bad_seal} open={bad_open} lib={ptls_hip.LIB_PATH}", flush=True)


if __name__ == "__main__":
    main()
