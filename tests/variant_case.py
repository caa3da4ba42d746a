"""Parity cases for the TEST-ONLY alternate builds of the batch kernel (hsig-picotls_amd/alt/, used by
tests/test_gpu_variants.py).

DESIGN.md §4.7 keeps two measured-and-rejected designs behind compile-time switches that are off in the product
build: VALU_TREE=1 (the G <= 16 partial sums combined by one VALU multiply per lane instead of the nibble-table
tree) and HYBRID=4 (the last 4 waves of a workgroup run their full-block stretch as bit-sliced AES).  Run as a
script under PTLS_HIP_LIB=<alternate build> it prints one MISMATCHES line per case:
  sweep   the golden length sweep (tests/golden/sweep.json, lib/fusion.c digests) at 4 / 8 / 16 lanes per record;
  deal    the cross-chunk dealing case of tests/dealing_case.py (grid capped at 2 workgroups);
  long    one key run per key size of 2-17 KiB records with the grid capped at 2 workgroups, so every wave of a
          workgroup (the bit-sliced ones included) takes full-block stretches.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(HERE, "golden"), os.path.join(ROOT, "hsig-picotls_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

LANES = (4, 8, 16)


def sweep_case(engine, oracle, key_len, lanes):
    from hip_helpers import HostBatch
    from make_golden import sweep_inputs
    with open(os.path.join(HERE, "golden", "sweep.json")) as f:
        vecs = [v for v in json.load(f)["vectors"] if v["key_len"] == key_len]
    recs = [sweep_inputs(oracle, v["idx"], key_len, v["L"], v["A"]) for v in vecs]
    hb = HostBatch(engine, recs)
    outs = hb.seal(lanes)
    bad_seal = sum(1 for v, o in zip(vecs, outs) if hashlib.sha256(o).hexdigest() != v["sha256"])
    res, pts = hb.open(outs, lanes)
    bad_open = sum(1 for v, r, x, p in zip(vecs, recs, res, pts) if x != v["L"] or p != r[4])
    hb.close()
    return bad_seal, bad_open


def long_case(engine, oracle, key_len, lanes):
    from hip_helpers import HostBatch
    from oracle_lib import tls_aad
    rng = np.random.default_rng(4242 + key_len + lanes)
    key, iv = oracle.gen_key(900 + key_len, key_len)
    recs = []
    for i in range(160):
        L = int(rng.integers(2048, 17 * 1024))
        recs.append((key, iv, i, tls_aad(L), oracle.stream(9000 + i, L)))
    hb = HostBatch(engine, recs)
    hb.batch.set_max_workgroups(2)
    outs = hb.seal(lanes)
    expect = [oracle.seal(*r) for r in recs]
    bad_seal = sum(1 for o, e in zip(outs, expect) if o != e)
    res, pts = hb.open(expect, lanes)
    bad_open = sum(1 for r, x, p in zip(recs, res, pts) if x != len(r[4]) or p != r[4])
    hb.close()
    return bad_seal, bad_open


def main():
    import torch
    # torch first: its HIP runtime must be the process's one before libptls_hip.so loads (tests/dealing_case.py)
    assert torch.cuda.is_available()
    import dealing_case
    import ptls_hip
    from oracle_lib import Oracle
    eng, o = ptls_hip.Engine(0), Oracle()
    for key_len in (16, 32):
        for lanes in LANES:
            for name, fn in (("sweep", sweep_case), ("deal", dealing_case.mismatches), ("long", long_case)):
                if name == "deal" and lanes == 4:
                    continue
                s, p = fn(eng, o, key_len, lanes)
                print(f"MISMATCHES case={name} key_len={key_len} lanes={lanes} seal={s} open={p}", flush=True)
    eng.close()
    print(f"DONE lib={ptls_hip.LIB_PATH}", flush=True)


if __name__ == "__main__":
    main()
