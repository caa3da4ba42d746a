"""BASELINE configs[3]'s real execution path under parity (used by tests/test_gpu_c4_keyruns.py).

configs[3] is 4M mixed-length (64 B - 16 KiB) AES-256 records over 64K keys: 64 records per key.  The planner
(planner.cpp choose_lanes) runs such key runs on the 32-lane batch kernel, each run one chunk of 32 wave tasks (the
chunk cap: bench.py's full shape and this one plan the same chunks), so every chunk is a key switch: a workgroup
rebuilds the key's GHASH tables and resets its task counter between two barriers (batch_kernel.h).  The config samples
of tests/golden/configs.json hold <= 8 records per key, which the planner sends to the sparse kernel instead, so this
case seals WHOLE key runs: keys 0..255, every one of their 64 records, in key-run order, compared with lib/fusion.c's
digests in tests/golden/c4_keyruns.npy; opened back; one tag per key run flipped.

Run as a script (`python c4_keyruns_case.py MAX_WG`) it prints the mismatch counts for whichever libptls_hip.so
PTLS_HIP_LIB names: tests/test_gpu_c4_keyruns.py runs it on the TEST-ONLY dealing mutants and expects failures.
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(HERE, "golden"), os.path.join(ROOT, "hsig-picotls_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

UINT64_MAX = (1 << 64) - 1


def records(oracle):
    from make_golden import CONFIGS, c4_keyrun_index, config_record
    cfg = CONFIGS["c4_mixed_aes256_64k"]
    return [config_record(oracle, cfg, i) for i in c4_keyrun_index()]


def digests():
    return np.load(os.path.join(HERE, "golden", "c4_keyruns.npy"), allow_pickle=False)


def run(engine, oracle, max_wg=0, recs=None):
    """dict(lanes, chunks, seal, open, tamper): the planner's lanes and chunk count, and the numbers of records whose
    sealed digest, open result / plaintext or tampered-open result is wrong; max_wg > 0 caps the grid (every workgroup
    then takes many key runs in turn)"""
    from hip_helpers import HostBatch
    from make_golden import C4_KEYRUN_LEN
    recs = records(oracle) if recs is None else recs
    dig = digests()
    hb = HostBatch(engine, recs)
    try:
        if max_wg:
            hb.batch.set_max_workgroups(max_wg)
        outs = hb.seal()
        lanes, chunks = hb.batch.lanes, hb.batch.chunks
        bad_seal = sum(1 for k, o in enumerate(outs) if hashlib.sha256(o).digest() != dig[k].tobytes())
        res, pts = hb.open(outs)
        bad_open = sum(1 for r, x, p in zip(recs, res, pts) if x != len(r[4]) or p != r[4])
        # one flipped tag byte per key run, at a different record and byte each time
        flip = {j * C4_KEYRUN_LEN + (7 * j) % C4_KEYRUN_LEN: j % 16 for j in range(len(recs) // C4_KEYRUN_LEN)}
        bad = list(outs)
        for k, b in flip.items():
            t = bytearray(bad[k])
            t[len(t) - 16 + b] ^= 0x40
            bad[k] = bytes(t)
        res2, _ = hb.open(bad)
        bad_tamper = sum(1 for k, (r, x) in enumerate(zip(recs, res2)) if x != (UINT64_MAX if k in flip else len(r[4])))
    finally:
        hb.close()
    return dict(lanes=lanes, chunks=chunks, seal=bad_seal, open=bad_open, tamper=bad_tamper)


def main():
    max_wg = int(sys.argv[1])
    import torch
    # torch first: its HIP runtime must be the process's one before libptls_hip.so loads (tests/conftest.py's order)
    assert torch.cuda.is_available()
    import ptls_hip
    from oracle_lib import Oracle
    eng = ptls_hip.Engine(0)
    r = run(eng, Oracle(), max_wg)
    eng.close()
    print(f"MISMATCHES seal={r['seal']} open={r['open']} tamper={r['tamper']} lanes={r['lanes']} chunks={r['chunks']} "
          f"lib={ptls_hip.LIB_PATH}", flush=True)


if __name__ == "__main__":
    main()
