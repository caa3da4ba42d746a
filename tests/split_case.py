"""Parity cases of split records (batch_kernel.h SPLIT_TASKS; planned by engine.cpp plan_splits), run under
PTLS_HIP_LIB=hsig-picotls_amd/alt/libptls_hip_split.so by tests/test_gpu_split.py (the switch is off in the product:
DESIGN.md §4.7 "split records").  When a key run has few wave tasks for the workgroup's waves (configs[3]: 64 records
per key), that build deals the run's longest tasks as two part tasks each: GHASH elements [0, N - B) and [N - B, N) of
the task's records, part A's partial times H^B, the part that finishes second sums both into the tag.  One line per
case: MISMATCHES case=... split_tasks=<planned part pairs> seal=<records != oracle> open=<bad results or plaintexts>."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(ROOT, "hsig-picotls_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def c4_like(oracle, key_len, runs, per_run, seed, max_len=16384):
    """`runs` keys x `per_run` records of configs[3]'s lengths (64 B .. 16 KiB), key-major"""
    from oracle_lib import tls_aad
    rng = np.random.default_rng(seed)
    recs = []
    for k in range(runs):
        key, iv = oracle.gen_key(900 + k + 10 * key_len, key_len)
        for i in range(per_run):
            L = int(rng.integers(64, max_len + 1))
            recs.append((key, iv, 64 * k + i, tls_aad(L), oracle.stream(0x5A17 + 1000 * k + i, L)))
    return recs


def parity_case(engine, oracle, key_len, lanes, max_wg=0, runs=6, per_run=None, max_len=16384):
    """seal == oracle, open back, and a flipped tag byte fails on split and whole records alike"""
    import ptls_hip
    from hip_helpers import HostBatch
    per_run = per_run or (64 if lanes == 16 else 32)
    recs = c4_like(oracle, key_len, runs, per_run, seed=lanes + key_len + max_wg, max_len=max_len)
    hb = HostBatch(engine, recs)
    hb.batch.set_lanes(lanes)
    if max_wg:
        hb.batch.set_max_workgroups(max_wg)
    nsplit = hb.batch.split_tasks
    outs = hb.seal(lanes)
    expect = [oracle.seal(*r) for r in recs]
    bad_seal = sum(1 for o, e in zip(outs, expect) if o != e)
    sealed = [bytearray(e) for e in expect]
    tampered = {0, 1, per_run, len(recs) - 1}
    for i in tampered:
        sealed[i][-1] ^= 0x40  # a tag byte
    res, pts = hb.open([bytes(x) for x in sealed], lanes)
    bad_open = sum(1 for i, r in enumerate(recs)
                   if res[i] != (ptls_hip.UINT64_MAX if i in tampered else len(r[4])) or pts[i] != r[4])
    hb.close()
    return nsplit, bad_seal, bad_open


def supp_case(engine, oracle):
    """seal_batch_supp over split records: the part that finishes a record computes its header-protection mask after
    the tag is written (the sample covers the tag, lib/fusion.c:636-650)"""
    import torch
    import ptls_hip
    from hip_helpers import HostBatch
    recs = c4_like(oracle, 16, runs=4, per_run=64, seed=5)
    hb = HostBatch(engine, recs)
    hb.batch.set_lanes(16)
    nsplit = hb.batch.split_tasks
    n = len(recs)
    hp = ptls_hip.KeySet(engine, 16, 1)
    hp_key = bytes(range(16))
    hp.set(0, hp_key, None)
    supp = np.zeros(n, dtype=ptls_hip.SUPP_DTYPE)
    for i, rec in enumerate(hb.recs):
        supp[i] = (int(rec["out_off"]) + int(rec["len"]) - 4, 16 * i, 0, ptls_hip.SUPP_ENABLE)  # last 4 ct + 12 tag bytes
    d_in = torch.from_numpy(hb._input([r[4] for r in recs])).cuda()
    d_aad = torch.from_numpy(np.concatenate([hb.aad, np.zeros(16, np.uint8)])).cuda()
    d_out = torch.zeros(hb.out_total + 16, dtype=torch.uint8, device="cuda")
    d_mask = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
    hb.batch.seal_supp(hb.keyset, hp, torch.from_numpy(supp.view(np.uint8)).cuda(), d_in, d_aad, d_out, d_mask)
    torch.cuda.synchronize()
    out, mask = d_out.cpu().numpy(), d_mask.cpu().numpy()
    bad_seal = bad_mask = 0
    for i, (r, rec) in enumerate(zip(recs, hb.recs)):
        bad_seal += out[rec["out_off"]: rec["out_off"] + rec["len"] + 16].tobytes() != oracle.seal(*r)
        sample = out[supp[i]["sample_off"]: supp[i]["sample_off"] + 16].tobytes()
        bad_mask += mask[16 * i: 16 * i + 16].tobytes() != oracle.aes_ecb(hp_key, sample)
    hp.close()
    hb.close()
    return nsplit, bad_seal, bad_mask


def main():
    """`split_case.py runs`: configs[3]-shaped key runs at 16 / 32 lanes and header protection (the default threshold);
    `split_case.py chunks` (run with PTLS_HIP_SPLIT_PCT=20, a low threshold): key runs of 40 tasks that span two
    chunks of one workgroup (grid capped at 2), so the split slots are numbered across chunks"""
    import torch
    assert torch.cuda.is_available()  # torch's HIP runtime first (tests/dealing_case.py)
    import ptls_hip
    from oracle_lib import Oracle
    eng, o = ptls_hip.Engine(0), Oracle()
    which = sys.argv[1] if len(sys.argv) > 1 else "runs"
    if which == "runs":
        for key_len in (16, 32):
            for lanes in (16, 32):
                ns, s, p = parity_case(eng, o, key_len, lanes)
                print(f"MISMATCHES case=runs key_len={key_len} lanes={lanes} split_tasks={ns} seal={s} open={p}", flush=True)
        ns, s, p = supp_case(eng, o)
        print(f"MISMATCHES case=supp key_len=16 lanes=16 split_tasks={ns} seal={s} open={p}", flush=True)
    else:
        for lanes in (16, 32):
            ns, s, p = parity_case(eng, o, 32, lanes, max_wg=2, runs=3, per_run=160 if lanes == 16 else 80, max_len=12000)
            print(f"MISMATCHES case=chunks key_len=32 lanes={lanes} split_tasks={ns} seal={s} open={p}", flush=True)
    eng.close()
    print(f"DONE lib={ptls_hip.LIB_PATH}", flush=True)


if __name__ == "__main__":
    main()
