"""Parity of split records (batch_kernel.h, G >= 16; planned by engine.cpp plan_splits).  When a key run has few wave
tasks for the workgroup's waves (configs[3]: 64 records per key), the planner deals the run's longest tasks as two part
tasks each: GHASH elements [0, N - B) and [N - B, N) of the task's records, part A's partial times H^B, the part that
finishes second sums both into the tag.  Every record must equal the oracle (oracle/, pinned by lib/fusion.c), open
back, fail on a tampered tag, and carry the same header-protection mask."""
import numpy as np
import pytest

import ptls_hip
from hip_helpers import HostBatch
from oracle_lib import tls_aad

pytestmark = pytest.mark.gpu


def c4_like(oracle, key_len, runs, per_run, seed, max_len=16384):
    """`runs` keys x `per_run` records of configs[3]'s lengths (64 B .. 16 KiB), key-major"""
    rng = np.random.default_rng(seed)
    recs = []
    for k in range(runs):
        key, iv = oracle.gen_key(900 + k + 10 * key_len, key_len)
        for i in range(per_run):
            L = int(rng.integers(64, max_len + 1))
            recs.append((key, iv, 64 * k + i, tls_aad(L), oracle.stream(0x5A17 + 1000 * k + i, L)))
    return recs


@pytest.mark.parametrize("key_len", [16, 32])
@pytest.mark.parametrize("lanes", [16, 32])
def test_split_records_parity(engine, oracle, lanes, key_len):
    recs = c4_like(oracle, key_len, runs=6, per_run=64 if lanes == 16 else 32, seed=lanes + key_len)
    hb = HostBatch(engine, recs)
    hb.batch.set_lanes(lanes)
    assert hb.batch.split_tasks > 0, "the planner should split this batch's longest tasks"
    outs = hb.seal(lanes)
    expect = [oracle.seal(*r) for r in recs]
    bad = [i for i, (o, e) in enumerate(zip(outs, expect)) if o != e]
    assert not bad, f"{len(bad)} of {len(recs)} sealed records differ, first {bad[:8]}"
    sealed = [bytearray(e) for e in expect]
    tampered = [0, 1, 64, len(recs) - 1]  # the longest records of the first runs are split ones
    for i in tampered:
        sealed[i][-1] ^= 0x40  # tag byte
    res, pts = hb.open([bytes(x) for x in sealed], lanes)
    for i, r in enumerate(recs):
        assert res[i] == (ptls_hip.UINT64_MAX if i in tampered else len(r[4])), i
        assert pts[i] == r[4], i  # plaintext written either way (decrypt-then-verify, lib/fusion.c:822-840)
    hb.close()


@pytest.mark.parametrize("lanes", [16, 32])
def test_split_records_across_chunks_of_one_workgroup(engine, oracle, lanes):
    """the grid capped at 2 workgroups: a key run of 40 (16 lanes) / 80 (32 lanes) tasks spans two chunks of one
    workgroup, so the split slots are numbered across chunks (sbase) and tasks carry over between them"""
    per_run = 160 if lanes == 16 else 320
    recs = c4_like(oracle, 32, runs=3, per_run=per_run, seed=77 + lanes, max_len=12000)
    hb = HostBatch(engine, recs)
    hb.batch.set_lanes(lanes)
    hb.batch.set_max_workgroups(2)
    outs = hb.seal(lanes)
    expect = [oracle.seal(*r) for r in recs]
    assert [i for i, (o, e) in enumerate(zip(outs, expect)) if o != e] == []
    res, pts = hb.open(expect, lanes)
    assert res == [len(r[4]) for r in recs] and pts == [r[4] for r in recs]
    hb.close()


def test_split_records_with_header_protection(engine, oracle):
    """seal_batch_supp over split records: the part that finishes the record computes its header-protection mask after
    the tag is written (the sample may cover the tag, lib/fusion.c:636-650)"""
    import torch
    recs = c4_like(oracle, 16, runs=4, per_run=64, seed=5)
    hb = HostBatch(engine, recs)
    hb.batch.set_lanes(16)
    assert hb.batch.split_tasks > 0
    n = len(recs)
    hp = ptls_hip.KeySet(engine, 16, 1)
    hp_key = bytes(range(16))
    hp.set(0, hp_key, None)
    supp = np.zeros(n, dtype=ptls_hip.SUPP_DTYPE)
    for i, rec in enumerate(hb.recs):
        supp[i] = (int(rec["out_off"]) + int(rec["len"]) - 4, 16 * i, 0, ptls_hip.SUPP_ENABLE)  # sample = last 4 ct + 12 tag
    d_in = torch.from_numpy(hb._input([r[4] for r in recs])).cuda()
    d_aad = torch.from_numpy(np.concatenate([hb.aad, np.zeros(16, np.uint8)])).cuda()
    d_out = torch.zeros(hb.out_total + 16, dtype=torch.uint8, device="cuda")
    d_mask = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
    hb.batch.seal_supp(hb.keyset, hp, torch.from_numpy(supp.view(np.uint8)).cuda(), d_in, d_aad, d_out, d_mask)
    torch.cuda.synchronize()
    out, mask = d_out.cpu().numpy(), d_mask.cpu().numpy()
    for i, (r, rec) in enumerate(zip(recs, hb.recs)):
        sealed = out[rec["out_off"]: rec["out_off"] + rec["len"] + 16].tobytes()
        assert sealed == oracle.seal(*r), i
        sample = out[supp[i]["sample_off"]: supp[i]["sample_off"] + 16].tobytes()
        assert mask[16 * i: 16 * i + 16].tobytes() == oracle.aes_ecb(hp_key, sample), i
    hp.close()
    hb.close()


def test_no_split_for_long_key_runs(engine, oracle):
    """a key run with many tasks per wave balances by itself: nothing is split (configs[1] / [2] shapes)"""
    recs = [(*oracle.gen_key(3, 16), i, tls_aad(8000), b"\0" * 8000) for i in range(16 * 64)]
    lens = [8000] * len(recs)
    r, *_ = ptls_hip.layout_records(lens, [5] * len(lens), [0] * len(lens), np.arange(len(lens)))
    b = ptls_hip.Batch(engine, r)
    b.set_lanes(16)
    assert b.split_tasks == 0
    b.close()
