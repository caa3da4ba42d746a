"""The chunk-queue slots are reused correctly.

Every batch-kernel and sparse-kernel launch takes the next of the engine's queue slots (engine.cpp queue_slot) round
robin: two words {next chunk / record, workgroups done} that must be zero when handed out.  No launch zeroes them first:
the kernel's last workgroup to draw past the end resets both (batch_kernel.h next_chunk, sparse_kernel.hip).  If that
reset ever failed, every later launch on the slot would find its queue exhausted and skip chunks or records, leaving
their output unwritten.  So: one batch sealed over and over on every kernel that takes a slot (32, 8 and 4 lanes per
record, the sparse kernel), the output zeroed before every launch and compared with the oracle's after it, long past the
point where every slot has been reused:

* on an engine whose round robin has only 3 slots (PTLS_HIP_QUEUE_SLOTS), so each slot serves every kernel in turn;
* on a default engine, for more launches than its 4 096 slots.
"""
import os

import numpy as np
import pytest
import torch

import ptls_hip
from oracle_lib import tls_aad

pytestmark = pytest.mark.gpu
LANES = (32, 8, 4, 64)  # 64: the sparse kernel


def _workload(oracle):
    rng = np.random.default_rng(4242)
    recs = []
    for k, n in enumerate((400, 250, 350)):
        key, iv = oracle.gen_key(300 + k, 16)
        for i in range(n):
            L = int(rng.integers(0, 3000))
            recs.append((key, iv, 1000 * k + i, tls_aad(L), oracle.stream(600 + 1000 * k + i, L)))
    return recs


class Case:
    def __init__(self, engine, oracle):
        recs = _workload(oracle)
        lens = [len(r[4]) for r in recs]
        slot = [0] * 400 + [1] * 250 + [2] * 350
        d, in_total, out_total, aad_total = ptls_hip.layout_records(lens, [5] * len(recs), slot, [r[2] for r in recs])
        self.ks = ptls_hip.KeySet(engine, 16, 3)
        keys = [oracle.gen_key(300 + k, 16) for k in range(3)]
        self.ks.set(0, b"".join(k for k, _ in keys), b"".join(v for _, v in keys))
        h_in, h_aad, h_exp = (np.zeros(t + 64, np.uint8) for t in (in_total, aad_total, out_total))
        for r, e in zip(recs, d):
            h_in[e["in_off"]: e["in_off"] + e["len"]] = np.frombuffer(r[4], np.uint8)
            h_aad[e["aad_off"]: e["aad_off"] + 5] = np.frombuffer(r[3], np.uint8)
            h_exp[e["out_off"]: e["out_off"] + e["len"] + 16] = np.frombuffer(oracle.seal(*r), np.uint8)
        self.d_in, self.d_aad, self.d_exp = (torch.from_numpy(a).cuda() for a in (h_in, h_aad, h_exp))
        self.d_out = torch.zeros_like(self.d_exp)
        self.batches = []
        for lanes in LANES:
            b = ptls_hip.Batch(engine, d)
            b.set_lanes(lanes)
            assert b.lanes == lanes and b.grid > 1
            self.batches.append(b)
        self.bad = torch.zeros(len(LANES), dtype=torch.int64, device="cuda")

    def launches(self, rounds):
        """rounds x len(LANES) seal launches, each checked against the oracle's output on the device (no host sync)"""
        for _ in range(rounds):
            for j, b in enumerate(self.batches):
                self.d_out.zero_()
                b.seal(self.ks, self.d_in, self.d_aad, self.d_out)
                self.bad[j] += (self.d_out != self.d_exp).any().to(torch.int64)
        torch.cuda.synchronize()
        return dict(zip(LANES, self.bad.cpu().tolist()))

    def close(self):
        for b in self.batches:
            b.close()
        self.ks.close()


def test_queue_slots_reused_every_few_launches(oracle):
    os.environ["PTLS_HIP_QUEUE_SLOTS"] = "3"
    try:
        eng = ptls_hip.Engine(0)
    finally:
        del os.environ["PTLS_HIP_QUEUE_SLOTS"]
    c = Case(eng, oracle)
    try:
        assert c.launches(60) == {lanes: 0 for lanes in LANES}  # 240 launches over 3 slots
    finally:
        c.close()
        eng.close()


def test_more_launches_than_queue_slots(engine, oracle):
    c = Case(engine, oracle)
    try:
        assert c.launches(1030) == {lanes: 0 for lanes in LANES}  # 4 120 launches > 4 096 slots
    finally:
        c.close()
