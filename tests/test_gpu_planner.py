"""The launch planner's lanes-per-record choice (planner.cpp choose_lanes), pinned on the shapes it was measured on.

Descriptors only: no record bytes are touched (a Batch plans on creation), so full-size shapes cost nothing but their
descriptor upload.  The seal-rate evidence behind each row: round 5 small batches (tools/calls_r05/r05_call11.sh,
r05_call12.sh: a 64 MiB batch of 16 KiB records 207 -> 538 GiB/s seal at 32 lanes), round 4 long key runs
(tools/calls_r04/r04_call26.sh, r04_call30.sh), round 3 short key runs (tools/calls_r03/r03_call17.sh, r03_call24.sh).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import ptls_hip  # noqa: E402


def _lanes(engine, n, length, keys=1, aad=5):
    key = (np.arange(n, dtype=np.uint64) % np.uint64(keys)).astype(np.uint32)
    key = np.sort(key, kind="stable")  # same-key records adjacent, as the planner expects
    recs, _, _, _ = ptls_hip.layout_records(np.full(n, length), np.full(n, aad), key, np.arange(n), align=128)
    b = ptls_hip.Batch(engine, recs)
    try:
        return b.lanes
    finally:
        b.close()


@pytest.mark.parametrize("n,expect", [(1 << 20, 4), (262144, 4), (65536, 8), (16384, 32), (4096, 32)])
def test_lanes_for_16k_records_by_batch_size(engine, n, expect):
    """configs[1]'s 16 KiB records: 4 lanes per record at full size; smaller batches take more lanes so that the launch's
    12 waves per CU get two wave tasks each (a batch of 4 096 records is 1 024 tasks at 4 lanes for 3 072 waves)"""
    assert _lanes(engine, n, 16384) == expect


@pytest.mark.parametrize("n,expect", [(1 << 22, 4), (786432, 4), (65536, 8)])
def test_lanes_for_quic_records_by_batch_size(engine, n, expect):
    """configs[2]'s 1 350 B records (87 GHASH elements): 4 lanes; a small batch takes 8 (>= 8 elements per lane)"""
    assert _lanes(engine, n, 1350, aad=13) == expect


@pytest.mark.parametrize("per_key,expect", [(1, 64), (16, 64), (64, 32), (128, 16), (256, 8)])
def test_lanes_for_key_runs(engine, per_key, expect):
    """many keys: the wave-per-record sparse kernel below 20 records per key run, then the largest G whose chunk holds a
    whole key run (8 224-B records, 65 536 records in all)"""
    n = 65536
    assert _lanes(engine, n, 8224, keys=n // per_key) == expect
