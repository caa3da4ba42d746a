"""CPU tests: the oracle (oracle/aesgcm_oracle.c) against the reference's golden vectors.

The oracle is only trusted because these pass: every KAT of t/fusion.c, every sweep vector and every
per-config sample that lib/fusion.c itself produced (tests/golden/make_golden.py), and -- when the
reference build oracle/_ref is present -- randomized differential runs against lib/fusion.c in-process.
"""
import hashlib
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from make_golden import CONFIGS, config_record, sweep_inputs  # noqa: E402
from oracle_lib import Ref  # noqa: E402


def test_ecb_kats(oracle, golden):
    for v in golden["kats"]["ecb"]:  # t/fusion.c:71-85
        assert oracle.aes_ecb(bytes.fromhex(v["key"]), bytes.fromhex(v["pt"])).hex() == v["ct"]


def test_gfmul_kats_fusion_domain(oracle, golden):
    g = golden["kats"]["gfmul"]  # t/fusion.c:87-233 (H and result in fusion's transformH domain)
    for c in g["cases"]:
        assert oracle.fusion_domain_ghash(bytes.fromhex(g["H_fusion"]), bytes.fromhex(c["blocks"])).hex() == c["lo"]


def test_aead_kats(oracle, golden):
    for v in golden["kats"]["aead"]:  # gcm_basic, gcm_capacity
        args = (bytes.fromhex(v["key"]), bytes.fromhex(v["iv"]), v["seq"], bytes.fromhex(v["aad"]), bytes.fromhex(v["pt"]))
        out = oracle.seal(*args)
        assert out.hex() == v["out"], v["name"]
        assert oracle.open(*args[:4], out) == (len(args[4]), args[4])


def test_gcm_test_vectors_and_supp(oracle, golden):
    """t/fusion.c:289-343 incl. the supplementary (QUIC header protection) block: AES-ECB(01*16, out[2:18])"""
    for v in golden["kats"]["gcm_test_vectors"]:
        out = oracle.seal(bytes(16), bytes(12), 0, bytes(v["aadlen"]), bytes(v["ptlen"]))
        assert out[v["ptlen"]:].hex() == v["tag"]
        assert oracle.aes_ecb(b"\x01" * 16, out[2:18]).hex() == v["supp"]


def test_iv96(oracle, golden):
    v, basic2 = golden["kats"]["gcm_iv96"], golden["kats"]["aead"][1]
    iv = bytes(a ^ b for a, b in zip(bytes.fromhex(v["iv"]), bytes.fromhex(v["xor"]).ljust(12, b"\0")))
    out = oracle.seal(bytes.fromhex(v["key"]), iv, 0, bytes.fromhex(basic2["aad"]), bytes.fromhex(basic2["pt"]))
    assert out.hex() == basic2["out"]
    bad = bytes(a ^ b for a, b in zip(iv, bytes.fromhex(v["bad_xor"]).ljust(12, b"\0")))
    assert oracle.open(bytes.fromhex(v["key"]), bad, 0, bytes.fromhex(basic2["aad"]), out)[0] is None


def test_tamper_and_short_input(oracle):
    key, iv = bytes(range(16)), bytes(12)
    out = oracle.seal(key, iv, 5, b"aad", b"payload bytes")
    for pos in (0, len(out) - 1, len(out) - 17):
        bad = bytearray(out)
        bad[pos] ^= 0x80
        assert oracle.open(key, iv, 5, b"aad", bytes(bad))[0] is None
    assert oracle.open(key, iv, 5, b"aad", out[:15])[0] is None  # inlen < 16 -> SIZE_MAX (lib/fusion.c:1156)
    assert oracle.open(key, iv, 6, b"aad", out)[0] is None       # wrong seq


def test_length_sweep(oracle, golden):
    for v in golden["sweep"]["vectors"]:
        r = sweep_inputs(oracle, v["idx"], v["key_len"], v["L"], v["A"])
        out = oracle.seal(*r)
        assert hashlib.sha256(out).hexdigest() == v["sha256"], v["idx"]
        if "out" in v:
            assert out.hex() == v["out"]
        assert oracle.open(*r[:4], out) == (v["L"], r[4])


@pytest.mark.parametrize("name", list(CONFIGS))
def test_config_samples(oracle, golden, name):
    cfg = golden["configs"]["configs"][name]
    for rec in cfg["records"][:: 4 if name.startswith("c2") else 1]:
        out = oracle.seal(*config_record(oracle, CONFIGS[name], rec["i"]))
        assert hashlib.sha256(out).hexdigest() == rec["sha256"], rec["i"]


def test_c4_keyruns_fixture(oracle, golden):
    """tests/golden/c4_keyruns.npy (configs[3]'s whole key runs 0..255, lib/fusion.c digests): the oracle matches every
    record of key runs 0, 1 and 255 and the first record of every run; the runs' records that configs.json also holds
    (record i < 64: the first record of key run i) carry the same digest there"""
    from make_golden import C4_KEYRUN_LEN, c4_keyrun_index
    dig = np.load(os.path.join(HERE, "golden", "c4_keyruns.npy"), allow_pickle=False)
    idx = c4_keyrun_index()
    assert dig.shape == (len(idx), 32) and len(idx) == 256 * C4_KEYRUN_LEN
    cfg = CONFIGS["c4_mixed_aes256_64k"]
    check = set(range(0, len(idx), C4_KEYRUN_LEN)) | set(range(2 * C4_KEYRUN_LEN)) | set(range(len(idx) - C4_KEYRUN_LEN, len(idx)))
    for k in sorted(check):
        out = oracle.seal(*config_record(oracle, cfg, idx[k]))
        assert hashlib.sha256(out).digest() == dig[k].tobytes(), idx[k]
    sample = {r["i"]: r["sha256"] for r in golden["configs"]["configs"]["c4_mixed_aes256_64k"]["records"]}
    shared = [k for k, i in enumerate(idx) if i in sample]
    assert len(shared) == 64
    for k in shared:
        assert dig[k].tobytes().hex() == sample[idx[k]]


def test_generator_matches_bench(oracle):
    """bench.py's vectorised splitmix64 workload generator == the oracle's scalar one"""
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    idx = np.array([0, 1, 12345, (1 << 20) - 1], dtype=np.uint64)
    got = bench.stream_bytes(np.uint64(bench.SEED_DATA) ^ idx, 100)
    for i, row in zip(idx, got):
        assert row.tobytes() == oracle.gen_record(int(i), 100)
    keys, ivs = bench.make_keys(dict(keys=3, key_len=32))
    for j in range(3):
        k, iv = oracle.gen_key(j, 32)
        assert keys[32 * j: 32 * j + 32] == k and ivs[12 * j: 12 * j + 12] == iv
    lens = np.uint64(64) + bench.splitmix_at(np.uint64(bench.SEED_LEN) ^ idx, 0) % np.uint64(16321)
    assert [int(x) for x in lens] == [oracle.mixed_len(int(i)) for i in idx]


@pytest.mark.skipif(not Ref.available, reason="oracle/_ref (reference build) not present")
def test_differential_vs_reference(oracle):
    """t/fusion.c test_generated (:384-465) shape: random keys/ivs/seq/aad/text < 256, both directions,
    both key sizes, plus longer texts; oracle vs lib/fusion.c in-process."""
    ref = Ref()
    rng = np.random.default_rng(2024)
    for key_len in (16, 32):
        for i in range(1500):
            key = rng.integers(0, 256, key_len, dtype=np.uint8).tobytes()
            iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
            seq = int(rng.integers(0, 2 ** 63))
            aad = rng.integers(0, 256, int(rng.integers(0, 256)), dtype=np.uint8).tobytes()
            n = int(rng.integers(0, 256)) if i % 10 else int(rng.integers(256, 5000))
            text = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            a = oracle.seal(key, iv, seq, aad, text)
            assert a == ref.seal(key, iv, seq, aad, text)
            assert ref.open(key, iv, seq, aad, a) == (n, text)
            assert oracle.open(key, iv, seq, aad, ref.seal(key, iv, seq, aad, text)) == (n, text)


@pytest.mark.skipif(not Ref.available, reason="oracle/_ref (reference build) not present")
def test_supp_vs_reference(oracle):
    ref = Ref()
    rng = np.random.default_rng(5)
    for key_len in (16, 32):
        for _ in range(50):
            key = rng.integers(0, 256, key_len, dtype=np.uint8).tobytes()
            hp = rng.integers(0, 256, key_len, dtype=np.uint8).tobytes()
            text = rng.integers(0, 256, int(rng.integers(20, 300)), dtype=np.uint8).tobytes()
            off = int(rng.integers(0, len(text) - 4))
            out, supp = ref.seal_supp(key, bytes(12), 1, b"hdr", text, hp, off)
            assert out == oracle.seal(key, bytes(12), 1, b"hdr", text)
            assert supp == oracle.aes_ecb(hp, out[off:off + 16])
