"""Parity of the MI355X kernels (through the C ABI of libptls_hip.so) with the reference engine.

Pins: tests/golden/*.json were produced by running lib/fusion.c itself (tests/golden/make_golden.py);
the CPU oracle (oracle/) is used as a checker for data the fixtures do not cover.  Bar: bit-exact.
Shapes follow the reference's own tests (t/fusion.c): KATs, length sweep incl. partial blocks and
empty AAD/payload, iv96, tamper -> SIZE_MAX, differential runs, plus the batch-only cases (mixed
keys / lengths in one launch, lanes-per-record variants, unaligned and in-place layouts).
"""
import hashlib
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import ptls_hip  # noqa: E402

TRANSPORTS = {"copy": ptls_hip.TRANSPORT_COPY, "mapped": ptls_hip.TRANSPORT_MAPPED}  # host pipeline transports
from hip_helpers import HostBatch  # noqa: E402
from make_golden import CONFIGS, config_record, sweep_inputs  # noqa: E402
from oracle_lib import tls_aad  # noqa: E402

UINT64_MAX = (1 << 64) - 1
LANES = (1, 2, 4, 8, 16, 32, 64)  # 64: the wave-per-record sparse-key kernel


def kat_records(golden):
    k = golden["kats"]
    recs, outs = [], []
    for v in k["aead"]:
        recs.append((bytes.fromhex(v["key"]), bytes.fromhex(v["iv"]), v["seq"], bytes.fromhex(v["aad"]),
                     bytes.fromhex(v["pt"])))
        outs.append(bytes.fromhex(v["out"]))
    return recs, outs


@pytest.mark.parametrize("lanes", LANES)
def test_gcm_basic_and_capacity_kats(engine, golden, lanes):
    """t/fusion.c gcm_basic (:235-274) and gcm_capacity (:276-287)"""
    recs, outs = kat_records(golden)
    hb = HostBatch(engine, recs)
    assert hb.seal(lanes) == outs
    res, pts = hb.open(outs, lanes)
    assert res == [len(r[4]) for r in recs] and pts == [r[4] for r in recs]
    hb.close()


@pytest.mark.parametrize("lanes", LANES)
def test_gcm_test_vectors(engine, golden, lanes):
    """t/fusion.c gcm_test_vectors (:289-343): key 0, iv 0, all-zero AAD/payload, 19 (aadlen, ptlen)"""
    tv = golden["kats"]["gcm_test_vectors"]
    recs = [(bytes(16), bytes(12), 0, bytes(v["aadlen"]), bytes(v["ptlen"])) for v in tv]
    hb = HostBatch(engine, recs)
    outs = hb.seal(lanes)
    for v, o in zip(tv, outs):
        assert o[v["ptlen"]:].hex() == v["tag"], v
    res, pts = hb.open(outs, lanes)
    assert res == [v["ptlen"] for v in tv]
    assert all(p == bytes(len(p)) for p in pts)
    hb.close()


def test_is_supported_on_mi355x(engine):
    """ptls_hip_is_supported (ptls_fusion_is_supported_by_cpu's counterpart) reports the gfx950 device"""
    assert ptls_hip.is_supported()


def test_lowlevel_context_fusion_tests(engine, oracle, golden):
    """ptls_hip_aesgcm_* as t/fusion.c drives ptls_fusion_aesgcm_*: gcm_basic (:235-251), gcm_capacity
    (:276-287, capacity 2 then a larger record) and gcm_test_vectors (:289-343, without and with the supp
    block from ptls_hip_aes128ctr); counter block 0 there is the all-zero nonce here"""
    k = golden["kats"]
    zero_nonce = bytes(12)
    b1 = k["aead"][0]
    ctx = ptls_hip.AesGcm(bytes(16), 5 + 16)
    exp = bytes.fromhex(b1["out"])
    assert ctx.encrypt(bytes(16), zero_nonce, b"hello") == exp
    assert ctx.decrypt(exp[:16], zero_nonce, b"hello", exp[16:]) == (True, bytes(16))
    ctx.close()
    cap = k["aead"][2]
    ctx = ptls_hip.AesGcm(bytes(16), 2)
    exp = bytes.fromhex(cap["out"])
    assert ctx.encrypt(b"X", zero_nonce, b"a") == exp
    assert ctx.decrypt(exp[:1], zero_nonce, b"a", exp[1:]) == (True, b"X")
    big = bytes(range(256)) * 20  # past the initial capacity: staging grows
    assert ctx.encrypt(big, zero_nonce, b"a") == oracle.seal(bytes(16), zero_nonce, 0, b"a", big)
    ctx.set_capacity(1 << 16)
    assert ctx.encrypt(b"X", zero_nonce, b"a") == exp
    ctx.close()
    from oracle_lib import Ref
    tv = k["gcm_test_vectors"]
    ctx = ptls_hip.AesGcm(bytes(16), 2048)
    for v in tv:
        out = ctx.encrypt(bytes(v["ptlen"]), zero_nonce, bytes(v["aadlen"]))
        assert out[v["ptlen"]:].hex() == v["tag"], v
        ok, pt = ctx.decrypt(out[:v["ptlen"]], zero_nonce, bytes(v["aadlen"]), out[v["ptlen"]:])
        assert ok and pt == bytes(v["ptlen"])
    if Ref.available:
        import plugin_driver
        drv = plugin_driver.PluginDriver()
        cctx = drv.cipher_new(128, bytes([1] * 16))
        for v in tv:
            out, supp = ctx.encrypt(bytes(v["ptlen"]), zero_nonce, bytes(v["aadlen"]), cctx, 2)
            assert out[v["ptlen"]:].hex() == v["tag"] and supp.hex() == v["supp"], v
        drv.cipher_free(cctx)
    ctx.close()


def test_lowlevel_context_random_and_tamper(engine, oracle):
    """ptls_hip_aesgcm_* against the oracle on random keys/nonces/lengths, the nonce changing per call;
    a bad detached tag returns 0 with the plaintext still written (lib/fusion.c:660-..., decrypt-then-verify)"""
    rng = np.random.default_rng(1234)
    for key_len in (16, 32):
        key = rng.integers(0, 256, key_len, dtype=np.uint8).tobytes()
        ctx = ptls_hip.AesGcm(key, 1500)
        for _ in range(12):
            nonce = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
            aad = rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes()
            text = rng.integers(0, 256, int(rng.integers(0, 5000)), dtype=np.uint8).tobytes()
            out = ctx.encrypt(text, nonce, aad)
            assert out == oracle.seal(key, nonce, 0, aad, text)
            assert ctx.decrypt(out[:len(text)], nonce, aad, out[len(text):]) == (True, text)
            bad = bytearray(out[len(text):])
            bad[5] ^= 0x80
            ok, pt = ctx.decrypt(out[:len(text)], nonce, aad, bytes(bad))
            assert not ok and pt == text
        ctx.close()


def test_key_slot_out_of_range_is_rejected(engine):
    """a record naming a key slot outside the keyset fails with EINVAL before anything is launched
    (device-resident batch and host pipeline), instead of reading past the keyset on the device"""
    recs, it, ot, _ = ptls_hip.layout_records(np.array([100, 200]), np.array([5, 5]), np.array([0, 1]), np.array([0, 1]))
    ks = ptls_hip.KeySet(engine, 16, 1)
    ks.set(0, bytes(16), bytes(12))
    b = ptls_hip.Batch(engine, recs)
    d_in = torch.zeros(it + 64, dtype=torch.uint8, device="cuda")
    d_out = torch.zeros(ot + 64, dtype=torch.uint8, device="cuda")
    with pytest.raises(ptls_hip.HipError, match="key slot 1"):
        b.seal(ks, d_in, d_in, d_out)
    pipe = ptls_hip.Pipeline(engine, 64 << 10)
    h_in = torch.zeros(it + 64, dtype=torch.uint8).pin_memory()
    h_out = torch.zeros(ot + 64, dtype=torch.uint8).pin_memory()
    with pytest.raises(ptls_hip.HipError, match="key slot 1"):
        pipe.seal(ks, recs, h_in, h_in, h_out)
    ks2 = ptls_hip.KeySet(engine, 16, 2)
    ks2.set(0, bytes(32), bytes(24))
    b.seal(ks2, d_in, d_in, d_out)  # in range: runs
    torch.cuda.synchronize()
    for o in (pipe, b, ks, ks2):
        o.close()


def test_tamper_returns_size_max_and_writes_plaintext(engine, golden):
    """aead_do_decrypt returns SIZE_MAX on a bad tag (lib/fusion.c:1162-1164) but the plaintext has
    already been written (decrypt-then-verify, :822-840); t/picotls.c test_ciphersuite flips a bit."""
    recs, outs = kat_records(golden)
    hb = HostBatch(engine, recs)
    bad = []
    for o in outs:
        b = bytearray(o)
        b[len(b) // 2] ^= 0x01
        bad.append(bytes(b))
    res, pts = hb.open(bad)
    assert res == [UINT64_MAX] * len(recs)
    # every byte except the flipped one decrypts correctly (CTR), as fusion would leave it
    for (key, iv, seq, aad, pt), p, o in zip(recs, pts, outs):
        flip = len(o) // 2
        exp = bytearray(pt)
        if flip < len(pt):
            exp[flip] ^= 0x01
        assert p == bytes(exp)
    hb.close()


def test_iv96_xor_iv(engine, golden):
    """t/fusion.c gcm_iv96 (:345-379) through the keyset's xor_iv (ptls_aead_xor_iv semantics)"""
    k = golden["kats"]
    v = k["gcm_iv96"]
    basic2 = k["aead"][1]
    key, iv = bytes.fromhex(v["key"]), bytes.fromhex(v["iv"])
    pt, aad = bytes.fromhex(basic2["pt"]), bytes.fromhex(basic2["aad"])
    hb = HostBatch(engine, [(key, iv, 0, aad, pt)])
    hb.keyset.xor_iv(0, bytes.fromhex(v["xor"]))
    assert hb.keyset.get_iv(0) == bytes.fromhex(basic2["iv"])
    out = hb.seal()
    assert out[0].hex() == basic2["out"]
    hb.keyset.xor_iv(0, bytes.fromhex(v["xor"]))
    hb.keyset.xor_iv(0, bytes.fromhex(v["bad_xor"]))
    res, _ = hb.open(out)
    assert res == [UINT64_MAX]
    hb.keyset.xor_iv(0, bytes.fromhex(v["bad_xor"]))
    hb.keyset.xor_iv(0, bytes.fromhex(v["xor"]))
    res, pts = hb.open(out)
    assert res == [len(pt)] and pts == [pt]
    hb.close()


@pytest.mark.parametrize("key_len", [16, 32])
@pytest.mark.parametrize("lanes", (0,) + LANES)
def test_length_sweep(engine, oracle, golden, key_len, lanes):
    """L in {0..97, 1328..1339, 1350, 4095..4097, 16383, 16384} x AAD {0,5,13,20,32};
    each record its own key slot, all in ONE launch; compared with lib/fusion.c output digests."""
    vecs = [v for v in golden["sweep"]["vectors"] if v["key_len"] == key_len]
    recs = [sweep_inputs(oracle, v["idx"], key_len, v["L"], v["A"]) for v in vecs]
    hb = HostBatch(engine, recs)
    outs = hb.seal(lanes)
    bad = [v["idx"] for v, o in zip(vecs, outs) if hashlib.sha256(o).hexdigest() != v["sha256"]]
    assert not bad, f"{len(bad)} mismatching vectors, first idx {bad[:8]}"
    res, pts = hb.open(outs, lanes)
    assert res == [v["L"] for v in vecs]
    assert pts == [r[4] for r in recs]
    hb.close()


@pytest.mark.parametrize("name", list(CONFIGS))
def test_baseline_config_samples(engine, oracle, golden, name):
    """first/last 64 records (+ shard seams) of every BASELINE config"""
    cfg = golden["configs"]["configs"][name]
    recs = [config_record(oracle, CONFIGS[name], r["i"]) for r in cfg["records"]]
    recs_sorted = sorted(range(len(recs)), key=lambda j: recs[j][0])  # group same-key records
    hb = HostBatch(engine, [recs[j] for j in recs_sorted])
    outs = hb.seal()
    for j, o in zip(recs_sorted, outs):
        assert hashlib.sha256(o).hexdigest() == cfg["records"][j]["sha256"], (name, cfg["records"][j]["i"])
    hb.close()


@pytest.mark.parametrize("align", [1, 4])
def test_unaligned_layout(engine, oracle, align):
    """records packed at 1- and 4-byte granularity take the byte-granular path; must stay exact"""
    rng = np.random.default_rng(7)
    recs = []
    for i in range(300):
        L = int(rng.integers(0, 1500))
        A = int(rng.integers(0, 40))
        key, iv = oracle.gen_key(i % 3, 16)
        recs.append((key, iv, i, oracle.stream(1000 + i, A), oracle.stream(5000 + i, L)))
    recs.sort(key=lambda r: r[0])
    hb = HostBatch(engine, recs, align=align)
    outs = hb.seal()
    for r, o in zip(recs, outs):
        assert o == oracle.seal(*r)
    res, pts = hb.open(outs)
    assert res == [len(r[4]) for r in recs] and pts == [r[4] for r in recs]
    hb.close()


@pytest.mark.parametrize("wg", [512, 768])
@pytest.mark.parametrize("lanes", [2, 4, 8, 16, 32, 64])
def test_key_runs_mixed_lengths(engine, oracle, wg, lanes):
    """BASELINE configs[3] shape in miniature: AES-256, several keys with runs of 150-400 records of
    random 0..6000-byte lengths (the planner reorders each key chunk by length), every workgroup size"""
    rng = np.random.default_rng(wg * 10 + lanes)
    recs = []
    for k in range(5):
        key, iv = oracle.gen_key(k, 32)
        for i in range(int(rng.integers(150, 400))):
            L = int(rng.integers(0, 6000))
            recs.append((key, iv, 1000 * k + i, tls_aad(L), oracle.stream(77 * k + i, L)))
    hb = HostBatch(engine, recs)
    outs = hb.seal(lanes, wg=wg)
    bad = [j for j, (r, o) in enumerate(zip(recs, outs)) if o != oracle.seal(*r)]
    assert not bad, f"{len(bad)} mismatches, first {bad[:8]}"
    res, pts = hb.open(outs, lanes, wg=wg)
    assert res == [len(r[4]) for r in recs] and pts == [r[4] for r in recs]
    hb.close()


def test_in_place_seal(engine, oracle):
    """output == input is allowed (fusion, SURVEY.md §7 hard parts)"""
    recs = []
    for i in range(64):
        key, iv = oracle.gen_key(0, 32)
        recs.append((key, iv, i, tls_aad(100 + 37 * i), oracle.gen_record(i, 100 + 37 * i)))
    hb = HostBatch(engine, recs)
    outs = hb.seal(in_place=True)
    for r, o in zip(recs, outs):
        assert o == oracle.seal(*r)
    hb.close()


def test_differential_random(engine, oracle):
    """t/fusion.c test_generated (:384-465) in batch form: random keys/ivs/seq/aad/text < 256 B,
    both key sizes, 10 000 records each as in the reference, compared with the CPU oracle; then opened back."""
    rng = np.random.default_rng(12345)
    for key_len in (16, 32):
        recs = []
        for i in range(10000):
            key = rng.integers(0, 256, key_len, dtype=np.uint8).tobytes()
            iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
            seq = int(rng.integers(0, 2 ** 63))
            aad = rng.integers(0, 256, int(rng.integers(0, 256)), dtype=np.uint8).tobytes()
            pt = rng.integers(0, 256, int(rng.integers(0, 256)), dtype=np.uint8).tobytes()
            recs.append((key, iv, seq, aad, pt))
        hb = HostBatch(engine, recs)
        outs = hb.seal()
        for r, o in zip(recs, outs):
            assert o == oracle.seal(*r)
        res, pts = hb.open(outs)
        assert res == [len(r[4]) for r in recs] and pts == [r[4] for r in recs]
        hb.close()


@pytest.mark.parametrize("lanes", [0, 2, 16, 32, 64])
@pytest.mark.parametrize("key_len", [16, 32])
def test_large_records_counter_past_16_bits(engine, oracle, key_len, lanes):
    """records past 2^16 blocks (1 MiB): the counter-mode shortcut holds only while the 32-bit block
    counter stays below 2^16, so the full-block stretch stops at block 65533 and the rest of the record
    takes the full-AES path (inc32 stays exact: fusion's 64-bit lane increment equals it for any record
    under 64 GiB, lib/fusion.c:406-418).  Lengths straddle the boundary; seal == oracle, open round trips."""
    rng = np.random.default_rng(key_len + lanes)
    lens = [65533 * 16 - 3, 65534 * 16, 65535 * 16 + 7, (1 << 21) + 3]
    recs = []
    for i, L in enumerate(lens):
        key, iv = oracle.gen_key(50 + i, key_len)
        recs.append((key, iv, 1000 + i, rng.integers(0, 256, 13, dtype=np.uint8).tobytes(),
                     rng.integers(0, 256, L, dtype=np.uint8).tobytes()))
    hb = HostBatch(engine, recs)
    outs = hb.seal(lanes)
    for r, o in zip(recs, outs):
        assert o == oracle.seal(*r), len(r[4])
    res, pts = hb.open(outs, lanes)
    assert res == lens and pts == [r[4] for r in recs]
    hb.close()


def test_full_size_roundtrip_16k(engine, oracle):
    """64K x 16 KiB (1 GiB) synthetic records filled on the GPU: seal -> open must return every
    record with its length and the original bytes (size-independent property), and sampled records
    must equal the oracle's seal of the generator's bytes."""
    n, L = 1 << 16, 16384
    key, iv = oracle.gen_key(0, 16)
    recs, in_total, out_total, _ = ptls_hip.layout_records([L] * n, [5] * n, [0] * n, np.arange(n))
    aad = np.tile(np.frombuffer(tls_aad(L), np.uint8), (n, 1))
    aad = np.concatenate([aad, np.zeros((n, 11), np.uint8)], axis=1).reshape(-1)  # 16-B aligned AAD slots
    recs["aad_off"] = np.arange(n, dtype=np.uint64) * 16
    ks = ptls_hip.KeySet(engine, 16, 1)
    ks.set(0, key, iv)
    b = ptls_hip.Batch(engine, recs)
    d_in = torch.empty(in_total, dtype=torch.uint8, device="cuda")
    d_aad = torch.from_numpy(aad).cuda()
    d_ct = torch.empty(out_total, dtype=torch.uint8, device="cuda")
    d_pt = torch.empty(in_total, dtype=torch.uint8, device="cuda")
    d_res = torch.zeros(n, dtype=torch.int64, device="cuda")
    b.fill(d_in, 0x70746C7300000001)
    b.seal(ks, d_in, d_aad, d_ct)
    # open reads ct||tag at in_off = out_off of the seal
    recs_o = recs.copy()
    recs_o["in_off"] = recs["out_off"]
    recs_o["out_off"] = recs["in_off"]
    bo = ptls_hip.Batch(engine, recs_o)
    bo.open(ks, d_ct, d_aad, d_pt, d_res)
    torch.cuda.synchronize()
    assert bool((d_res == L).all())
    assert torch.equal(d_pt, d_in)
    ct = d_ct.cpu().numpy()
    for i in (0, 1, 777, n // 2, n - 1):
        pt = oracle.gen_record(i, L)
        assert d_in[recs["in_off"][i]: recs["in_off"][i] + L].cpu().numpy().tobytes() == pt
        exp = oracle.seal(key, iv, i, tls_aad(L), pt)
        assert ct[recs["out_off"][i]: recs["out_off"][i] + L + 16].tobytes() == exp
    for o in (b, bo, ks):
        o.close()


def test_non_temporal_objects_through_reference_picotls(engine, oracle):
    """ptls_hip_non_temporal_aes{128,256}gcm through the reference's ptls_aead_new_direct: per-direction
    vtables as non_temporal_setup (lib/fusion.c:2109-2142) sets them, do_encrypt_v (what ptls_send uses)
    and do_decrypt equal to lib/fusion.c's bytes"""
    from oracle_lib import Ref
    if not Ref.available:
        pytest.skip("oracle/_ref not built")
    import plugin_driver
    drv = plugin_driver.PluginDriver()
    ref = Ref()
    rng = np.random.default_rng(4242)
    for bits in (128, 256):
        key = rng.integers(0, 256, bits // 8, dtype=np.uint8).tobytes()
        iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        enc = drv.new(bits, key, iv, is_enc=1, non_temporal=True)
        dec = drv.new(bits, key, iv, is_enc=0, non_temporal=True)
        ve, vd = plugin_driver.AeadContext.from_address(enc), plugin_driver.AeadContext.from_address(dec)
        assert ve.do_encrypt and ve.do_encrypt_v and not ve.do_decrypt
        assert vd.do_decrypt and not vd.do_encrypt and not vd.do_encrypt_v
        assert not (ve.do_encrypt_init or ve.do_encrypt_update or ve.do_encrypt_final)
        for L in (0, 1, 16, 100, 1350, 16384):
            seq = int(rng.integers(0, 2 ** 40))
            aad = rng.integers(0, 256, 5, dtype=np.uint8).tobytes()
            text = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
            expect = ref.seal(key, iv, seq, aad, text)
            cut = [0, L // 3, L]
            assert drv.encrypt_v(enc, [text[cut[i]:cut[i + 1]] for i in range(2)], seq, aad) == expect
            assert drv.encrypt(enc, text, seq, aad) == expect
            assert drv.decrypt(dec, expect, seq, aad) == text
        drv.free(enc)
        drv.free(dec)


def test_plugin_through_reference_picotls(engine, oracle, golden):
    """Drop-in: the reference's own ptls_aead_new_direct / ptls_aead_xor_iv (oracle/_ref, i.e.
    lib/picotls.c) instantiate ptls_hip_aes128gcm / aes256gcm and drive them through the vtable,
    as picotls applications do; outputs compared with lib/fusion.c in the same process."""
    from oracle_lib import Ref
    if not Ref.available:
        pytest.skip("oracle/_ref not built")
    import plugin_driver
    drv = plugin_driver.PluginDriver()
    k = golden["kats"]
    basic2 = k["aead"][1]
    key, iv = bytes.fromhex(basic2["key"]), bytes.fromhex(basic2["iv"])
    pt, aad = bytes.fromhex(basic2["pt"]), bytes.fromhex(basic2["aad"])
    ctx = drv.new(128, key, iv)
    assert drv.encrypt(ctx, pt, 0, aad).hex() == basic2["out"]
    assert drv.decrypt(ctx, bytes.fromhex(basic2["out"]), 0, aad) == pt
    bad = bytearray.fromhex(basic2["out"])
    bad[3] ^= 1
    assert drv.decrypt(ctx, bytes(bad), 0, aad) is None
    assert drv.decrypt(ctx, b"short", 0, aad) is None  # inlen < 16 -> SIZE_MAX
    drv.free(ctx)
    # gcm_iv96 through the reference's ptls_aead_xor_iv
    v = k["gcm_iv96"]
    ctx = drv.new(128, key, bytes.fromhex(v["iv"]))
    drv.xor_iv(ctx, bytes.fromhex(v["xor"]))
    assert drv.encrypt(ctx, pt, 0, aad).hex() == basic2["out"]
    drv.free(ctx)
    # encrypt_v with three iovecs (what ptls_send uses, lib/picotls.c:705-715)
    ctx = drv.new(256, bytes(range(32)), bytes(12))
    out_v = drv.encrypt_v(ctx, [pt[:10], pt[10:50], pt[50:]], 7, aad)
    assert out_v == oracle.seal(bytes(range(32)), bytes(12), 7, aad, pt)
    drv.free(ctx)
    # test_generated-style differential vs lib/fusion.c, both directions
    ref = Ref()
    rng = np.random.default_rng(99)
    for bits in (128, 256):
        for i in range(40):
            key = rng.integers(0, 256, bits // 8, dtype=np.uint8).tobytes()
            iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
            seq = int(rng.integers(0, 2 ** 62))
            aad = rng.integers(0, 256, int(rng.integers(0, 64)), dtype=np.uint8).tobytes()
            text = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
            ctx = drv.new(bits, key, iv)
            sealed = drv.encrypt(ctx, text, seq, aad)
            assert sealed == ref.seal(key, iv, seq, aad, text)
            assert ref.open(key, iv, seq, aad, sealed) == (len(text), text)
            assert drv.decrypt(ctx, ref.seal(key, iv, seq + 1, aad, text), seq + 1, aad) == text
            drv.free(ctx)


def _supp_array(rows):
    arr = np.zeros(len(rows), dtype=ptls_hip.SUPP_DTYPE)
    for i, (sample_off, mask_off, hp_key, flags) in enumerate(rows):
        arr[i] = (sample_off, mask_off, hp_key, flags)
    return torch.from_numpy(arr.view(np.uint8)).cuda()


@pytest.mark.parametrize("keys", ["3", "per_packet"])
@pytest.mark.parametrize("path", ["device", "copy", "mapped"])
@pytest.mark.parametrize("key_len", [16, 32])
def test_seal_batch_quic_header_protection(engine, oracle, key_len, path, keys):
    """QUIC header protection fused into the seal launch (fusion's supp,
    lib/fusion.c:424-428, :636-650).  Packets of 20-1500 B with 16-40 B headers as AAD, 3 AEAD keys,
    2 header-protection keys, samples anywhere in ciphertext || tag (incl. covering the tag), some
    records without HP, some naming an hp key slot outside the keyset (skipped, mask untouched).
    Ciphertext == oracle, mask == AES-ECB(hp key, sample of the output).  keys="per_packet": every packet
    has its own AEAD key (one record per key run), which the planner sends to the sparse-key kernel."""
    rng = np.random.default_rng(key_len)
    hp_keys = [rng.integers(0, 256, key_len, dtype=np.uint8).tobytes() for _ in range(2)]
    recs = []
    for i in range(600):
        L = int(rng.integers(20, 1500))
        key, iv = oracle.gen_key(i * 3 // 600 if keys == "3" else 1000 + i, key_len)
        recs.append((key, iv, 10_000 + i, oracle.stream(900 + i, int(rng.integers(16, 41))), oracle.stream(3000 + i, L)))
    hb = HostBatch(engine, recs)
    assert (hb.batch.lanes == 64) == (keys == "per_packet")
    hp = ptls_hip.KeySet(engine, key_len, 2)
    hp.set(0, b"".join(hp_keys), None)
    rows, expect = [], []
    for j, (r, rec) in enumerate(zip(recs, hb.recs)):
        L = len(r[4])
        off = int(rng.integers(0, L + 1)) if j % 5 else L  # j % 5 == 0: sample == the tag
        enabled = j % 7 != 3
        hp_key = 7 if j % 11 == 5 else j % 2  # 7: outside the 2-slot keyset -> skipped on the device
        rows.append((int(rec["out_off"]) + off, 16 * j, hp_key, ptls_hip.SUPP_ENABLE if enabled else 0))
        expect.append((off, j % 2, enabled and hp_key < 2))
    h_in = hb._input([r[4] for r in recs])
    h_aad = np.concatenate([hb.aad, np.zeros(16, np.uint8)])
    if path == "device":
        d_supp = _supp_array(rows)
        d_in = torch.from_numpy(h_in).cuda()
        d_aad = torch.from_numpy(h_aad).cuda()
        d_out = torch.zeros(hb.out_total + 32, dtype=torch.uint8, device="cuda")
        d_mask = torch.zeros(16 * len(recs), dtype=torch.uint8, device="cuda")
        hb.batch.seal_supp(hb.keyset, hp, d_supp, d_in, d_aad, d_out, d_mask)
        torch.cuda.synchronize()
        out, mask = d_out.cpu().numpy(), d_mask.cpu().numpy()
    else:  # host-resident: pinned buffers, host supp descriptors, 64 KiB slices
        supp = np.zeros(len(rows), dtype=ptls_hip.SUPP_DTYPE)
        for i, row in enumerate(rows):
            supp[i] = row
        p_out = torch.zeros(hb.out_total + 32, dtype=torch.uint8).pin_memory()
        p_mask = torch.zeros(16 * len(recs), dtype=torch.uint8).pin_memory()
        pipe = ptls_hip.Pipeline(engine, 64 << 10, transport=TRANSPORTS.get(path))
        pipe.seal_supp(hb.keyset, hp, hb.recs, supp, torch.from_numpy(h_in).pin_memory(), torch.from_numpy(h_aad).pin_memory(),
                       p_out, p_mask)
        assert pipe.last_transport == TRANSPORTS[path]
        pipe.close()
        out, mask = p_out.numpy(), p_mask.numpy()
    for j, (r, rec, (off, k, enabled)) in enumerate(zip(recs, hb.recs, expect)):
        sealed = out[rec["out_off"]: rec["out_off"] + rec["len"] + 16].tobytes()
        assert sealed == oracle.seal(*r), j
        m = mask[16 * j: 16 * j + 16].tobytes()
        assert m == (oracle.aes_ecb(hp_keys[k], sealed[off: off + 16]) if enabled else bytes(16)), j
    hp.close()
    hb.close()


def test_supp_kats_gcm_test_vectors(engine, golden):
    """t/fusion.c gcm_test_vectors (:289-343): supp = AES-ECB(01 x 16, output[2:18]) in the same launch"""
    tv = golden["kats"]["gcm_test_vectors"]
    recs = [(bytes(16), bytes(12), 0, bytes(v["aadlen"]), bytes(v["ptlen"])) for v in tv]
    hb = HostBatch(engine, recs)
    hp = ptls_hip.KeySet(engine, 16, 1)
    hp.set(0, b"\x01" * 16, None)
    d_supp = _supp_array([(int(rec["out_off"]) + 2, 16 * j, 0, ptls_hip.SUPP_ENABLE) for j, rec in enumerate(hb.recs)])
    d_in = torch.from_numpy(hb._input([r[4] for r in recs])).cuda()
    d_aad = torch.from_numpy(np.concatenate([hb.aad, np.zeros(16, np.uint8)])).cuda()
    d_out = torch.zeros(hb.out_total + 32, dtype=torch.uint8, device="cuda")
    d_mask = torch.zeros(16 * len(recs), dtype=torch.uint8, device="cuda")
    hb.batch.seal_supp(hb.keyset, hp, d_supp, d_in, d_aad, d_out, d_mask)
    torch.cuda.synchronize()
    out, mask = d_out.cpu().numpy(), d_mask.cpu().numpy()
    for j, (v, rec) in enumerate(zip(tv, hb.recs)):
        assert out[rec["out_off"] + v["ptlen"]: rec["out_off"] + v["ptlen"] + 16].tobytes().hex() == v["tag"]
        assert mask[16 * j: 16 * j + 16].tobytes().hex() == v["supp"], v
    hp.close()
    hb.close()


@pytest.mark.parametrize("key_len", [16, 32])
def test_aesecb_batch_receive_side(engine, oracle, key_len):
    """receive side of header protection: masks from samples of received ciphertext, many hp keys"""
    rng = np.random.default_rng(100 + key_len)
    nkeys, n = 37, 5000
    keys = rng.integers(0, 256, (nkeys, key_len), dtype=np.uint8)
    hp = ptls_hip.KeySet(engine, key_len, nkeys)
    hp.set(0, keys.tobytes(), None)
    src = rng.integers(0, 256, 70_000, dtype=np.uint8)
    rows = [(int(rng.integers(0, len(src) - 16)), 16 * j, int(rng.integers(0, nkeys)), ptls_hip.SUPP_ENABLE)
            for j in range(n)]
    d_mask = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
    engine.aesecb(hp, _supp_array(rows), torch.from_numpy(src).cuda(), d_mask)
    torch.cuda.synchronize()
    mask = d_mask.cpu().numpy()
    for j, (so, mo, k, _) in enumerate(rows):
        assert mask[mo: mo + 16].tobytes() == oracle.aes_ecb(keys[k].tobytes(), src[so: so + 16].tobytes()), j
    hp.close()


def test_plugin_ctr_cipher_and_fused_supp(engine, oracle):
    """ptls_hip_aes{128,256}ctr through the reference's ptls_cipher_new (lib/picotls.c), and
    ptls_aead_encrypt_s with it as supp: output and supp block equal lib/fusion.c's (ref_seal_supp uses
    ptls_fusion_aes*ctr the same way, t/fusion.c:321-331)"""
    from oracle_lib import Ref
    if not Ref.available:
        pytest.skip("oracle/_ref not built")
    import plugin_driver
    drv = plugin_driver.PluginDriver()
    ref = Ref()
    rng = np.random.default_rng(8)
    for bits in (128, 256):
        hp_key = rng.integers(0, 256, bits // 8, dtype=np.uint8).tobytes()
        cctx = drv.cipher_new(bits, hp_key)
        for _ in range(5):
            iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
            ks = oracle.aes_ecb(hp_key, iv)
            assert drv.cipher_encrypt(cctx, iv, bytes(16)) == ks
            data = rng.integers(0, 256, 5, dtype=np.uint8).tobytes()  # a QUIC header mask use: 5 bytes
            assert drv.cipher_encrypt(cctx, iv, data) == bytes(a ^ b for a, b in zip(data, ks))
        key = rng.integers(0, 256, bits // 8, dtype=np.uint8).tobytes()
        iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        actx = drv.new(bits, key, iv)
        for L in (20, 100, 1200):
            text = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
            aad = rng.integers(0, 256, 20, dtype=np.uint8).tobytes()
            for off in (0, 3, L):  # L: the sample is the tag
                out, supp = drv.encrypt_s(actx, text, 77, aad, cctx, off)
                ref_out, ref_supp = ref.seal_supp(key, iv, 77, aad, text, hp_key, off)
                assert out == ref_out and supp == ref_supp, (bits, L, off)
        drv.free(actx)
        drv.cipher_free(cctx)


@pytest.mark.parametrize("transport", ["copy", "mapped"])
@pytest.mark.parametrize("slice_kib", [64, 1024])
def test_host_pipeline_seal_open(engine, oracle, slice_kib, transport):
    """host-resident path: records in pinned host memory, sliced; transport copy = H2D -> kernel -> D2H over 3
    streams, mapped = the kernels on the host buffers directly; mixed lengths, two keys, TLS and QUIC-sized
    records; bit-exact vs the oracle, then opened back"""
    rng = np.random.default_rng(3)
    recs_in = []
    for i in range(700):
        L = int(rng.choice([0, 1, 15, 16, 100, 1350, 4096, 16384, int(rng.integers(0, 20000))]))
        key, iv = oracle.gen_key(i // 350, 16)
        recs_in.append((key, iv, i, tls_aad(L), oracle.gen_record(i, L)))
    lens = [len(r[4]) for r in recs_in]
    recs, in_total, out_total, aad_total = ptls_hip.layout_records(lens, [5] * len(lens), [i // 350 for i in range(700)],
                                                                   np.arange(700), align=16, tag_in_input=True)
    ks = ptls_hip.KeySet(engine, 16, 2)
    k0, iv0 = oracle.gen_key(0, 16)
    k1, iv1 = oracle.gen_key(1, 16)
    ks.set(0, k0 + k1, iv0 + iv1)
    h_in = torch.zeros(in_total + 16, dtype=torch.uint8).pin_memory()
    h_aad = torch.zeros(aad_total + 16, dtype=torch.uint8).pin_memory()
    h_out = torch.zeros(out_total + 16, dtype=torch.uint8).pin_memory()
    hin, haad = h_in.numpy(), h_aad.numpy()
    for r, rec in zip(recs_in, recs):
        hin[rec["in_off"]: rec["in_off"] + len(r[4])] = np.frombuffer(r[4], np.uint8)
        haad[rec["aad_off"]: rec["aad_off"] + 5] = np.frombuffer(r[3], np.uint8)
    pipe = ptls_hip.Pipeline(engine, slice_kib << 10, transport=TRANSPORTS[transport])
    pipe.seal(ks, recs, h_in, h_aad, h_out)
    assert pipe.last_transport == TRANSPORTS[transport]
    hout = h_out.numpy()
    sealed = []
    for r, rec in zip(recs_in, recs):
        got = hout[rec["out_off"]: rec["out_off"] + len(r[4]) + 16].tobytes()
        assert got == oracle.seal(*r)
        sealed.append(got)
    # open: ct||tag as input (in layout has room for the tag), plaintext out
    hin[:] = 0
    for s_, rec in zip(sealed, recs):
        hin[rec["in_off"]: rec["in_off"] + len(s_)] = np.frombuffer(s_, np.uint8)
    hin[recs["in_off"][5] + 3] ^= 1 if recs["len"][5] > 3 else 0  # tamper record 5 (if it has payload)
    h_res = torch.zeros(700, dtype=torch.int64).pin_memory()
    h_out.zero_()
    pipe.open(ks, recs, h_in, h_aad, h_out, h_res)
    res = [int(x) & ((1 << 64) - 1) for x in h_res.numpy()]
    for i, (r, rec) in enumerate(zip(recs_in, recs)):
        if i == 5 and recs["len"][5] > 3:
            assert res[i] == UINT64_MAX
            continue
        assert res[i] == len(r[4]), i
        assert hout[rec["out_off"]: rec["out_off"] + len(r[4])].tobytes() == r[4]
    pipe.close()
    ks.close()


def test_iv_only_resetup_of_a_keyed_context(engine, oracle):
    """setup_crypto(ctx, is_enc, NULL, iv2) on a keyed context only replaces the static IV (lib/fusion.c:1188-1191):
    the next seal equals lib/fusion.c's after the same IV-only re-setup, and a keyed seal under iv2"""
    from oracle_lib import Ref
    if not Ref.available:
        pytest.skip("oracle/_ref not built")
    import plugin_driver
    drv = plugin_driver.PluginDriver()
    ref = Ref()
    rng = np.random.default_rng(77)
    for bits in (128, 256):
        key = rng.integers(0, 256, bits // 8, dtype=np.uint8).tobytes()
        iv, iv2 = (rng.integers(0, 256, 12, dtype=np.uint8).tobytes() for _ in range(2))
        text = rng.integers(0, 256, 1000, dtype=np.uint8).tobytes()
        aad = b"hdr"
        for non_temporal in (False, True):
            ctx = drv.new(bits, key, iv, is_enc=1, non_temporal=non_temporal)
            assert drv.encrypt(ctx, text, 5, aad) == ref.seal(key, iv, 5, aad, text)
            assert ref.lib.ref_aead_setup_iv_only(ctx, 1, iv2) == 0
            assert drv.encrypt(ctx, text, 5, aad) == ref.seal_reiv(key, iv, iv2, 5, aad, text) == ref.seal(key, iv2, 5, aad, text)
            drv.free(ctx)


def test_aesecb_api_fusion_kats(engine, oracle, golden):
    """ptls_hip_aesecb_init / _encrypt / _dispose replay t/fusion.c test_ecb (:71-85: all-zero AES-128 and AES-256
    keys on "hello world!!!!!"), then random keys and blocks against the oracle"""
    for v in golden["kats"]["ecb"]:
        ecb = ptls_hip.AesEcb(bytes.fromhex(v["key"]))
        assert ecb.rounds == (10 if len(v["key"]) == 32 else 14)
        assert ecb.encrypt(bytes.fromhex(v["pt"])).hex() == v["ct"]
        ecb.close()
    rng = np.random.default_rng(5)
    for key_len in (16, 32):
        key = rng.integers(0, 256, key_len, dtype=np.uint8).tobytes()
        ecb = ptls_hip.AesEcb(key)
        for _ in range(8):
            blk = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
            assert ecb.encrypt(blk) == oracle.aes_ecb(key, blk)
        ecb.close()
    with pytest.raises(ptls_hip.HipError):
        ptls_hip.AesEcb(bytes(16), is_enc=0)  # fusion: assert(is_enc) (lib/fusion.c:859)


@pytest.mark.parametrize("bits", [128, 256])
def test_tls12_record_layer_over_non_temporal_objects(engine, bits):
    """The tls12 = {4, 8} fields ptls_hip_non_temporal_aes*gcm advertise, exercised by the reference's TLS 1.2
    record layer: two post-handshake TLS 1.2 connections made by ptls_build_tls12_export_params + ptls_import
    from one master secret, one on lib/fusion.c's ptls_non_temporal_aes*gcm and one on ours.  ptls_send
    (8-byte explicit record IV from the counter, 13-byte AAD of build_tls12_aad, lib/picotls.c:730-794) emits
    the same wire bytes; each side's ptls_receive (handle_input_tls12, :5927-5990) decrypts the other's; a
    flipped byte is rejected the same way by both."""
    from oracle_lib import Ref, RefTLS12
    if not Ref.available:
        pytest.skip("oracle/_ref not built")
    import plugin_driver
    drv = plugin_driver.PluginDriver()
    rng = np.random.default_rng(bits)
    master = rng.integers(0, 256, 48, dtype=np.uint8).tobytes()
    randoms = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    rec_iv = int(rng.integers(0, 2 ** 62))
    ours = drv.nt_algos[bits]
    f_srv = RefTLS12(bits, master, randoms, rec_iv, None, is_server=1)
    h_srv = RefTLS12(bits, master, randoms, rec_iv, ours, is_server=1)
    f_cli = RefTLS12(bits, master, randoms, 0, None, is_server=0)
    h_cli = RefTLS12(bits, master, randoms, 0, ours, is_server=0)

    def receive_all(conn, wire):
        got, pos = b"", 0
        while pos < len(wire):
            ret, used, pt = conn.receive(wire[pos:])
            assert ret == 0 and used > 0, (ret, used)
            got += pt
            pos += used
        return got

    for L in (1, 15, 16, 17, 1350, 16384, 16385, 40000):
        payload = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        wire_f, wire_h = f_srv.send(payload), h_srv.send(payload)
        assert wire_h == wire_f, L
        assert receive_all(h_cli, wire_f) == payload
        assert receive_all(f_cli, wire_h) == payload
    # tamper: the same response from both record layers (fusion's NT decrypt vs ours)
    payload = rng.integers(0, 256, 500, dtype=np.uint8).tobytes()
    wire = bytearray(f_srv.send(payload))
    assert bytes(wire) == h_srv.send(payload)
    wire[40] ^= 0x10
    assert h_cli.receive(bytes(wire)) == f_cli.receive(bytes(wire))
    for c in (f_srv, h_srv, f_cli, h_cli):
        c.close()


@pytest.mark.parametrize("lanes", (0, 1, 8, 32, 64))
def test_empty_batches_and_empty_records(engine, oracle, lanes):
    """a batch of no records is a no-op on every path (batch, copy / mapped pipeline); a batch of records with no
    payload (tag = E_K(J0) ^ GHASH of the AAD and length block only) equals the oracle and opens to length 0"""
    empty = np.zeros(0, dtype=ptls_hip.RECORD_DTYPE)
    ks = ptls_hip.KeySet(engine, 16, 1)
    k0, iv0 = oracle.gen_key(0, 16)
    ks.set(0, k0, iv0)
    b = ptls_hip.Batch(engine, empty)
    b.set_lanes(lanes)
    buf = torch.zeros(64, dtype=torch.uint8, device="cuda")
    res = torch.zeros(1, dtype=torch.int64, device="cuda")
    b.seal(ks, buf, buf, buf)
    b.open(ks, buf, buf, buf, res)
    torch.cuda.synchronize()
    b.close()
    h = torch.zeros(64, dtype=torch.uint8).pin_memory()
    h_res = torch.zeros(1, dtype=torch.int64).pin_memory()
    for t in TRANSPORTS.values():
        pipe = ptls_hip.Pipeline(engine, 1 << 20, transport=t)
        pipe.seal(ks, empty, h, h, h)
        pipe.open(ks, empty, h, h, h, h_res)
        pipe.close()
    ks.close()
    recs = []
    for i, A in enumerate([0, 0, 5, 13, 16, 17, 0, 32]):
        key, iv = oracle.gen_key(i % 3, 16)
        recs.append((key, iv, 1000 + i, oracle.gen_record(50 + i, A), b""))
    hb = HostBatch(engine, recs)
    outs = hb.seal(lanes)
    assert outs == [oracle.seal(*r) for r in recs]
    res_, pts = hb.open(outs, lanes)
    assert res_ == [0] * len(recs) and pts == [b""] * len(recs)
    hb.close()


@pytest.mark.parametrize("key_len", [16, 32])
def test_key_setup_for_many_slots(engine, oracle, key_len):
    """key setup runs one wave per slot up to 4096 slots per call (keysetup_wide_kernel, every other test) and one
    thread per slot above (keysetup_kernel): 4100 keys in one call, one record each of 0-4000 B, sealed at every
    lanes-per-record value (each reads its own H-power planes: H .. H^64 and the lane powers), equal the oracle"""
    rng = np.random.default_rng(4100 + key_len)
    recs = []
    for i in range(4100):
        key, iv = oracle.gen_key(20000 + i, key_len)
        L = int(rng.integers(0, 4000))
        recs.append((key, iv, i, tls_aad(L), oracle.stream(30000 + i, L)))
    expect = [oracle.seal(*r) for r in recs]
    hb = HostBatch(engine, recs)
    for lanes in LANES:
        outs = hb.seal(lanes)
        bad = [j for j, (o, e) in enumerate(zip(outs, expect)) if o != e]
        assert not bad, f"lanes {lanes}: {len(bad)} mismatches, first {bad[:8]}"
    hb.close()


@pytest.mark.parametrize("transport", ["copy", "mapped"])
@pytest.mark.parametrize("shape", ["equal", "descending"])
def test_host_pipeline_plan_keeps_caller_order(engine, oracle, transport, shape):
    """records that already come as the planner orders them (equal lengths, or non-increasing within each key run):
    the pipeline reuses the caller-order descriptors as the plan-order ones (no gather, one upload per slice,
    planner.cpp identity_order); several slices, two key runs; bit-exact vs the oracle and opened back"""
    n = 1200
    if shape == "equal":
        lens = [1350] * n
    else:
        lens = sorted((int(x) for x in np.random.default_rng(11).integers(0, 5000, n // 2)), reverse=True) * 2
    recs_in = []
    for i, L in enumerate(lens):
        key, iv = oracle.gen_key(50 + i // (n // 2), 16)
        recs_in.append((key, iv, i, tls_aad(L), oracle.gen_record(9000 + i, L)))
    recs, in_total, out_total, aad_total = ptls_hip.layout_records(lens, [5] * n, [i // (n // 2) for i in range(n)],
                                                                   np.arange(n), align=16, tag_in_input=True)
    ks = ptls_hip.KeySet(engine, 16, 2)
    k0, iv0 = oracle.gen_key(50, 16)
    k1, iv1 = oracle.gen_key(51, 16)
    ks.set(0, k0 + k1, iv0 + iv1)
    h_in = torch.zeros(in_total + 16, dtype=torch.uint8).pin_memory()
    h_aad = torch.zeros(aad_total + 16, dtype=torch.uint8).pin_memory()
    h_out = torch.zeros(out_total + 16, dtype=torch.uint8).pin_memory()
    hin, haad = h_in.numpy(), h_aad.numpy()
    for r, rec in zip(recs_in, recs):
        hin[rec["in_off"]: rec["in_off"] + len(r[4])] = np.frombuffer(r[4], np.uint8)
        haad[rec["aad_off"]: rec["aad_off"] + 5] = np.frombuffer(r[3], np.uint8)
    pipe = ptls_hip.Pipeline(engine, 256 << 10, transport=TRANSPORTS[transport])
    pipe.seal(ks, recs, h_in, h_aad, h_out)
    hout = h_out.numpy()
    sealed = [hout[rec["out_off"]: rec["out_off"] + len(r[4]) + 16].tobytes() for r, rec in zip(recs_in, recs)]
    bad = [i for i, (r, s_) in enumerate(zip(recs_in, sealed)) if s_ != oracle.seal(*r)]
    assert not bad, f"{len(bad)} mismatches, first {bad[:8]}"
    for s_, rec in zip(sealed, recs):
        hin[rec["in_off"]: rec["in_off"] + len(s_)] = np.frombuffer(s_, np.uint8)
    h_res = torch.zeros(n, dtype=torch.int64).pin_memory()
    h_out.zero_()
    pipe.open(ks, recs, h_in, h_aad, h_out, h_res)
    assert [int(x) for x in h_res.numpy()] == lens
    assert all(hout[rec["out_off"]: rec["out_off"] + len(r[4])].tobytes() == r[4] for r, rec in zip(recs_in, recs))
    pipe.close()
    ks.close()
