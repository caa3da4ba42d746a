"""GPU parity of the TLS 1.3 record layer over the batch engine and of the
plugin inside the reference's own record layer.

Oracle: the reference itself -- ptls_send / ptls_receive of lib/picotls.c on a ptls_t made by
ptls_import from traffic secrets (oracle/_ref, tests/oracle_lib.RefTLS), whose AEAD keys come from
its HKDF-Expand-Label.  Bar: bit-exact wire bytes, identical plaintexts, picotls's error semantics.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import ptls_hip  # noqa: E402

from oracle_lib import Ref, RefTLS, ref_traffic_keys, tls13_wire  # noqa: E402

TRANSPORTS = {"copy": ptls_hip.TRANSPORT_COPY, "mapped": ptls_hip.TRANSPORT_MAPPED}  # host pipeline transports
needs_ref = pytest.mark.skipif(not Ref.available, reason="oracle/_ref (reference build) not present")


def conn_secrets(bits, n, seed):
    rng = np.random.default_rng(seed)
    ds = 48 if bits == 256 else 32
    return [(rng.integers(0, 256, ds, dtype=np.uint8).tobytes(), rng.integers(0, 256, ds, dtype=np.uint8).tobytes())
            for _ in range(n)]


@needs_ref
@pytest.mark.parametrize("path", ["device", "copy", "mapped"])
@pytest.mark.parametrize("bits", [128, 256])
def test_tls13_seal_batch_equals_ptls_send(engine, oracle, bits, path):
    """many connections x messages of 0..40000 bytes and three content types, framed + sealed in one
    batch; every connection's wire bytes == the reference's ptls_send (appdata) or its restatement
    (other content types, same code path with `type`, lib/picotls.c:747-794)"""
    rng = np.random.default_rng(bits)
    nconn = 6
    secs = conn_secrets(bits, nconn, bits + 1)
    keys = [ref_traffic_keys(bits, s[0]) for s in secs]
    ks = ptls_hip.KeySet(engine, bits // 8, nconn)
    ks.set(0, b"".join(k for k, _ in keys), b"".join(iv for _, iv in keys))
    refs = [RefTLS(bits, s[0], s[1], enc_seq=100 * c) for c, s in enumerate(secs)]
    msgs, payloads, expect = [], [], []
    in_off = out_off = 0
    seqs = [100 * c for c in range(nconn)]
    for i in range(40):
        c = i % nconn
        L = int(rng.choice([0, 1, 15, 16, 17, 1350, 16383, 16384, 16385, int(rng.integers(0, 40000))]))
        ctype = 23 if i % 4 else int(rng.choice([21, 22]))
        payload = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        if ctype == 23:
            wire = refs[c].send(payload)
        else:
            wire = tls13_wire(oracle, keys[c][0], keys[c][1], seqs[c], ctype, payload)
            refs[c].close()  # keep the reference connection's seq in step: re-import after the other-type records
            refs[c] = RefTLS(bits, secs[c][0], secs[c][1], enc_seq=seqs[c] + (L + 16383) // 16384)
        msgs.append((in_off, out_off + 3 * i, seqs[c], L, c, ctype, 0))  # ragged gaps between messages
        seqs[c] += (L + 16383) // 16384
        payloads.append(payload)
        expect.append(wire)
        in_off += L + (i % 5)
        out_off += len(wire)
    marr = np.array(msgs, dtype=ptls_hip.TLS13_MESSAGE_DTYPE)
    recs = ptls_hip.tls13_frame(marr)
    h_in = np.zeros(in_off + 16, np.uint8)
    for m, p in zip(marr, payloads):
        h_in[m["in_off"]: m["in_off"] + len(p)] = np.frombuffer(p, np.uint8)
    b = None
    if path == "device":
        d_in = torch.from_numpy(h_in).cuda()
        d_out = torch.zeros(out_off + 3 * len(msgs) + 16, dtype=torch.uint8, device="cuda")
        b = ptls_hip.Batch(engine, recs)
        b.tls13_seal(ks, d_in, d_out)
        torch.cuda.synchronize()
        out = d_out.cpu().numpy()
    else:  # host-resident: pinned message buffer -> pinned wire buffer, 64 KiB slices (many slices, 3 streams)
        p_in = torch.from_numpy(h_in).pin_memory()
        p_out = torch.zeros(out_off + 3 * len(msgs) + 16, dtype=torch.uint8).pin_memory()
        pipe = ptls_hip.Pipeline(engine, 64 << 10, transport=TRANSPORTS.get(path))
        pipe.tls13_seal(ks, recs, p_in, p_out)
        assert pipe.last_transport == TRANSPORTS[path]
        pipe.close()
        out = p_out.numpy()
    for i, (m, wire) in enumerate(zip(marr, expect)):
        got = out[m["out_off"]: m["out_off"] + len(wire)].tobytes()
        assert got == wire, (i, int(m["len"]), int(m["type"]))
    for r in refs:
        r.close()
    if b is not None:
        b.close()
    ks.close()


@needs_ref
@pytest.mark.parametrize("path", ["device", "copy", "mapped"])
@pytest.mark.parametrize("bits", [128, 256])
def test_tls13_open_batch_equals_ptls_receive(engine, oracle, bits, path):
    """a received byte stream (ptls_send output, plus records with TLSInnerPlaintext padding, an all-zero
    record and a tampered one) is parsed on the host and opened in one batch: content, content type and
    picotls's errors (BAD_RECORD_MAC, UNEXPECTED_MESSAGE) as handle_input decides them (lib/picotls.c:5866-5883)"""
    s_enc, s_dec = conn_secrets(bits, 1, 9 + bits)[0]
    key, iv = ref_traffic_keys(bits, s_enc)
    sender = RefTLS(bits, s_enc, s_dec)
    receiver = RefTLS(bits, s_dec, s_enc, is_server=0)
    rng = np.random.default_rng(3)
    pieces, expect = [], []
    seq = 0
    for L in (1, 100, 16384, 40000, 0, 5):
        payload = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        wire = sender.send(payload)
        pieces.append(wire)
        for pos in range(0, L, 16384):
            expect.append(("ok", 23, payload[pos:pos + 16384]))
        seq += (L + 16383) // 16384
    # records built by the restatement: padding after the content type, alert-type content, all-zero, tampered
    def rec(inner, s):
        hdr = bytes([0x17, 3, 3]) + (len(inner) + 16).to_bytes(2, "big")
        return hdr + oracle.seal(key, iv, s, hdr, inner)
    pieces.append(rec(b"padded" + bytes([23]) + bytes(40), seq)); expect.append(("ok", 23, b"padded")); seq += 1
    pieces.append(rec(bytes([2, 40]) + bytes([21]), seq)); expect.append(("ok", 21, bytes([2, 40]))); seq += 1
    pieces.append(rec(bytes(33), seq)); expect.append(("nocontent", None, None)); seq += 1
    bad = bytearray(rec(b"tampered" + bytes([23]), seq)); bad[9] ^= 4
    pieces.append(bytes(bad)); expect.append(("badmac", None, None)); seq += 1
    stream = b"".join(pieces)
    recs, consumed = ptls_hip.tls13_parse(stream, wire_off=0, key=0, seq=0, out_base=0)
    assert consumed == len(stream) and len(recs) == len(expect)
    ks = ptls_hip.KeySet(engine, bits // 8, 1)
    ks.set(0, key, iv)
    out_size = int(recs["out_off"][-1] + recs["len"][-1]) + 32
    b = None
    if path == "device":
        b = ptls_hip.Batch(engine, recs)
        d_in = torch.from_numpy(np.frombuffer(stream + bytes(16), np.uint8).copy()).cuda()
        d_out = torch.zeros(out_size, dtype=torch.uint8, device="cuda")
        d_res = torch.zeros(len(recs), dtype=torch.int64, device="cuda")
        b.tls13_open(ks, d_in, d_out, d_res)
        torch.cuda.synchronize()
        out = d_out.cpu().numpy()
        res = [int(x) & ((1 << 64) - 1) for x in d_res.cpu().numpy()]
    else:  # host-resident: the received stream in pinned memory, 64 KiB slices
        p_in = torch.from_numpy(np.frombuffer(stream + bytes(16), np.uint8).copy()).pin_memory()
        p_out = torch.zeros(out_size, dtype=torch.uint8).pin_memory()
        p_res = torch.zeros(len(recs), dtype=torch.int64).pin_memory()
        pipe = ptls_hip.Pipeline(engine, 64 << 10, transport=TRANSPORTS.get(path))
        pipe.tls13_open(ks, recs, p_in, p_out, p_res)
        assert pipe.last_transport == TRANSPORTS[path]
        pipe.close()
        out = p_out.numpy()
        res = [int(x) & ((1 << 64) - 1) for x in p_res.numpy()]
    for r, v, (kind, ctype, content) in zip(recs, res, expect):
        if kind == "badmac":
            assert v == ptls_hip.TLS13_BAD_RECORD_MAC
        elif kind == "nocontent":
            assert v == ptls_hip.TLS13_NO_CONTENT_TYPE
        else:
            n, t = v & ((1 << 56) - 1), v >> 56
            assert (t, out[r["out_off"]: r["out_off"] + n].tobytes()) == (ctype, content)
    # the reference's own receive path agrees on the application data of the ptls_send part
    got, pos = b"", 0
    sent = b"".join(pieces[:6])
    while pos < len(sent):
        ret, used, pt = receiver.receive(sent[pos:])
        assert ret == 0
        pos += used
        got += pt
    assert got == b"".join(c for k, t, c in expect if k == "ok" and t == 23)[: len(got)]
    for o in (b, ks, sender, receiver):
        if o is not None:
            o.close()


@needs_ref
@pytest.mark.parametrize("bits", [128, 256])
def test_reference_record_layer_on_hip_aead(engine, bits):
    """drop-in for ptls_send / ptls_receive: the reference's TLS 1.3 record layer (ptls_import, aead_encrypt ->
    ptls_aead_encrypt_v, aead_decrypt, lib/picotls.c:705-726) running on ptls_hip_aes{128,256}gcm produces and
    accepts exactly the bytes it does on minicrypto's AES-GCM"""
    hip = ptls_hip.lib()
    import ctypes
    algo = ctypes.addressof(ctypes.c_char.in_dll(hip, f"ptls_hip_aes{bits}gcm"))
    s_enc, s_dec = conn_secrets(bits, 1, 40 + bits)[0]
    on_hip = RefTLS(bits, s_enc, s_dec, enc_seq=7, aead=algo)
    on_ref = RefTLS(bits, s_enc, s_dec, enc_seq=7)
    peer_hip = RefTLS(bits, s_dec, s_enc, dec_seq=7, aead=algo, is_server=0)
    rng = np.random.default_rng(bits)
    for L in (0, 1, 17, 1350, 16384, 20000):
        payload = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        wire = on_hip.send(payload)
        assert wire == on_ref.send(payload), L
        got, pos = b"", 0
        while pos < len(wire):
            ret, used, pt = peer_hip.receive(wire[pos:])
            assert ret == 0
            pos += used
            got += pt
        assert got == payload
    # a flipped bit is PTLS_ALERT_BAD_RECORD_MAC (20) through the HIP AEAD as well
    bad = bytearray(on_ref.send(b"x" * 50))
    bad[20] ^= 1
    ret, _, _ = peer_hip.receive(bytes(bad))
    assert ret == 20
    for o in (on_hip, on_ref, peer_hip):
        o.close()


@needs_ref
@pytest.mark.parametrize("bits", [128, 256])
def test_keyset_from_traffic_secrets(engine, oracle, bits):
    """§8(f) rank 4: 3000 connections keyed on the GPU from TLS 1.3 traffic secrets (SHA-256 / SHA-384
    HKDF-Expand-Label "key" / "iv"), then one record each sealed in a batch: == oracle seal with the keys
    the reference's ptls_hkdf_expand_label derives; the static IVs read back equal the reference's"""
    from oracle_lib import ref_traffic_keys
    n, hs = 3000, 48 if bits == 256 else 32
    rng = np.random.default_rng(bits + 5)
    secrets = rng.integers(0, 256, n * hs, dtype=np.uint8).tobytes()
    ks = ptls_hip.KeySet(engine, bits // 8, n)
    ks.set_secrets(0, secrets, hs)
    lens = [int(rng.integers(0, 300)) for _ in range(n)]
    recs, in_total, out_total, _ = ptls_hip.layout_records(lens, [0] * n, np.arange(n), np.arange(n) * 3)
    payloads = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in lens]
    h_in = np.zeros(in_total + 16, np.uint8)
    for r, p in zip(recs, payloads):
        h_in[r["in_off"]: r["in_off"] + len(p)] = np.frombuffer(p, np.uint8)
    b = ptls_hip.Batch(engine, recs)
    d_out = torch.zeros(out_total + 16, dtype=torch.uint8, device="cuda")
    b.seal(ks, torch.from_numpy(h_in).cuda(), torch.zeros(16, dtype=torch.uint8, device="cuda"), d_out)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    for i in range(0, n, 7):
        key, iv = ref_traffic_keys(bits, secrets[i * hs:(i + 1) * hs])
        assert ks.get_iv(i) == iv
        r = recs[i]
        assert out[r["out_off"]: r["out_off"] + r["len"] + 16].tobytes() == oracle.seal(key, iv, 3 * i, b"", payloads[i]), i
    b.close()
    ks.close()


@needs_ref
@pytest.mark.parametrize("bits", [128, 256])
def test_key_update_matches_ptls_send(engine, oracle, bits):
    """the TLS 1.3 key update on the GPU (update_traffic_key, lib/picotls.c:4980-4996) for many connections:
    next secrets == the reference's HKDF-Expand-Label(secret, "traffic upd"), and a connection at seq 2^24
    -- where the reference's own ptls_send performs the update (lib/picotls.c:6129-6141) -- sends its next
    application record exactly as the GPU-updated slot seals it"""
    from oracle_lib import ref_hkdf_expand_label
    n, hs = 512, 48 if bits == 256 else 32
    rng = np.random.default_rng(bits + 9)
    secrets = rng.integers(0, 256, n * hs, dtype=np.uint8).tobytes()
    ks = ptls_hip.KeySet(engine, bits // 8, n)
    ks.set_secrets(0, secrets, hs)
    nxt = ks.update_secrets(0, secrets, hs)
    for i in range(0, n, 5):
        assert nxt[i * hs:(i + 1) * hs] == ref_hkdf_expand_label(bits, secrets[i * hs:(i + 1) * hs], b"traffic upd", hs), i
    # connection 0 through the reference's ptls_send at the key-update threshold
    peer_secret = rng.integers(0, 256, hs, dtype=np.uint8).tobytes()
    conn = RefTLS(bits, secrets[:hs], peer_secret, enc_seq=1 << 24)
    payload = rng.integers(0, 256, 700, dtype=np.uint8).tobytes()
    wire = conn.send(payload)
    conn.close()
    first_len = 5 + int.from_bytes(wire[3:5], "big")  # the KeyUpdate handshake record, old key
    app = wire[first_len:]
    recs, in_total, out_total, _ = ptls_hip.layout_records([len(payload) + 1], [5], [0], [0])
    recs["flags"] = ptls_hip.record_tls13_type(23)
    hdr = app[:5]
    d_in = torch.from_numpy(np.frombuffer(payload + bytes(32), np.uint8).copy()).cuda()
    d_aad = torch.from_numpy(np.frombuffer(hdr + bytes(11), np.uint8).copy()).cuda()
    d_out = torch.zeros(out_total + 32, dtype=torch.uint8, device="cuda")
    b = ptls_hip.Batch(engine, recs)
    b.seal(ks, d_in, d_aad, d_out)  # slot 0 now holds the updated key, seq restarts at 0
    torch.cuda.synchronize()
    assert d_out.cpu().numpy()[: len(payload) + 17].tobytes() == app[5:]
    b.close()
    ks.close()
