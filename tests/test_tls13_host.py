"""CPU tests of the TLS 1.3 record layer pieces that run on the host:
the oracle's restatement of picotls's send path pinned against the reference's own ptls_send, and the
engine's framing planner / record parser (ptls_hip_tls13_frame / _parse, plain C, no GPU needed)
checked against the wire bytes the reference produces."""
import os

import numpy as np
import pytest

import ptls_hip
from oracle_lib import Ref, RefTLS, ref_traffic_keys, tls13_wire

needs_ref = pytest.mark.skipif(not Ref.available, reason="oracle/_ref (reference build) not present")

SIZES = [0, 1, 15, 16, 17, 1000, 16383, 16384, 16385, 32768, 40000]


def secrets(bits, seed):
    rng = np.random.default_rng(seed)
    n = 48 if bits == 256 else 32
    return rng.integers(0, 256, n, dtype=np.uint8).tobytes(), rng.integers(0, 256, n, dtype=np.uint8).tobytes()


@needs_ref
@pytest.mark.parametrize("bits", [128, 256])
def test_reference_send_receive_and_restatement(oracle, bits):
    """ptls_send / ptls_receive of the reference round-trip, and tests/oracle_lib.tls13_wire (the restatement
    the GPU tests compare with) reproduces ptls_send byte for byte, including 16384-byte chunking and
    the sequence numbers across calls"""
    s_enc, s_dec = secrets(bits, bits)
    server = RefTLS(bits, s_enc, s_dec, enc_seq=5)
    client = RefTLS(bits, s_dec, s_enc, dec_seq=5, is_server=0)
    key, iv = ref_traffic_keys(bits, s_enc)
    seq = 5
    for L in SIZES:
        payload = os.urandom(L)
        wire = server.send(payload)
        assert wire == tls13_wire(oracle, key, iv, seq, 23, payload), L
        assert len(wire) == ptls_hip.lib().ptls_hip_tls13_wire_size(L)
        seq += (L + 16383) // 16384
        got, pos = b"", 0
        while pos < len(wire):
            ret, used, pt = client.receive(wire[pos:])
            assert ret == 0
            pos += used
            got += pt
        assert got == payload
    server.close()
    client.close()


@needs_ref
def test_frame_planner_matches_reference_layout(oracle):
    """ptls_hip_tls13_frame: the record descriptors of several messages place every header / ciphertext /
    tag exactly where ptls_send puts them, with one sequence number per record"""
    msgs = np.zeros(len(SIZES), dtype=ptls_hip.TLS13_MESSAGE_DTYPE)
    in_off = out_off = 0
    for i, L in enumerate(SIZES):
        msgs[i] = (in_off, out_off, 1000 * i, L, i % 3, 23 if i % 2 else 22, 0)
        in_off += L + 7
        out_off += ptls_hip.lib().ptls_hip_tls13_wire_size(L) + 3
    recs = ptls_hip.tls13_frame(msgs)
    assert len(recs) == sum((L + 16383) // 16384 for L in SIZES)
    k = 0
    for i, L in enumerate(SIZES):
        wire = msgs[i]["out_off"]
        for j, pos in enumerate(range(0, L, 16384)):
            chunk = min(16384, L - pos)
            r = recs[k]
            assert (r["in_off"], r["aad_off"], r["out_off"]) == (msgs[i]["in_off"] + pos, wire, wire + 5)
            assert (r["seq"], r["len"], r["aad_len"], r["key"]) == (1000 * i + j, chunk + 1, 5, i % 3)
            assert r["flags"] == ptls_hip.record_tls13_type(int(msgs[i]["type"]))
            wire += 5 + chunk + 17
            k += 1


@needs_ref
def test_parse_reference_wire():
    """ptls_hip_tls13_parse on ptls_send output: one descriptor per record (AAD = header, ciphertext after
    it, plaintext packed at out_base), stops at an incomplete record and at a non-application-data record,
    rejects oversized / tag-less records like parse_record_header (lib/picotls.c:5020-5031)"""
    s_enc, s_dec = secrets(128, 1)
    server = RefTLS(128, s_enc, s_dec)
    wire = b"".join(server.send(os.urandom(L)) for L in (100, 40000, 1))
    server.close()
    recs, consumed = ptls_hip.tls13_parse(wire, wire_off=64, key=7, seq=3, out_base=4096)
    assert consumed == len(wire) and len(recs) == 1 + 3 + 1
    pos, out = 0, 4096
    for i, r in enumerate(recs):
        length = int.from_bytes(wire[pos + 3:pos + 5], "big")
        assert (r["aad_off"], r["in_off"], r["len"], r["seq"], r["key"], r["out_off"]) == \
            (64 + pos, 64 + pos + 5, length - 16, 3 + i, 7, out)
        out += length - 16
        pos += 5 + length
    # incomplete tail
    recs2, consumed2 = ptls_hip.tls13_parse(wire[:-1])
    assert len(recs2) == 4 and consumed2 == len(wire) - (5 + 1 + 17)
    # a handshake / alert record stops the parse (picotls's record layer handles those)
    recs3, consumed3 = ptls_hip.tls13_parse(wire[:122] + b"\x15\x03\x03\x00\x02\x02\x28")
    assert len(recs3) == 1 and consumed3 == 122
    with pytest.raises(ptls_hip.HipError):
        ptls_hip.tls13_parse(b"\x17\x03\x03" + (16384 + 257).to_bytes(2, "big") + bytes(16384 + 257))
    with pytest.raises(ptls_hip.HipError):
        ptls_hip.tls13_parse(b"\x17\x03\x03\x00\x0f" + bytes(15))


@needs_ref
@pytest.mark.parametrize("bits", [128, 256])
def test_traffic_key_derivation_vectors(oracle, bits):
    """HKDF-Expand-Label key / iv of the reference, used by the GPU tests to key the batch engine the way
    ptls_aead_new keys a connection: sealing with them reproduces ptls_send"""
    s_enc, s_dec = secrets(bits, 77)
    key, iv = ref_traffic_keys(bits, s_enc)
    assert len(key) == bits // 8 and len(iv) == 12
    server = RefTLS(bits, s_enc, s_dec)
    payload = b"hello"
    assert server.send(payload) == tls13_wire(oracle, key, iv, 0, 23, payload)
    server.close()
