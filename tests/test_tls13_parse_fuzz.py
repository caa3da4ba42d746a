"""ptls_hip_tls13_parse against the reference's own receive path on malformed streams.

The engine's receive side parses untrusted wire bytes on the host (ptls_hip_tls13_parse), then opens the records on the
device and strips the inner padding (tls13_open_batch / pipeline_tls13_open).  The reference does all of that in
ptls_receive (lib/picotls.c:6061-6100: handle_input :5840-5925, parse_record :5033-5095, parse_record_header
:5020-5031, aead_decrypt :717-726).  Here 12 000 streams are built from valid ptls_send output of the reference
(oracle/_ref, random payloads over 1-4 sends) and then damaged: truncated, a length field replaced (small / random /
oversized / zero / shorter than a tag), a type byte replaced (another record type or no record type at all), garbage
appended, or several of these at once.  Each stream goes

* through the reference: a fresh receiving ptls_t (ptls_import from the sender's traffic secret, at the sender's
  sequence number) and ptls_receive called until it fails, stops producing data or has taken every byte;
* through the engine's parse, then each produced record opened by the CPU oracle (lib/fusion.c restated, pinned by
  tests/golden: test infrastructure standing in for the device open, which tests/test_gpu_tls13.py covers) and its
  padding stripped as tls13_inner_kernel does;

and both must agree on the records accepted, the wire bytes they span and the first error (the alert code and where it
happened).  Where the engine stops at a record it leaves to the caller's picotls record layer by contract (another record
type, or legacy_record_version bytes other than 03 03, which picotls ignores), the caller runs ptls_receive on the rest:
the engine's records followed by that must give exactly what ptls_receive gives on the whole stream.
"""
import numpy as np
import pytest

import ptls_hip
from oracle_lib import Ref, RefTLS, ref_traffic_keys

needs_ref = pytest.mark.skipif(not Ref.available, reason="oracle/_ref (reference build) not present")
STREAMS = 12000
DECODE_ERROR, BAD_RECORD_MAC, UNEXPECTED_MESSAGE = 50, 20, 10  # PTLS_ALERT_* (include/picotls.h)


def _damage(rng, wire, bounds):
    """one to three random damages of a valid record stream; bounds = start offsets of its records"""
    w = bytearray(wire)
    for _ in range(int(rng.integers(1, 4))):
        kind = int(rng.integers(0, 7))
        rec = bounds[int(rng.integers(0, len(bounds)))] if bounds else 0
        if kind == 0 and len(w):  # truncate anywhere
            del w[int(rng.integers(0, len(w) + 1)):]
        elif kind == 1 and rec + 5 <= len(w):  # a nearby length
            L = int.from_bytes(w[rec + 3: rec + 5], "big") + int(rng.integers(-20, 21))
            w[rec + 3: rec + 5] = (L & 0xFFFF).to_bytes(2, "big")
        elif kind == 2 and rec + 5 <= len(w):  # any length, or one of the edges
            L = int(rng.choice([int(rng.integers(0, 65536)), 0, 15, 16, 17, 16384 + 256, 16384 + 257, 65535]))
            w[rec + 3: rec + 5] = L.to_bytes(2, "big")
        elif kind == 3 and rec < len(w):  # another record type, or a byte that is none
            w[rec] = int(rng.choice([20, 21, 22, 24, 0, 0x80, int(rng.integers(0, 256))]))
        elif kind == 4:  # garbage after the records
            w += rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8).tobytes()
        elif kind == 5 and rec + 5 <= len(w):  # a tag-less record
            w[rec + 3: rec + 5] = int(rng.integers(0, 16)).to_bytes(2, "big")
        elif kind == 6 and rec + 5 <= len(w):  # the version bytes (not checked by parse_record_header)
            w[rec + 1: rec + 3] = rng.integers(0, 256, 2, dtype=np.uint8).tobytes()
    return bytes(w)


def _aead(bits):
    """lib/fusion.c's ptls_non_temporal_aes{128,256}gcm (AES-NI; the same bytes as the fusion AEAD, and it implements the
    do_encrypt_v ptls_send needs, lib/fusion.c:2154-2179) instead of RefTLS's default minicrypto, ~100x slower"""
    return Ref().algo(f"ptls_non_temporal_aes{bits}gcm")


def _reference(bits, secret, seq, stream):
    """(records accepted, bytes they span, first error) of ptls_receive called until it fails or stops"""
    rx = RefTLS(bits, bytes(len(secret)), secret, dec_seq=seq, is_server=0, aead=_aead(bits))
    pos, accepted, err = 0, 0, 0
    try:
        while pos < len(stream):
            ret, used, pt = rx.receive(stream[pos:])
            if ret != 0:
                err = ret
                break
            if not pt:  # an incomplete record buffered (it took the rest), or nothing decodable: stop
                if pos + used >= len(stream) or used == 0:
                    break
            else:
                accepted += 1
            pos += used
    finally:
        rx.close()
    return accepted, pos, err


def _engine(oracle, key, iv, seq, stream):
    """(records accepted, bytes they span, first error, how it ended) from ptls_hip_tls13_parse + the open and padding
    strip of the records it produced; "deferred" = it stopped at a complete record it leaves to picotls"""
    rc, recs, consumed = ptls_hip.tls13_parse(stream, seq=seq, with_rc=True)
    pos = 0
    for i, r in enumerate(recs):
        a, b = int(r["in_off"]), int(r["in_off"]) + int(r["len"]) + 16
        n, pt = oracle.open(key, iv, seq + i, stream[int(r["aad_off"]): a], stream[a:b])
        if n is None:
            return i, pos, BAD_RECORD_MAC, "mac"
        body = pt.rstrip(b"\x00")
        if not body:
            return i, pos, UNEXPECTED_MESSAGE, "type"
        assert body[-1] == 23, "ptls_send output carries application data only"
        pos = b
    assert pos == consumed
    if rc == ptls_hip.TLS13_DECODE_ERROR:
        return len(recs), pos, DECODE_ERROR, "parse"
    if rc == ptls_hip.TLS13_SHORT_RECORD:
        return len(recs), pos, BAD_RECORD_MAC, "parse"
    assert rc == 0, rc
    if pos < len(stream) and (stream[pos] in (20, 21, 22) or (len(stream) - pos >= 5 and stream[pos + 1: pos + 3] != b"\x03\x03")):
        return len(recs), pos, None, "deferred"  # another record type or version bytes: picotls's record layer decides
    return len(recs), pos, 0, "stop"


@needs_ref
@pytest.mark.parametrize("bits", [128, 256])
def test_parse_agrees_with_ptls_receive_on_damaged_streams(oracle, bits):
    rng = np.random.default_rng(0x7a5e + bits)
    n = 48 if bits == 256 else 32
    s_tx, s_rx = rng.integers(0, 256, n, dtype=np.uint8).tobytes(), rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    tx = RefTLS(bits, s_tx, s_rx, aead=_aead(bits))
    key, iv = ref_traffic_keys(bits, s_tx)
    seq = 0
    kinds = {}
    for s in range(STREAMS // 2):
        wire, bounds = b"", []
        seq0 = seq
        for _ in range(int(rng.integers(1, 5))):
            L = int(rng.choice([int(rng.integers(1, 300)), int(rng.integers(300, 3000)), 16384, int(rng.integers(16385, 40000))],
                               p=[0.6, 0.3, 0.05, 0.05]))
            w = tx.send(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
            p = 0
            while p < len(w):
                bounds.append(len(wire) + p)
                p += 5 + int.from_bytes(w[p + 3: p + 5], "big")
                seq += 1
            wire += w
        stream = _damage(rng, wire, bounds)
        ref = _reference(bits, s_tx, seq0, stream)
        eng = _engine(oracle, key, iv, seq0, stream)
        kinds[eng[3]] = kinds.get(eng[3], 0) + 1
        if eng[3] == "deferred":  # the caller hands the rest to its picotls: together they must give ptls_receive's result
            rest = _reference(bits, s_tx, seq0 + eng[0], stream[eng[1]:])
            assert ref == (eng[0] + rest[0], eng[1] + rest[1], rest[2]), (s, ref, eng, rest)
        else:
            assert ref == eng[:3], (s, ref, eng, stream[:64].hex())
        # the undamaged stream as well: every record accepted, no error
        if s % 50 == 0:
            assert _reference(bits, s_tx, seq0, wire) == (len(bounds), len(wire), 0)
            assert _engine(oracle, key, iv, seq0, wire)[:3] == (len(bounds), len(wire), 0)
    tx.close()
    # every outcome was exercised
    assert all(kinds.get(k, 0) >= 50 for k in ("mac", "parse", "deferred", "stop")), kinds
