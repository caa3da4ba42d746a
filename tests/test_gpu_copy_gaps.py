"""The COPY host transport writes exactly the records' bytes into the caller's buffers.

fusion writes a record's output and nothing else (storen128 for the partial block, lib/fusion.c:388-397; the tag store,
:632).  The copy transport stages a slice's records through device buffers; it used to copy the slice's whole output span
back, so every byte lying between two records in the caller's buffer received whatever the staging held, e.g. the
plaintext of an earlier open on the same pipeline.  Here ONE copy-transport pipeline (pageable numpy buffers, as a socket
buffer would be) first opens records so that its staging holds plaintext, then seals, seals with QUIC header protection,
seals TLS 1.3 messages and opens again, every time into output buffers pre-filled with 0xA5 with 1-64-byte gaps between
the records: every record equals the oracle's (lib/fusion.c restated, pinned by tests/golden) and every other byte is
still 0xA5.  Cases: both key sizes; 64 KiB and 1 MiB slices; many records per slice (the gap-filled copies) and five
(one copy per record run); descriptors in output order and shuffled (a slice's gaps then hold other slices' records,
which must not be overwritten).
"""
import numpy as np
import pytest

import ptls_hip

pytestmark = pytest.mark.gpu
FILL, MFILL = 0xA5, 0x5A


def _place(rng, sizes, gap_max):
    """offsets of back-to-back ranges of `sizes` with a 1..gap_max-byte gap before each one, and the buffer size"""
    off, pos = [], 0
    for s in sizes:
        pos += int(rng.integers(1, gap_max + 1))
        off.append(pos)
        pos += int(s)
    return off, pos + int(rng.integers(1, gap_max + 1))


def _touched(size, ranges):
    m = np.zeros(size, bool)
    for lo, n in ranges:
        m[lo: lo + n] = True
    return m


class Case:
    def __init__(self, engine, oracle, bits, n, seed):
        rng = np.random.default_rng(seed)
        self.rng = rng
        kb = bits // 8
        self.keys = [oracle.gen_key(70 + k, kb) for k in range(2)]
        self.ks = ptls_hip.KeySet(engine, kb, 2)
        self.ks.set(0, self.keys[0][0] + self.keys[1][0], self.keys[0][1] + self.keys[1][1])
        choices = [0, 1, 15, 16, 17, 100, 1350, 4095, 16384]
        self.lens = [int(rng.choice(choices)) if i % 3 else int(rng.integers(0, 3000)) for i in range(n)]
        self.key = [i * 2 // n for i in range(n)]  # two key runs
        self.seq = [1000 + i for i in range(n)]
        self.aad = [oracle.stream(500 + i, 13) for i in range(n)]
        self.pt = [oracle.stream(900 + i, L) for i, L in enumerate(self.lens)]
        self.sealed = [oracle.seal(*self.keys[self.key[i]], self.seq[i], self.aad[i], self.pt[i]) for i in range(n)]

    def recs(self, in_off, out_off, aad_off):
        n = len(self.lens)
        r = np.zeros(n, dtype=ptls_hip.RECORD_DTYPE)
        r["in_off"], r["out_off"], r["aad_off"] = in_off, out_off, aad_off
        r["seq"], r["len"], r["aad_len"], r["key"] = self.seq, self.lens, 13, self.key
        return r

    def aad_buffer(self):
        aad_off, size = _place(self.rng, [13] * len(self.lens), 8)
        buf = self.rng.integers(0, 256, size, dtype=np.uint8)
        for o, a in zip(aad_off, self.aad):
            buf[o: o + 13] = np.frombuffer(a, np.uint8)
        return aad_off, buf


def _order(n, shuffled, rng):
    return rng.permutation(n) if shuffled else np.arange(n)


def _seal(case, pipe, gap_max, perm):
    in_off, in_size = _place(case.rng, case.lens, 4)
    h_in = case.rng.integers(0, 256, in_size, dtype=np.uint8)
    for o, p in zip(in_off, case.pt):
        h_in[o: o + len(p)] = np.frombuffer(p, np.uint8)
    aad_off, h_aad = case.aad_buffer()
    out_off, out_size = _place(case.rng, [L + 16 for L in case.lens], gap_max)
    h_out = np.full(out_size, FILL, np.uint8)
    recs = case.recs(in_off, out_off, aad_off)
    pipe.seal(case.ks, recs[perm], h_in, h_aad, h_out)
    assert pipe.last_transport == ptls_hip.TRANSPORT_COPY
    for i, o in enumerate(out_off):
        assert h_out[o: o + case.lens[i] + 16].tobytes() == case.sealed[i], ("seal", i)
    untouched = ~_touched(out_size, [(o, L + 16) for o, L in zip(out_off, case.lens)])
    assert (h_out[untouched] == FILL).all(), ("seal wrote between records", np.flatnonzero(h_out[untouched] != FILL)[:8])
    return out_off, h_out


def _open(case, pipe, gap_max, perm):
    in_off, in_size = _place(case.rng, [L + 16 for L in case.lens], 4)
    h_in = case.rng.integers(0, 256, in_size, dtype=np.uint8)
    for o, s in zip(in_off, case.sealed):
        h_in[o: o + len(s)] = np.frombuffer(s, np.uint8)
    aad_off, h_aad = case.aad_buffer()
    out_off, out_size = _place(case.rng, case.lens, gap_max)
    h_out = np.full(out_size, FILL, np.uint8)
    h_res = np.zeros(len(case.lens), np.uint64)
    recs = case.recs(in_off, out_off, aad_off)
    pipe.open(case.ks, recs[perm], h_in, h_aad, h_out, h_res)
    assert pipe.last_transport == ptls_hip.TRANSPORT_COPY
    assert [int(x) for x in h_res] == [case.lens[i] for i in perm]
    for i, o in enumerate(out_off):
        assert h_out[o: o + case.lens[i]].tobytes() == case.pt[i], ("open", i)
    untouched = ~_touched(out_size, list(zip(out_off, case.lens)))
    assert (h_out[untouched] == FILL).all(), ("open wrote between records", np.flatnonzero(h_out[untouched] != FILL)[:8])


def _seal_supp(case, pipe, oracle, gap_max, perm):
    kb = len(case.keys[0][0])
    hp_key = oracle.stream(77, kb)
    hp = ptls_hip.KeySet(pipe.engine, kb, 1)
    hp.set(0, hp_key, None)
    n = len(case.lens)
    in_off, in_size = _place(case.rng, case.lens, 4)
    h_in = case.rng.integers(0, 256, in_size, dtype=np.uint8)
    for o, p in zip(in_off, case.pt):
        h_in[o: o + len(p)] = np.frombuffer(p, np.uint8)
    aad_off, h_aad = case.aad_buffer()
    out_off, out_size = _place(case.rng, [L + 16 for L in case.lens], gap_max)
    h_out = np.full(out_size, FILL, np.uint8)
    h_mask = np.full(32 * n + 16, MFILL, np.uint8)  # masks at 32 j + 8: 16 bytes between any two stay untouched
    supp = np.zeros(n, dtype=ptls_hip.SUPP_DTYPE)
    samp = []
    for i in range(n):
        off = int(case.rng.integers(0, case.lens[i] + 1))  # the sample may cover the tag
        samp.append(off)
        supp[i] = (out_off[i] + off, 32 * i + 8, 0, ptls_hip.SUPP_ENABLE if i % 5 != 2 else 0)
    recs = case.recs(in_off, out_off, aad_off)
    pipe.seal_supp(case.ks, hp, recs[perm], supp[perm], h_in, h_aad, h_out, h_mask)
    for i, o in enumerate(out_off):
        assert h_out[o: o + case.lens[i] + 16].tobytes() == case.sealed[i], ("seal_supp", i)
        want = oracle.aes_ecb(hp_key, case.sealed[i][samp[i]: samp[i] + 16]) if i % 5 != 2 else bytes([MFILL]) * 16
        assert h_mask[32 * i + 8: 32 * i + 24].tobytes() == want, ("mask", i)
    untouched = ~_touched(out_size, [(o, L + 16) for o, L in zip(out_off, case.lens)])
    assert (h_out[untouched] == FILL).all(), "seal_supp wrote between records"
    mtouched = _touched(len(h_mask), [(32 * i + 8, 16) for i in range(n)])
    assert (h_mask[~mtouched] == MFILL).all(), "seal_supp wrote between masks"
    hp.close()


@pytest.mark.parametrize("order", ["in_order", "shuffled"])
@pytest.mark.parametrize("n", [300, 5])
@pytest.mark.parametrize("slice_kib", [64, 1024])
@pytest.mark.parametrize("bits", [128, 256])
def test_copy_transport_writes_only_record_bytes(engine, oracle, bits, slice_kib, n, order):
    case = Case(engine, oracle, bits, n, seed=bits + slice_kib + n)
    perm = _order(n, order == "shuffled", case.rng)
    pipe = ptls_hip.Pipeline(engine, slice_kib << 10, transport=ptls_hip.TRANSPORT_COPY)
    _open(case, pipe, 64, perm)  # first: the staging now holds plaintext
    _seal(case, pipe, 64, perm)
    _seal_supp(case, pipe, oracle, 64, perm)
    _open(case, pipe, 64, perm)
    _seal(case, pipe, 1, perm)  # 1-byte gaps
    pipe.close()
    case.ks.close()


def test_copy_transport_auto_for_pageable_buffers(engine, oracle):
    """AUTO picks the copy transport for pageable buffers, with the same exact-bytes output"""
    case = Case(engine, oracle, 128, 120, seed=11)
    pipe = ptls_hip.Pipeline(engine, 64 << 10)
    _open(case, pipe, 32, np.arange(120))
    _seal(case, pipe, 32, np.arange(120))
    pipe.close()
    case.ks.close()


@pytest.mark.parametrize("slice_kib", [64, 1024])
def test_copy_transport_tls13_seal_gaps_between_messages(engine, oracle, slice_kib):
    """TLS 1.3 seal through the copy transport: each message's records back to back (header, ciphertext, tag), messages
    1-64 bytes apart in a 0xA5-filled wire buffer; the records equal ptls_send's framing restated (5-byte header as AAD,
    the content type appended, lib/picotls.c:696-715) and the bytes between messages stay 0xA5"""
    rng = np.random.default_rng(slice_kib)
    key, iv = oracle.gen_key(5, 16)
    ks = ptls_hip.KeySet(engine, 16, 1)
    ks.set(0, key, iv)
    lens = [int(rng.integers(1, 40000)) for _ in range(40)]
    pts = [oracle.stream(40 + m, L) for m, L in enumerate(lens)]
    wire_sizes = [ptls_hip.lib().ptls_hip_tls13_wire_size(L) for L in lens]
    wire_off, wire_size = _place(rng, wire_sizes, 64)
    in_off, in_size = _place(rng, lens, 4)
    h_in = np.zeros(in_size, np.uint8)
    for o, p in zip(in_off, pts):
        h_in[o: o + len(p)] = np.frombuffer(p, np.uint8)
    msgs = np.zeros(len(lens), dtype=ptls_hip.TLS13_MESSAGE_DTYPE)
    seq, seqs = 0, []
    for m, L in enumerate(lens):
        msgs[m] = (in_off[m], wire_off[m], seq, L, 0, 23, 0)
        seqs.append(seq)
        seq += (L + 16383) // 16384
    recs = ptls_hip.tls13_frame(msgs)
    h_wire = np.full(wire_size, FILL, np.uint8)
    pipe = ptls_hip.Pipeline(engine, slice_kib << 10, transport=ptls_hip.TRANSPORT_COPY)
    pipe.tls13_seal(ks, recs, h_in, h_wire)
    for m, (L, p) in enumerate(zip(lens, pts)):
        pos, s = wire_off[m], seqs[m]
        for c in range(0, L, 16384):
            chunk = p[c: c + 16384]
            hdr = bytes([0x17, 3, 3]) + (len(chunk) + 17).to_bytes(2, "big")
            want = hdr + oracle.seal(key, iv, s, hdr, chunk + b"\x17")
            assert h_wire[pos: pos + len(want)].tobytes() == want, (m, c)
            pos += len(want)
            s += 1
        assert pos == wire_off[m] + wire_sizes[m]
    untouched = ~_touched(wire_size, list(zip(wire_off, wire_sizes)))
    assert (h_wire[untouched] == FILL).all()
    pipe.close()
    ks.close()
