"""ctypes bindings for the CPU checkers -- TEST INFRASTRUCTURE ONLY.

* ``Oracle``  -> oracle/liboracle.so, the plain-C restatement (oracle/aesgcm_oracle.c).
* ``Ref``     -> oracle/_ref/libptls_fusion_ref.so, the reference's own lib/fusion.c built unmodified
                 by oracle/Makefile (absent on a box that never had /root/reference; tests that need it
                 skip, the committed golden fixtures still pin parity).
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libptls_fusion_ref.so")
SIZE_MAX = (1 << 64) - 1

_c = ctypes
_u8p = _c.c_void_p


def _buf(b):
    return _c.create_string_buffer(bytes(b), max(len(b), 1))


def build_oracle():
    if not os.path.exists(ORACLE_SO):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


class Oracle:
    def __init__(self):
        build_oracle()
        L = self.lib = _c.CDLL(ORACLE_SO)
        L.oracle_aes_expand.restype = _c.c_int
        L.oracle_aes_expand.argtypes = [_u8p, _c.c_size_t, _u8p]
        L.oracle_aes_ecb.argtypes = [_u8p, _c.c_size_t, _u8p, _u8p]
        L.oracle_gf128_mul.argtypes = [_u8p, _u8p, _u8p]
        L.oracle_ghash.argtypes = [_u8p, _u8p, _c.c_size_t, _u8p, _c.c_size_t, _u8p]
        L.oracle_build_iv.argtypes = [_u8p, _c.c_uint64, _u8p]
        for f in (L.oracle_aesgcm_seal, L.oracle_aesgcm_open):
            f.restype = _c.c_size_t
            f.argtypes = [_u8p, _c.c_size_t, _u8p, _c.c_uint64, _u8p, _c.c_size_t, _u8p, _c.c_size_t, _u8p]
        L.oracle_fusion_domain_ghash.argtypes = [_u8p, _u8p, _c.c_size_t, _u8p]
        L.oracle_splitmix64_at.restype = _c.c_uint64
        L.oracle_splitmix64_at.argtypes = [_c.c_uint64, _c.c_uint64]
        L.oracle_stream_bytes.argtypes = [_c.c_uint64, _u8p, _c.c_size_t]
        L.oracle_gen_key.argtypes = [_c.c_uint64, _c.c_size_t, _u8p, _u8p]
        L.oracle_gen_record.argtypes = [_c.c_uint64, _u8p, _c.c_size_t]
        L.oracle_gen_quic_aad.argtypes = [_c.c_uint64, _u8p]
        L.oracle_mixed_len.restype = _c.c_uint32
        L.oracle_mixed_len.argtypes = [_c.c_uint64]
        L.oracle_bench_seal.restype = _c.c_double
        L.oracle_bench_seal.argtypes = [_c.c_size_t, _c.c_size_t, _c.c_size_t, _c.c_int]

    def aes_ecb(self, key, block):
        out = _c.create_string_buffer(16)
        self.lib.oracle_aes_ecb(_buf(key), len(key), _buf(block), out)
        return out.raw

    def gf128_mul(self, x, y):
        out = _c.create_string_buffer(16)
        self.lib.oracle_gf128_mul(_buf(x), _buf(y), out)
        return out.raw

    def ghash(self, H, aad, ct):
        out = _c.create_string_buffer(16)
        self.lib.oracle_ghash(_buf(H), _buf(aad), len(aad), _buf(ct), len(ct), out)
        return out.raw

    def seal(self, key, iv, seq, aad, pt):
        out = _c.create_string_buffer(len(pt) + 16)
        n = self.lib.oracle_aesgcm_seal(_buf(key), len(key), _buf(iv), seq, _buf(aad), len(aad), _buf(pt), len(pt), out)
        assert n == len(pt) + 16
        return out.raw

    def open(self, key, iv, seq, aad, ct):
        out = _c.create_string_buffer(max(len(ct), 16))
        n = self.lib.oracle_aesgcm_open(_buf(key), len(key), _buf(iv), seq, _buf(aad), len(aad), _buf(ct), len(ct), out)
        return (None if n == SIZE_MAX else n), out.raw[: max(len(ct) - 16, 0)]

    def fusion_domain_ghash(self, Hf, blocks):
        out = _c.create_string_buffer(16)
        self.lib.oracle_fusion_domain_ghash(_buf(Hf), _buf(blocks), len(blocks) // 16, out)
        return out.raw

    def stream(self, seed, n):
        out = _c.create_string_buffer(max(n, 1))
        self.lib.oracle_stream_bytes(seed, out, n)
        return out.raw[:n]

    def gen_key(self, j, key_len):
        key = _c.create_string_buffer(32)
        iv = _c.create_string_buffer(12)
        self.lib.oracle_gen_key(j, key_len, key, iv)
        return key.raw[:key_len], iv.raw

    def gen_record(self, i, n):
        out = _c.create_string_buffer(max(n, 1))
        self.lib.oracle_gen_record(i, out, n)
        return out.raw[:n]

    def gen_quic_aad(self, i):
        out = _c.create_string_buffer(13)
        self.lib.oracle_gen_quic_aad(i, out)
        return out.raw

    def mixed_len(self, i):
        return self.lib.oracle_mixed_len(i)


def tls_aad(payload_len):
    reclen = payload_len + 16
    return bytes([0x17, 0x03, 0x03, (reclen >> 8) & 0xFF, reclen & 0xFF])


class Ref:
    """The reference engine (lib/fusion.c) reached through picotls's public AEAD API."""

    available = os.path.exists(REF_SO)

    def __init__(self):
        L = self.lib = _c.CDLL(REF_SO)
        for name in ("ref_seal", "ref_open"):
            f = getattr(L, name)
            f.restype = _c.c_size_t
            f.argtypes = [_c.c_int, _u8p, _u8p, _c.c_uint64, _u8p, _c.c_size_t, _u8p, _c.c_size_t, _u8p]
        L.ref_seal_supp.restype = _c.c_size_t
        L.ref_seal_supp.argtypes = [_c.c_int, _u8p, _u8p, _c.c_uint64, _u8p, _c.c_size_t, _u8p, _c.c_size_t, _u8p,
                                    _u8p, _c.c_size_t, _u8p]
        L.ref_seal_iv96.restype = _c.c_size_t
        L.ref_seal_iv96.argtypes = [_c.c_int, _u8p, _u8p, _u8p, _c.c_size_t, _c.c_uint64, _u8p, _c.c_size_t, _u8p,
                                    _c.c_size_t, _u8p]
        L.ref_bench.restype = _c.c_double
        L.ref_bench.argtypes = [_c.c_int, _c.c_int, _u8p, _u8p, _u8p, _u8p, _c.c_size_t, _c.c_size_t, _c.c_size_t,
                                _u8p, _c.c_size_t, _c.c_int, _c.c_void_p, _c.c_int]
        L.ref_seal_reiv.restype = _c.c_size_t
        L.ref_seal_reiv.argtypes = [_c.c_int, _u8p, _u8p, _u8p, _c.c_uint64, _u8p, _c.c_size_t, _u8p, _c.c_size_t, _u8p]
        L.ref_aead_new_iv_only.restype = _c.c_void_p
        L.ref_aead_new_iv_only.argtypes = [_c.c_void_p, _c.c_int, _u8p]
        L.ref_aead_setup_iv_only.restype = _c.c_int
        L.ref_aead_setup_iv_only.argtypes = [_c.c_void_p, _c.c_int, _u8p]
        L.ref_ctx_free_raw.argtypes = [_c.c_void_p]
        L.ref_fusion_supported.restype = _c.c_int
        L.ref_fusion_can_aesni256.restype = _c.c_int
        self.supported = bool(L.ref_fusion_supported())

    def seal(self, key, iv, seq, aad, pt):
        out = _c.create_string_buffer(len(pt) + 16)
        n = self.lib.ref_seal(len(key) * 8, _buf(key), _buf(iv), seq, _buf(aad), len(aad), _buf(pt), len(pt), out)
        assert n == len(pt) + 16
        return out.raw

    def seal_supp(self, key, iv, seq, aad, pt, hp_key, supp_off):
        out = _c.create_string_buffer(len(pt) + 16)
        supp = _c.create_string_buffer(16)
        self.lib.ref_seal_supp(len(key) * 8, _buf(key), _buf(iv), seq, _buf(aad), len(aad), _buf(pt), len(pt), out,
                               _buf(hp_key), supp_off, supp)
        return out.raw, supp.raw

    def seal_iv96(self, key, iv, xor_bytes, seq, aad, pt):
        out = _c.create_string_buffer(len(pt) + 16)
        self.lib.ref_seal_iv96(len(key) * 8, _buf(key), _buf(iv), _buf(xor_bytes), len(xor_bytes), seq, _buf(aad),
                               len(aad), _buf(pt), len(pt), out)
        return out.raw

    def seal_reiv(self, key, iv, iv2, seq, aad, pt):
        """keyed with iv, IV-only re-setup to iv2 (setup_crypto(ctx, 1, NULL, iv2)), then seal"""
        out = _c.create_string_buffer(len(pt) + 16)
        n = self.lib.ref_seal_reiv(len(key) * 8, _buf(key), _buf(iv), _buf(iv2), seq, _buf(aad), len(aad), _buf(pt), len(pt),
                                   out)
        assert n == len(pt) + 16
        return out.raw

    def algo(self, name):
        return _c.addressof(_c.c_char.in_dll(self.lib, name))

    def open(self, key, iv, seq, aad, ct):
        out = _c.create_string_buffer(max(len(ct), 16))
        n = self.lib.ref_open(len(key) * 8, _buf(key), _buf(iv), seq, _buf(aad), len(aad), _buf(ct), len(ct), out)
        return (None if n == SIZE_MAX else n), out.raw[: max(len(ct) - 16, 0)]


def tls13_wire(oracle, key, iv, seq, ctype, payload):
    """Restatement of picotls's TLS 1.3 send path (buffer_push_encrypted_records + aead_encrypt + build_aad,
    lib/picotls.c:696-715, :747-794): 16384-byte chunks, header 17 03 03 BE16(chunk + 17) as the AAD,
    plaintext chunk || content type, one sequence number per record.  Checked against ptls_send itself."""
    out = []
    for j, pos in enumerate(range(0, len(payload), 16384)):
        chunk = payload[pos:pos + 16384]
        hdr = bytes([0x17, 0x03, 0x03]) + (len(chunk) + 17).to_bytes(2, "big")
        out.append(hdr + oracle.seal(key, iv, seq + j, hdr, chunk + bytes([ctype])))
    return b"".join(out)


class RefTLS:
    """A post-handshake TLS 1.3 connection of the REFERENCE (ptls_import from traffic secrets, then its own
    ptls_send / ptls_receive record layer, lib/picotls.c:5334-5432, :6061-6145).  `aead` = address of a
    ptls_aead_algorithm_t (None = minicrypto's AES-GCM: fusion's do_encrypt_v is a stub, lib/fusion.c:1145)."""

    def __init__(self, bits, enc_secret, dec_secret, enc_seq=0, dec_seq=0, aead=None, is_server=1):
        L = self.lib = _c.CDLL(REF_SO)
        L.ref_tls13_import.restype = _c.c_void_p
        L.ref_tls13_import.argtypes = [_c.c_int, _c.c_void_p, _c.c_int, _u8p, _c.c_uint64, _u8p, _c.c_uint64]
        L.ref_tls13_free.argtypes = [_c.c_void_p]
        L.ref_tls13_send.restype = _c.c_long
        L.ref_tls13_send.argtypes = [_c.c_void_p, _u8p, _c.c_size_t, _u8p, _c.c_size_t]
        L.ref_tls13_receive.restype = _c.c_int
        L.ref_tls13_receive.argtypes = [_c.c_void_p, _u8p, _c.c_size_t, _c.POINTER(_c.c_size_t), _u8p, _c.c_size_t,
                                        _c.POINTER(_c.c_size_t)]
        self.h = L.ref_tls13_import(bits, aead, is_server, _buf(enc_secret), enc_seq, _buf(dec_secret), dec_seq)
        assert self.h, "ptls_import failed"

    def send(self, payload):
        cap = len(payload) + 64 * (len(payload) // 16384 + 2)
        out = _c.create_string_buffer(cap)
        n = self.lib.ref_tls13_send(self.h, _buf(payload), len(payload), out, cap)
        assert n >= 0
        return out.raw[:n]

    def receive(self, wire):
        """(ret, consumed, plaintext) of ONE ptls_receive call"""
        out = _c.create_string_buffer(len(wire) + 16)
        consumed, outlen = _c.c_size_t(), _c.c_size_t()
        ret = self.lib.ref_tls13_receive(self.h, _buf(wire), len(wire), _c.byref(consumed), out, len(wire) + 16,
                                         _c.byref(outlen))
        return ret, consumed.value, out.raw[:outlen.value]

    def close(self):
        if self.h:
            self.lib.ref_tls13_free(self.h)
            self.h = None


class RefTLS12(RefTLS):
    """A post-handshake TLS 1.2 connection of the REFERENCE: ptls_build_tls12_export_params (the reference's PRF
    key block from master_secret and the hello randoms) + ptls_import, then its TLS 1.2 record layer
    (build_tls12_aad, lib/picotls.c:730-739).  `aead` = address of a ptls_aead_algorithm_t (None = fusion's
    ptls_non_temporal_aes{128,256}gcm, lib/fusion.c:2154-2179)."""

    def __init__(self, bits, master_secret, hello_randoms, next_send_record_iv=0, aead=None, is_server=1):
        L = self.lib = _c.CDLL(REF_SO)
        L.ref_tls12_import.restype = _c.c_void_p
        L.ref_tls12_import.argtypes = [_c.c_int, _c.c_void_p, _c.c_int, _u8p, _u8p, _c.c_uint64]
        L.ref_tls13_free.argtypes = [_c.c_void_p]
        L.ref_tls13_send.restype = _c.c_long
        L.ref_tls13_send.argtypes = [_c.c_void_p, _u8p, _c.c_size_t, _u8p, _c.c_size_t]
        L.ref_tls13_receive.restype = _c.c_int
        L.ref_tls13_receive.argtypes = [_c.c_void_p, _u8p, _c.c_size_t, _c.POINTER(_c.c_size_t), _u8p, _c.c_size_t,
                                        _c.POINTER(_c.c_size_t)]
        assert len(master_secret) == 48 and len(hello_randoms) == 64
        self.h = L.ref_tls12_import(bits, aead, is_server, _buf(master_secret), _buf(hello_randoms), next_send_record_iv)
        assert self.h, "ptls_build_tls12_export_params / ptls_import failed"


def ref_ptlsbench(aead_addr, n=1000, l=1500):
    """t/ptlsbench.c bench_run_one (:88-173) on the AEAD object at aead_addr: dict of encrypt / decrypt Mbps
    (ptlsbench's unit) and microseconds per call, wall clock and process CPU time"""
    L = _c.CDLL(REF_SO)
    L.ref_ptlsbench.restype = _c.c_int
    L.ref_ptlsbench.argtypes = [_c.c_void_p, _c.c_size_t, _c.c_size_t] + [_c.POINTER(_c.c_double)] * 4
    v = [_c.c_double() for _ in range(4)]
    rc = L.ref_ptlsbench(aead_addr, n, l, *[_c.byref(x) for x in v])
    assert rc == 0, f"ref_ptlsbench failed ({rc})"
    we, wd, ce, cd = (x.value for x in v)
    mbps = lambda us: round(n * l * 8 / us, 1)  # noqa: E731  (bits per microsecond = Mbps, t/ptlsbench.c:175-183)
    return dict(n=n, l=l, enc_mbps_wall=mbps(we), dec_mbps_wall=mbps(wd), enc_mbps_cpu=mbps(ce), dec_mbps_cpu=mbps(cd),
                enc_us_per_call=round(we / n, 3), dec_us_per_call=round(wd / n, 3))


def ref_hkdf_expand_label(bits, secret, label, outlen):
    """the reference's ptls_hkdf_expand_label with minicrypto SHA-256 (bits 128) / SHA-384 (bits 256), empty context"""
    L = _c.CDLL(REF_SO)
    L.ref_hkdf_expand_label.restype = _c.c_int
    L.ref_hkdf_expand_label.argtypes = [_c.c_int, _u8p, _c.c_size_t, _u8p, _c.c_char_p, _u8p, _c.c_size_t]
    out = _c.create_string_buffer(outlen)
    assert L.ref_hkdf_expand_label(bits, out, outlen, _buf(secret), label, None, 0) == 0
    return out.raw


def ref_traffic_keys(bits, secret):
    """(key, iv) picotls derives from a TLS 1.3 traffic secret: HKDF-Expand-Label "key" / "iv" (lib/picotls.c:6434-6456)"""
    L = _c.CDLL(REF_SO)
    L.ref_hkdf_expand_label.restype = _c.c_int
    L.ref_hkdf_expand_label.argtypes = [_c.c_int, _u8p, _c.c_size_t, _u8p, _c.c_char_p, _u8p, _c.c_size_t]
    key = _c.create_string_buffer(bits // 8)
    iv = _c.create_string_buffer(12)
    assert L.ref_hkdf_expand_label(bits, key, bits // 8, _buf(secret), b"key", None, 0) == 0
    assert L.ref_hkdf_expand_label(bits, iv, 12, _buf(secret), b"iv", None, 0) == 0
    return key.raw, iv.raw
