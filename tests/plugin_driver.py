"""Drive an AEAD engine the way a picotls application does, using the REFERENCE's own lifecycle code.

ptls_aead_new_direct / ptls_aead_free / ptls_aead_xor_iv come from oracle/_ref/libptls_fusion_ref.so
(lib/picotls.c:6458-6490, compiled unmodified); the algorithm object is ptls_hip_aes{128,256}gcm from
libptls_hip.so.  The inline dispatchers of include/picotls.h:1993-2055 (ptls_aead_encrypt,
ptls_aead_encrypt_v, ptls_aead_decrypt) are one indirect call each; they are reproduced here with
ctypes through the ptls_aead_context_t vtable.
"""
import ctypes

import ptls_hip
from oracle_lib import REF_SO

c = ctypes
SIZE_MAX = (1 << 64) - 1


class Iovec(c.Structure):
    _fields_ = [("base", c.c_void_p), ("len", c.c_size_t)]


class AeadContext(c.Structure):  # include/picotls.h:444-494
    _fields_ = [(n, c.c_void_p) for n in ("algo", "dispose_crypto", "do_get_iv", "do_set_iv", "do_encrypt_init",
                                            "do_encrypt_update", "do_encrypt_final", "do_encrypt", "do_encrypt_v",
                                            "do_decrypt")]


class CipherContext(c.Structure):  # include/picotls.h:397-403
    _fields_ = [(n, c.c_void_p) for n in ("algo", "do_dispose", "do_init", "do_transform")]


class Supp(c.Structure):  # ptls_aead_supplementary_encryption_t, include/picotls.h:421-436
    _fields_ = [("ctx", c.c_void_p), ("input", c.c_void_p), ("output", c.c_uint8 * 16)]


CIPHER_INIT = c.CFUNCTYPE(None, c.c_void_p, c.c_void_p)
CIPHER_TRANSFORM = c.CFUNCTYPE(None, c.c_void_p, c.c_void_p, c.c_void_p, c.c_size_t)
ENCRYPT = c.CFUNCTYPE(None, c.c_void_p, c.c_void_p, c.c_void_p, c.c_size_t, c.c_uint64, c.c_void_p, c.c_size_t, c.c_void_p)
ENCRYPT_V = c.CFUNCTYPE(None, c.c_void_p, c.c_void_p, c.POINTER(Iovec), c.c_size_t, c.c_uint64, c.c_void_p, c.c_size_t)
DECRYPT = c.CFUNCTYPE(c.c_size_t, c.c_void_p, c.c_void_p, c.c_void_p, c.c_size_t, c.c_uint64, c.c_void_p, c.c_size_t)


class PluginDriver:
    def __init__(self):
        hip = ptls_hip.lib()
        self.ref = c.CDLL(REF_SO)
        self.ref.ptls_aead_new_direct.restype = c.c_void_p
        self.ref.ptls_aead_new_direct.argtypes = [c.c_void_p, c.c_int, c.c_void_p, c.c_void_p]
        self.ref.ptls_aead_free.argtypes = [c.c_void_p]
        self.ref.ptls_aead_xor_iv.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t]
        self.ref.ptls_cipher_new.restype = c.c_void_p
        self.ref.ptls_cipher_new.argtypes = [c.c_void_p, c.c_int, c.c_void_p]
        self.ref.ptls_cipher_free.argtypes = [c.c_void_p]
        self.algos = {128: c.addressof(c.c_char.in_dll(hip, "ptls_hip_aes128gcm")),
                      256: c.addressof(c.c_char.in_dll(hip, "ptls_hip_aes256gcm"))}
        self.nt_algos = {128: c.addressof(c.c_char.in_dll(hip, "ptls_hip_non_temporal_aes128gcm")),
                         256: c.addressof(c.c_char.in_dll(hip, "ptls_hip_non_temporal_aes256gcm"))}
        self.ctr_algos = {128: c.addressof(c.c_char.in_dll(hip, "ptls_hip_aes128ctr")),
                          256: c.addressof(c.c_char.in_dll(hip, "ptls_hip_aes256ctr"))}

    def cipher_new(self, bits, key, is_enc=1):
        """ptls_cipher_new (lib/picotls.c) on ptls_hip_aes{128,256}ctr"""
        ctx = self.ref.ptls_cipher_new(self.ctr_algos[bits], is_enc, key)
        assert ctx, "ptls_cipher_new returned NULL: " + ptls_hip.last_error()
        return ctx

    def cipher_free(self, ctx):
        self.ref.ptls_cipher_free(ctx)

    @staticmethod
    def cipher_encrypt(ctx, iv, data):
        """ptls_cipher_init + ptls_cipher_encrypt (include/picotls.h inline dispatchers)"""
        vt = CipherContext.from_address(ctx)
        CIPHER_INIT(vt.do_init)(ctx, iv)
        out = c.create_string_buffer(max(len(data), 1))
        CIPHER_TRANSFORM(vt.do_transform)(ctx, out, data, len(data))
        return out.raw[:len(data)]

    def new(self, bits, key, iv, is_enc=1, non_temporal=False):
        algo = (self.nt_algos if non_temporal else self.algos)[bits]
        ctx = self.ref.ptls_aead_new_direct(algo, is_enc, key, iv)
        assert ctx, "ptls_aead_new_direct returned NULL: " + ptls_hip.last_error()
        return ctx

    def free(self, ctx):
        self.ref.ptls_aead_free(ctx)

    def xor_iv(self, ctx, data):
        self.ref.ptls_aead_xor_iv(ctx, data, len(data))

    @staticmethod
    def _vt(ctx):
        return AeadContext.from_address(ctx)

    def encrypt(self, ctx, pt, seq, aad):
        out = c.create_string_buffer(len(pt) + 16)
        ENCRYPT(self._vt(ctx).do_encrypt)(ctx, out, pt, len(pt), seq, aad, len(aad), None)
        return out.raw

    def encrypt_s(self, ctx, pt, seq, aad, supp_ctx, sample_off):
        """ptls_aead_encrypt_s with a supplementary (header-protection) block sampled from the output"""
        out = c.create_string_buffer(len(pt) + 16)
        supp = Supp(supp_ctx, c.addressof(out) + sample_off)
        ENCRYPT(self._vt(ctx).do_encrypt)(ctx, out, pt, len(pt), seq, aad, len(aad), c.byref(supp))
        return out.raw, bytes(supp.output)

    def encrypt_v(self, ctx, parts, seq, aad):
        bufs = [c.create_string_buffer(p, max(len(p), 1)) for p in parts]
        vec = (Iovec * len(parts))(*[Iovec(c.cast(b, c.c_void_p), len(p)) for b, p in zip(bufs, parts)])
        total = sum(len(p) for p in parts)
        out = c.create_string_buffer(total + 16)
        ENCRYPT_V(self._vt(ctx).do_encrypt_v)(ctx, out, vec, len(parts), seq, aad, len(aad))
        return out.raw

    def decrypt(self, ctx, ct, seq, aad):
        out = c.create_string_buffer(max(len(ct), 1))
        n = DECRYPT(self._vt(ctx).do_decrypt)(ctx, out, ct, len(ct), seq, aad, len(aad))
        return None if n == SIZE_MAX else out.raw[:n]
