"""Single-record plugin calls at every size around the two-wave record (sparse_kernel.hip mw_record: 65..128 GHASH
elements go to two waves, one element per lane; fewer stay on one wave; more run on two pairs of waves at stride 128,
sparse_record S = 128, each pair on its own part of the record), through the reference's own picotls (ptls_aead_new_direct / ptls_aead_encrypt / ptls_aead_decrypt /
ptls_aead_encrypt_s, tests/plugin_driver.py) and compared with lib/fusion.c (oracle/_ref) in the same process: every GHASH
length N from 60 to 134 with AADs of 0 to 3 blocks, and long records of 2 000 B to 17 KB with AADs of up to 128 blocks, both
key sizes, seal, open, a tampered tag or ciphertext, and QUIC header protection fused into the call.  Each case runs in its
own process, with the resident worker (default) and with one launch per call (PTLS_HIP_PLUGIN_WORKER=0)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CASE = r"""
import sys
sys.path[:0] = {paths!r}
import numpy as np
import plugin_driver
from oracle_lib import Ref
drv, ref = plugin_driver.PluginDriver(), Ref()
rng = np.random.default_rng({seed})

def rnd(n):
    return rng.integers(0, 256, n, dtype=np.uint8).tobytes()

calls = 0
for bits in (128, 256):
    key, iv = rnd(bits // 8), rnd(12)
    enc, dec = drv.new(bits, key, iv, 1), drv.new(bits, key, iv, 0)
    hp_key = rnd(bits // 8)
    cctx = drv.cipher_new(bits, hp_key)
    for A in (0, 5, 13, 17, 40):
        na = (A + 15) // 16
        for N in range(60, 135):
            nc = N - na - 1
            if nc < 0:
                continue
            for L in sorted({{max(0, 16 * nc - d) for d in (0, 7, 15)}}):
                if (L + 15) // 16 != nc:
                    continue
                seq = int(rng.integers(0, 2 ** 40))
                pt, aad = rnd(L), rnd(A)
                ct = drv.encrypt(enc, pt, seq, aad)
                assert ct == ref.seal(key, iv, seq, aad, pt), ("seal", bits, A, N, L)
                assert drv.decrypt(dec, ct, seq, aad) == pt, ("open", bits, A, N, L)
                bad = bytearray(ct)
                bad[-1 - (L % 16)] ^= 0x40
                assert drv.decrypt(dec, bytes(bad), seq, aad) is None, ("tamper", bits, A, N, L)
                if L >= 20 and L % 3 == 0:
                    out, supp = drv.encrypt_s(enc, pt, seq, aad, cctx, L % 4)
                    assert (out, supp) == ref.seal_supp(key, iv, seq, aad, pt, hp_key, L % 4), ("supp", bits, A, N, L)
                calls += 1
    # long records: two pairs of waves at stride 128 (sparse_record S = 128, SPLIT), around the 128-element switch, where
    # pair 0's part grows by 128 data blocks (N = 255 / 256 / 511 / 512), up to TLS's 16 KiB, and a 128-block AAD (pair 0's
    # part all AAD, pair 1's down to the length block)
    for A in (0, 5, 13, 100, 2048):
        for L in ((2000, 2015, 2016, 2017, 2047, 2048, 2049, 3000, 4064, 4080, 4095, 4096, 4097, 8160, 8176, 8191, 8192, 10007,
                   16383, 16384, 16385, int(rng.integers(2100, 17000))) if A < 2048 else (0, 1, 100, 2100, 14000)):
            seq = int(rng.integers(0, 2 ** 40))
            pt, aad = rnd(L), rnd(A)
            ct = drv.encrypt(enc, pt, seq, aad)
            assert ct == ref.seal(key, iv, seq, aad, pt), ("seal long", bits, A, L)
            assert drv.decrypt(dec, ct, seq, aad) == pt, ("open long", bits, A, L)
            bad = bytearray(ct)
            bad[L // 2] ^= 0x01
            assert drv.decrypt(dec, bytes(bad), seq, aad) is None, ("tamper long", bits, A, L)
            if L >= 16:
                out, supp = drv.encrypt_s(enc, pt, seq, aad, cctx, L - 16)
                assert (out, supp) == ref.seal_supp(key, iv, seq, aad, pt, hp_key, L - 16), ("supp long", bits, A, L)
            calls += 1
    drv.cipher_free(cctx)
    drv.free(enc)
    drv.free(dec)
print("ok", calls)
"""


@pytest.mark.parametrize("worker", ["1", "0"])
def test_plugin_record_sizes_around_two_waves(worker):
    from oracle_lib import Ref
    if not Ref.available:
        pytest.skip("oracle/_ref not built")
    paths = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "hsig-picotls_amd"), ROOT]
    env = dict(os.environ, PTLS_HIP_PLUGIN_WORKER=worker)
    r = subprocess.run([sys.executable, "-c", _CASE.format(paths=paths, seed=17 + int(worker))], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().startswith("ok"), (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
