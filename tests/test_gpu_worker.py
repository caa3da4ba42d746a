"""The plugin worker (plugin_worker.cpp worker_call, sparse_kernel.hip plugin_worker_kernel): a resident kernel whose workgroups
serve plugin calls from pinned mailboxes (one per calling thread) instead of one launch per call.  Its lifecycle is exercised through the
reference's own picotls lifecycle code (tests/plugin_driver.py) and every output is compared with lib/fusion.c
(oracle/_ref): calls separated by gaps longer than the worker's idle timeout (it leaves, the next call relaunches it),
IV changes (ptls_aead_xor_iv: the IV travels in the request), contexts created and freed between calls (a freed pooled
key slot comes back with other keys once no resident workgroup can hold it), header-protection ECB blocks (through the
worker's mailbox, WREQ_ECB, by default; one launch each with PTLS_HIP_ECB_LAUNCH=1) and fused header protection
interleaved with AEAD calls on the worker, and two threads sharing it.  Each case runs in its own process: worker on
(the default) with ECB blocks through the worker or launched, and worker off (PTLS_HIP_PLUGIN_WORKER=0: one launch per
call).
test_plugin_worker_threads: eight threads with their own contexts at once over 1, 4 and 8 mailboxes (shared homes, the
try-lock hand-off, a workgroup leaving while the others serve), with IV changes, context churn on every thread (pooled
slots recycled while other threads' requests run), records too long for a mailbox (the context's own staging) and gaps
past the idle timeout and the lifetime, every output against lib/fusion.c.
test_plugin_calls_beside_batch_launches: four threads make plugin calls while 1 GiB batch seals run back to back on the
same device (the worker's workgroups hold CUs the batch kernel's workgroups then start late on; neither may stall or
corrupt the other): every plugin output against lib/fusion.c, the batch opened back in full and sampled records against
lib/fusion.c."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CASE = r"""
import sys, time, threading
sys.path[:0] = {paths!r}
import numpy as np
import plugin_driver
from oracle_lib import Ref, Oracle, tls_aad
drv, ref, o = plugin_driver.PluginDriver(), Ref(), Oracle()
rng = np.random.default_rng(11)

def rnd(n):
    return rng.integers(0, 256, n, dtype=np.uint8).tobytes()

def check(ctx_e, ctx_d, key, iv, seq, L, tag):
    pt, aad = rnd(L), tls_aad(L)
    ct = drv.encrypt(ctx_e, pt, seq, aad)
    assert ct == ref.seal(key, iv, seq, aad, pt), (tag, seq, L)
    assert drv.decrypt(ctx_d, ct, seq, aad) == pt, (tag, seq, L)

for bits in (128, 256):
    key, iv = rnd(bits // 8), rnd(12)
    enc, dec = drv.new(bits, key, iv, 1), drv.new(bits, key, iv, 0)
    # gaps longer than the idle timeout (200 us) and the lifetime (2 ms): every call may find the worker gone
    for i, gap in enumerate((0, 0.0005, 0, 0.003, 0.0002, 0, 0.01, 0)):
        time.sleep(gap)
        check(enc, dec, key, iv, i, int(rng.integers(0, 2000)), "gap")
    # IV changes between back-to-back calls
    for i in range(6):
        x = rnd(int(rng.integers(1, 13)))
        drv.xor_iv(enc, x)
        drv.xor_iv(dec, x)
        iv = bytes(a ^ b for a, b in zip(iv, x + bytes(12 - len(x))))
        check(enc, dec, key, iv, 100 + i, int(rng.integers(0, 1500)), "xor_iv")
    drv.free(enc)
    drv.free(dec)
    # contexts created and freed between calls: slots (and their addresses) change hands under a busy worker
    for i in range(12):
        k2, iv2 = rnd(bits // 8), rnd(12)
        e2, d2 = drv.new(bits, k2, iv2, 1), drv.new(bits, k2, iv2, 0)
        check(e2, d2, k2, iv2, i, int(rng.integers(0, 600)), "churn")
        drv.free(e2)
        drv.free(d2)
    # header protection: ECB blocks and fused supp calls interleaved with AEAD calls
    hp_key = rnd(bits // 8)
    cctx = drv.cipher_new(bits, hp_key)
    key, iv = rnd(bits // 8), rnd(12)
    actx = drv.new(bits, key, iv)
    for i in range(20):
        civ = rnd(16)
        assert drv.cipher_encrypt(cctx, civ, bytes(16)) == o.aes_ecb(hp_key, civ), ("ecb", i)
        L = int(rng.integers(20, 1300))
        text, aad = rnd(L), rnd(20)
        out, supp = drv.encrypt_s(actx, text, i, aad, cctx, 3)
        assert (out, supp) == ref.seal_supp(key, iv, i, aad, text, hp_key, 3), ("supp", i)
    drv.free(actx)
    drv.cipher_free(cctx)

# two threads, each with its own contexts, calling through the one worker at once
errors = []
def worker_thread(t):
    try:
        r = np.random.default_rng(100 + t)
        key, iv = r.integers(0, 256, 16, dtype=np.uint8).tobytes(), r.integers(0, 256, 12, dtype=np.uint8).tobytes()
        e, d = drv.new(128, key, iv, 1), drv.new(128, key, iv, 0)
        for i in range(150):
            L = int(r.integers(0, 1500))
            pt, aad = r.integers(0, 256, L, dtype=np.uint8).tobytes(), tls_aad(L)
            ct = drv.encrypt(e, pt, i, aad)
            assert ct == ref.seal(key, iv, i, aad, pt), ("thread", t, i)
            assert drv.decrypt(d, ct, i, aad) == pt, ("thread", t, i)
        drv.free(e)
        drv.free(d)
    except Exception as ex:  # noqa: BLE001
        errors.append(repr(ex))
ts = [threading.Thread(target=worker_thread, args=(t,)) for t in range(2)]
for t in ts:
    t.start()
for t in ts:
    t.join()
assert not errors, errors
print("ok")
"""


_CASE_MT = r"""
import sys, time, threading
sys.path[:0] = {paths!r}
import numpy as np
import plugin_driver
from oracle_lib import Ref, tls_aad
drv, ref = plugin_driver.PluginDriver(), Ref()
errors = []

def thread_main(t):
    try:
        r = np.random.default_rng(1000 + t)
        rb = lambda n: r.integers(0, 256, n, dtype=np.uint8).tobytes()  # noqa: E731
        bits = 128 if t % 2 == 0 else 256
        key, iv = rb(bits // 8), rb(12)
        e, d = drv.new(bits, key, iv, 1), drv.new(bits, key, iv, 0)
        for i in range(60):
            if i % 15 == 7:  # a new connection on this thread: the old contexts go back to the pool
                drv.free(e)
                drv.free(d)
                key, iv = rb(bits // 8), rb(12)
                e, d = drv.new(bits, key, iv, 1), drv.new(bits, key, iv, 0)
            if i % 11 == 5:
                x = rb(int(r.integers(1, 13)))
                drv.xor_iv(e, x)
                drv.xor_iv(d, x)
                iv = bytes(a ^ b for a, b in zip(iv, x + bytes(12 - len(x))))
            if i % 20 == 13:
                time.sleep(0.003)  # past the idle timeout and the lifetime of the dispatch
            L = int(r.choice([0, 1, 15, 16, 17, 700, 1350, 1500, 4096, 16384, 17000, 20000]))
            pt, aad = rb(L), tls_aad(L)
            ct = drv.encrypt(e, pt, i, aad)
            assert ct == ref.seal(key, iv, i, aad, pt), ("seal", t, i, L)
            assert drv.decrypt(d, ct, i, aad) == pt, ("open", t, i, L)
            bad = bytearray(ct)
            if bad:
                bad[-1] ^= 1
                assert drv.decrypt(d, bytes(bad), i, aad) is None, ("tamper", t, i, L)
        drv.free(e)
        drv.free(d)
    except Exception as ex:  # noqa: BLE001
        errors.append(repr(ex))

ts = [threading.Thread(target=thread_main, args=(t,)) for t in range(8)]
for t in ts:
    t.start()
for t in ts:
    t.join()
assert not errors, errors
print("ok")
"""


_CASE_BESIDE = r"""
import sys, threading
sys.path[:0] = {paths!r}
import torch
torch.zeros(1, device="cuda")  # torch's HIP runtime first (the plugin's own initialisation otherwise hides the GPU from it)
import numpy as np
import ptls_hip
import plugin_driver
from oracle_lib import Ref, tls_aad
drv, ref = plugin_driver.PluginDriver(), Ref()
eng = ptls_hip.Engine(0)
rng = np.random.default_rng(21)
n, L = 65536, 16384
recs, in_total, out_total, aad_total = ptls_hip.layout_records(np.full(n, L), np.full(n, 5), np.zeros(n, np.uint32),
                                                               np.arange(n, dtype=np.uint64), align=128)
key, iv = rng.bytes(16), rng.bytes(12)
ks = ptls_hip.KeySet(eng, 16, 1)
ks.set(0, key, iv)
sb = ptls_hip.Batch(eng, recs)
ro = recs.copy()
ro["in_off"], ro["out_off"] = recs["out_off"], recs["in_off"]
ob = ptls_hip.Batch(eng, ro)
ob.set_lanes(sb.lanes)
pt = torch.randint(0, 256, (in_total,), dtype=torch.uint8, device="cuda")
aad_h = np.zeros(aad_total, dtype=np.uint8)
for i in range(n):
    o = int(recs["aad_off"][i])
    aad_h[o:o + 5] = np.frombuffer(tls_aad(L), dtype=np.uint8)
aad = torch.from_numpy(aad_h).cuda()
ct = torch.zeros(out_total, dtype=torch.uint8, device="cuda")
back = torch.zeros(in_total, dtype=torch.uint8, device="cuda")
res = torch.zeros(n, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()

stop, errors, calls = threading.Event(), [], [0] * 4
def caller(t):
    try:
        r = np.random.default_rng(300 + t)
        bits = 128 if t % 2 == 0 else 256
        k2, iv2 = r.bytes(bits // 8), r.bytes(12)
        e, d = drv.new(bits, k2, iv2, 1), drv.new(bits, k2, iv2, 0)
        i = 0
        while not stop.is_set() or i < 50:
            m = int(r.choice([0, 17, 1350, 1500, 4096, 16384]))
            p, a = r.bytes(m), tls_aad(m)
            c = drv.encrypt(e, p, i, a)
            assert c == ref.seal(k2, iv2, i, a, p), ("seal", t, i, m)
            assert drv.decrypt(d, c, i, a) == p, ("open", t, i, m)
            i += 1
        calls[t] = i
        drv.free(e)
        drv.free(d)
    except Exception as ex:  # noqa: BLE001
        errors.append(repr(ex))
        stop.set()
ts = [threading.Thread(target=caller, args=(t,)) for t in range(4)]
for t in ts:
    t.start()
for rep in range(40):
    sb.seal(ks, pt, aad, ct)
    if rep % 8 == 0:
        torch.cuda.synchronize()
torch.cuda.synchronize()
stop.set()
for t in ts:
    t.join()
assert not errors, errors
ob.open(ks, ct, aad, back, res)
torch.cuda.synchronize()
assert bool((res == L).all()), "a record failed to open"
assert torch.equal(back, pt), "the opened plaintext differs"
ct_h, pt_h = ct.cpu().numpy(), pt.cpu().numpy()
for i in (0, 1, 4097, 32768, n - 1):
    io, oo = int(recs["in_off"][i]), int(recs["out_off"][i])
    want = ref.seal(key, iv, i, tls_aad(L), pt_h[io:io + L].tobytes())
    assert ct_h[oo:oo + L + 16].tobytes() == want, ("batch record", i)
print("calls", calls)
print("ok")
"""


def test_plugin_calls_beside_batch_launches():
    from oracle_lib import Ref
    if not Ref.available:
        pytest.skip("oracle/_ref not built")
    paths = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "hsig-picotls_amd"), ROOT]
    env = dict(os.environ, PTLS_HIP_PLUGIN_WORKER="1")
    r = subprocess.run([sys.executable, "-c", _CASE_BESIDE.format(paths=paths)], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.returncode, r.stdout[-2000:], r.stderr[-3000:])


@pytest.mark.parametrize("workers", ["1", "4", "8"])
def test_plugin_worker_threads(workers):
    from oracle_lib import Ref
    if not Ref.available:
        pytest.skip("oracle/_ref not built")
    paths = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "hsig-picotls_amd"), ROOT]
    env = dict(os.environ, PTLS_HIP_PLUGIN_WORKER="1", PTLS_HIP_PLUGIN_WORKERS=workers)
    r = subprocess.run([sys.executable, "-c", _CASE_MT.format(paths=paths)], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.returncode, r.stdout[-2000:], r.stderr[-3000:])


@pytest.mark.parametrize("worker,ecb_launch", [("1", "0"), ("1", "1"), ("0", "0")])
def test_plugin_worker_lifecycle(worker, ecb_launch):
    from oracle_lib import Ref
    if not Ref.available:
        pytest.skip("oracle/_ref not built")
    paths = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "hsig-picotls_amd"), ROOT]
    env = dict(os.environ, PTLS_HIP_PLUGIN_WORKER=worker, PTLS_HIP_ECB_LAUNCH=ecb_launch)
    r = subprocess.run([sys.executable, "-c", _CASE.format(paths=paths)], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
