"""GPU tests of the multi-device node (ptls_hip_node_*) and of the host-buffer safety rules of the
host pipeline and the plugin staging.  Bar: bit-exact against the CPU oracle (oracle/, pinned by lib/fusion.c)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import ptls_hip
from oracle_lib import tls_aad

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRANSPORTS = {"copy": ptls_hip.TRANSPORT_COPY, "mapped": ptls_hip.TRANSPORT_MAPPED}


def _records(oracle, n, key_len, nkeys, seed, max_len=20000):
    """n records over nkeys keys (key-major), mixed lengths incl. 0, 1, 15, 16 and long ones, TLS-header AAD"""
    rng = np.random.default_rng(seed)
    out, slots = [], []
    for i in range(n):
        L = int(rng.choice([0, 1, 15, 16, 100, 1350, 4096, 16384, int(rng.integers(0, max_len))]))
        k = i * nkeys // n
        key, iv = oracle.gen_key(700 + k, key_len)
        out.append((key, iv, i, tls_aad(L), oracle.gen_record(50000 + i, L)))
        slots.append(k)
    return out, slots


def _host_buffers(recs_in, recs, in_total, out_total, aad_total):
    h_in = torch.zeros(in_total + 16, dtype=torch.uint8).pin_memory()
    h_aad = torch.zeros(aad_total + 16, dtype=torch.uint8).pin_memory()
    h_out = torch.zeros(out_total + 16, dtype=torch.uint8).pin_memory()
    hin, haad = h_in.numpy(), h_aad.numpy()
    for r, rec in zip(recs_in, recs):
        hin[rec["in_off"]: rec["in_off"] + len(r[4])] = np.frombuffer(r[4], np.uint8)
        haad[rec["aad_off"]: rec["aad_off"] + len(r[3])] = np.frombuffer(r[3], np.uint8)
    return h_in, h_aad, h_out


@pytest.mark.parametrize("transport", ["mapped", "copy"])
@pytest.mark.parametrize("key_len", [16, 32])
def test_node_splits_one_batch_over_two_engines(oracle, transport, key_len):
    """one batch over a node of two engines (both on device 0 here; one per GPU on a node): byte-balanced contiguous
    ranges (ptls_hip_partition_bytes), each sealed and opened by its own host thread and pipeline; every record equals
    the oracle's, opens back, and a tampered record fails on whichever device holds it"""
    n, nkeys = 900, 3
    recs_in, slots = _records(oracle, n, key_len, nkeys, seed=21 + key_len)
    lens = [len(r[4]) for r in recs_in]
    recs, in_total, out_total, aad_total = ptls_hip.layout_records(lens, [5] * n, slots, np.arange(n), align=16,
                                                                   tag_in_input=True)
    node = ptls_hip.Node([0, 0], key_len, nkeys, slice_bytes=1 << 20, transport=TRANSPORTS[transport])
    try:
        keys = [oracle.gen_key(700 + k, key_len) for k in range(nkeys)]
        node.set_keys(0, b"".join(k for k, _ in keys), b"".join(v for _, v in keys))
        h_in, h_aad, h_out = _host_buffers(recs_in, recs, in_total, out_total, aad_total)
        node.seal(recs, h_in, h_aad, h_out)
        sec, bounds = node.last_split()
        assert bounds == ptls_hip.partition_bytes(recs, 2) and 0 < bounds[1] < n
        share = [sum(lens[bounds[d]:bounds[d + 1]]) for d in range(2)]
        assert abs(share[0] - share[1]) <= 2 * max(lens)
        assert all(s > 0 for s in sec)
        hout = h_out.numpy()
        sealed = [hout[rec["out_off"]: rec["out_off"] + len(r[4]) + 16].tobytes() for r, rec in zip(recs_in, recs)]
        bad = [i for i, (r, s_) in enumerate(zip(recs_in, sealed)) if s_ != oracle.seal(*r)]
        assert not bad, f"{len(bad)} mismatches, first {bad[:8]}"
        hin = h_in.numpy()
        hin[:] = 0
        for s_, rec in zip(sealed, recs):
            hin[rec["in_off"]: rec["in_off"] + len(s_)] = np.frombuffer(s_, np.uint8)
        tampered = [i for i in (3, n - 5) if lens[i] > 0]
        for i in tampered:
            hin[recs["in_off"][i]] ^= 1
        h_res = torch.zeros(n, dtype=torch.int64).pin_memory()
        h_out.zero_()
        node.open(recs, h_in, h_aad, h_out, h_res)
        res = [int(x) & ((1 << 64) - 1) for x in h_res.numpy()]
        for i, L in enumerate(lens):
            assert res[i] == (ptls_hip.UINT64_MAX if i in tampered else L), i
            if i not in tampered:
                assert hout[recs["out_off"][i]: recs["out_off"][i] + L].tobytes() == recs_in[i][4]
    finally:
        node.close()


def test_partly_registered_input_is_refused(engine, oracle):
    """a buffer registered only in part must never reach the zero-copy transport (the kernel would touch
    unmapped host pages over PCIe), and the copy engines refuse it too (hipMemcpyAsync: invalid argument): every
    transport returns EINVAL before anything runs.  Registered over all its bytes, the same buffer goes zero-copy."""
    n = 64
    recs_in = [(*oracle.gen_key(5, 16), i, tls_aad(16000), oracle.gen_record(77000 + i, 16000)) for i in range(n)]
    recs, in_total, out_total, aad_total = ptls_hip.layout_records([16000] * n, [5] * n, [0] * n, np.arange(n), align=16,
                                                                   tag_in_input=True)
    ks = ptls_hip.KeySet(engine, 16, 1)
    ks.set(0, *oracle.gen_key(5, 16))
    page = 4096
    raw = np.zeros(in_total + 3 * page, dtype=np.uint8)
    off = (-raw.ctypes.data) % page
    buf = raw[off: off + in_total + page]  # page-aligned view; first only half of it gets registered
    for r, rec in zip(recs_in, recs):
        buf[rec["in_off"]: rec["in_off"] + len(r[4])] = np.frombuffer(r[4], np.uint8)
    half = (in_total // 2) // page * page
    h_aad = torch.zeros(aad_total + 16, dtype=torch.uint8).pin_memory()
    for r, rec in zip(recs_in, recs):
        h_aad.numpy()[rec["aad_off"]: rec["aad_off"] + 5] = np.frombuffer(r[3], np.uint8)
    h_out = torch.zeros(out_total + 16, dtype=torch.uint8).pin_memory()
    pipe = ptls_hip.Pipeline(engine, 1 << 20)
    assert ptls_hip.lib().ptls_hip_host_register(buf.ctypes.data, half) == 0, ptls_hip.last_error()
    try:
        for tr in (ptls_hip.TRANSPORT_MAPPED, ptls_hip.TRANSPORT_AUTO, ptls_hip.TRANSPORT_COPY):
            pipe.set_transport(tr)
            with pytest.raises(ptls_hip.HipError, match="registered only in part"):
                pipe.seal(ks, recs, buf, h_aad, h_out)
    finally:
        ptls_hip.lib().ptls_hip_host_unregister(buf.ctypes.data)
    assert ptls_hip.lib().ptls_hip_host_register(buf.ctypes.data, len(buf)) == 0, ptls_hip.last_error()
    try:
        pipe.set_transport(ptls_hip.TRANSPORT_AUTO)
        pipe.seal(ks, recs, buf, h_aad, h_out)
        assert pipe.last_transport == ptls_hip.TRANSPORT_MAPPED
        hout = h_out.numpy()
        for r, rec in zip(recs_in, recs):
            assert hout[rec["out_off"]: rec["out_off"] + len(r[4]) + 16].tobytes() == oracle.seal(*r)
    finally:
        ptls_hip.lib().ptls_hip_host_unregister(buf.ctypes.data)
        pipe.close()
        ks.close()


_BACK_TO_BACK = r"""
import sys
sys.path[:0] = {paths!r}
import numpy as np
import plugin_driver
from oracle_lib import Ref, Oracle, tls_aad
drv, ref, o = plugin_driver.PluginDriver(), Ref(), Oracle()
rng = np.random.default_rng(5)
for bits in (128, 256):
    key, iv = o.gen_key(bits, bits // 8)
    enc, dec = drv.new(bits, key, iv, 1), drv.new(bits, key, iv, 0)
    for i in range(300):
        L = int(rng.integers(0, 3000))
        pt, aad = o.gen_record(90000 + i, L), tls_aad(L)
        ct = drv.encrypt(enc, pt, i, aad)
        assert ct == ref.seal(key, iv, i, aad, pt), (bits, i, L)
        assert drv.decrypt(dec, ct, i, aad) == pt, (bits, i, L)
    drv.free(enc)
    drv.free(dec)
print("ok")
"""


@pytest.mark.parametrize("coherent", ["0", "1"])
def test_plugin_back_to_back_records_any_host_coherence(coherent):
    """the plugin's staging is allocated fine-grained (hipHostMallocCoherent) whatever HIP_HOST_COHERENT
    says, so 300 different records sealed and opened back to back through ONE context (no stream synchronize between
    calls) equal lib/fusion.c each, with HIP_HOST_COHERENT=0 and =1 set explicitly"""
    from oracle_lib import Ref
    if not Ref.available:
        pytest.skip("oracle/_ref not built")
    paths = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "hsig-picotls_amd"), ROOT]
    env = dict(os.environ, HIP_HOST_COHERENT=coherent)
    r = subprocess.run([sys.executable, "-c", _BACK_TO_BACK.format(paths=paths)], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-3000:]
