"""The engine reads and writes exactly each record's bytes: proved at an allocation edge.

fusion over-reads partial blocks inside the page by design (lib/fusion.c:51-60, :345-388) and pins that with
t/fusion.c test_loadn128 (:52-67, every offset of an 8 KiB buffer).  This engine claims more (batch_kernel.h tail_load /
load_block_nb / load_bytes, SURVEY.md §5: a caller's allocation may end at the record's last byte), so the test puts
the last byte of every buffer the kernels touch directly in front of an UNMAPPED page:

* each buffer (plaintext / ciphertext in, AAD, output) is its own anonymous mmap of whole pages plus one trailing page
  set to PROT_NONE; only the data pages are registered with the GPU (ptls_hip_host_register), so a device access past
  them has no mapping at all (a GPU page fault, not a silent read of a neighbour);
* the records are packed back to back and shifted so that the LAST record's bytes (and the last AAD's) end on the last
  byte of the last registered page, with that record's length L mod 16 in {0, 1, 15};
* the kernels read and write those buffers themselves over PCIe (host pipeline, PTLS_HIP_TRANSPORT_MAPPED): short and
  mid-size records (0-200, 300-800 B) go to the batch kernel at 1-2 and 16-32 lanes per record, records of >= 64 GHASH
  elements (1 100-3 000 B) to the wave-per-record kernel (pipeline.cpp mapped_lanes), packed at 1 byte (the
  byte-granular path) or 16 bytes (the aligned path: the last record is then a whole number of blocks, the only way an
  aligned record can end on a page boundary);
* the same buffers through the device-resident batch API at 4 and 8 lanes per record (the planner's choice for
  device-resident c2 / c3 shapes, which the mapped transport never makes), including the deferred-store seal path of
  records packed off the 128-byte line (batch_kernel.h, round 5);
* seal and open are compared with the CPU oracle; a tampered tag must fail.
"""
import ctypes
import mmap

import numpy as np
import pytest
import torch  # (the HIP runtime is torch's, loaded before libptls_hip.so: tests/conftest.py)

import ptls_hip

pytestmark = pytest.mark.gpu
UINT64_MAX = (1 << 64) - 1
PAGE = mmap.PAGESIZE
PROT_NONE = 0  # <sys/mman.h>; the mmap module has no PROT_NONE before Python 3.13

_libc = ctypes.CDLL(None, use_errno=True)
_libc.mmap.restype = ctypes.c_void_p
_libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
_libc.mprotect.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
_libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
_hip = ctypes.CDLL("libamdhip64.so")
_hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]


def _device_ptr(host_addr):
    """the device address of registered host memory (what the mapped transport hands the kernels)"""
    d = ctypes.c_void_p()
    assert _hip.hipHostGetDevicePointer(ctypes.byref(d), ctypes.c_void_p(host_addr), 0) == 0
    return d.value


class GuardedBuffer:
    """`nbytes` of host memory whose last byte is the last byte of a registered page, followed by a PROT_NONE page"""

    def __init__(self, nbytes):
        self.pages = max(1, (nbytes + PAGE - 1) // PAGE)
        self.size = (self.pages + 1) * PAGE
        addr = _libc.mmap(None, self.size, mmap.PROT_READ | mmap.PROT_WRITE, mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS, -1, 0)
        assert addr not in (None, ctypes.c_void_p(-1).value), "mmap failed"
        self.addr = addr
        self.end = addr + self.pages * PAGE  # first byte of the guard page
        assert _libc.mprotect(self.end, PAGE, PROT_NONE) == 0
        self.arr = np.ctypeslib.as_array((ctypes.c_uint8 * (self.pages * PAGE)).from_address(addr))
        self.base = self.end - nbytes  # the caller's buffer: [base, end)
        if ptls_hip.lib().ptls_hip_host_register(addr, self.pages * PAGE) != 0:
            pytest.fail(f"host_register: {ptls_hip.last_error()}")
        self.registered = True

    def view(self):
        off = self.base - self.addr
        return self.arr[off:]

    def close(self):
        if self.registered:
            ptls_hip.lib().ptls_hip_host_unregister(self.addr)
            self.registered = False
        if self.addr:
            _libc.munmap(self.addr, self.size)
            self.addr = 0


def _pack(sizes, align):
    """offsets of back-to-back fields of `sizes` at `align`, and the total with the last field ending the buffer"""
    off, pos = [], 0
    for s in sizes:
        pos = (pos + align - 1) // align * align
        off.append(pos)
        pos += s
    return off, pos


def _records(oracle, kind, last_mod, key_len, align):
    rng = np.random.default_rng(["short", "mid", "long"].index(kind) * 1000 + last_mod * 100 + key_len + align)
    lo, hi = {"short": (0, 200), "mid": (300, 800), "long": (1100, 3000)}[kind]
    n = 60
    lens = [int(rng.integers(lo, hi)) for _ in range(n)]
    last = lens[-1] - lens[-1] % 16 + last_mod
    lens[-1] = last if last >= lo else last + 16
    aad_lens = [int(rng.integers(0, 40)) for _ in range(n)]
    if align == 16:  # an aligned field ends on a page boundary only as whole blocks
        lens[-1] -= lens[-1] % 16
        aad_lens[-1] = 32
    recs = []
    for i, (L, A) in enumerate(zip(lens, aad_lens)):
        key, iv = oracle.gen_key(900 + i * 3 // n, key_len)  # three key runs of 20 records
        recs.append((key, iv, 70 + i, oracle.stream(4000 + i, A), oracle.stream(8000 + i, L)))
    return recs


def _descs(recs, in_sizes, out_sizes, align):
    n = len(recs)
    d = np.zeros(n, dtype=ptls_hip.RECORD_DTYPE)
    in_off, in_total = _pack(in_sizes, align)
    out_off, out_total = _pack(out_sizes, align)
    aad_off, aad_total = _pack([len(r[3]) for r in recs], align)
    d["in_off"], d["out_off"], d["aad_off"] = in_off, out_off, aad_off
    d["len"] = [len(r[4]) for r in recs]
    d["aad_len"] = [len(r[3]) for r in recs]
    d["key"] = [i * 3 // n for i in range(n)]
    d["seq"] = [r[2] for r in recs]
    return d, in_total, out_total, aad_total


@pytest.mark.parametrize("last_mod,align", [(0, 1), (1, 1), (15, 1), (0, 16)])  # aligned: only L mod 16 == 0 can end a page
@pytest.mark.parametrize("kind", ["short", "mid", "long"])
@pytest.mark.parametrize("key_len", [16, 32])
def test_no_access_past_the_last_record(engine, oracle, kind, last_mod, key_len, align):
    recs = _records(oracle, kind, last_mod, key_len, align)
    lens = [len(r[4]) for r in recs]
    ks = ptls_hip.KeySet(engine, key_len, 3)
    keys = [oracle.gen_key(900 + k, key_len) for k in range(3)]
    ks.set(0, b"".join(k for k, _ in keys), b"".join(v for _, v in keys))
    pipe = ptls_hip.Pipeline(engine, 1 << 20, transport=ptls_hip.TRANSPORT_MAPPED)
    bufs = []
    try:
        # ---- seal: plaintext in, ct || tag out, each buffer ending at its guard page ----
        d, in_total, out_total, aad_total = _descs(recs, lens, [L + 16 for L in lens], align)
        g_in, g_aad, g_out = GuardedBuffer(in_total), GuardedBuffer(aad_total), GuardedBuffer(out_total)
        bufs += [g_in, g_aad, g_out]
        if align == 16:
            assert all(g.base % 16 == 0 for g in (g_in, g_aad, g_out))
        vin, vaad, vout = g_in.view(), g_aad.view(), g_out.view()
        for r, e in zip(recs, d):
            vin[e["in_off"]: e["in_off"] + e["len"]] = np.frombuffer(r[4], np.uint8)
            vaad[e["aad_off"]: e["aad_off"] + e["aad_len"]] = np.frombuffer(r[3], np.uint8)
        assert int(d[-1]["in_off"]) + lens[-1] == in_total and int(d[-1]["aad_off"]) + len(recs[-1][3]) == aad_total
        pipe.seal(ks, d, g_in.base, g_aad.base, g_out.base)
        assert pipe.last_transport == ptls_hip.TRANSPORT_MAPPED
        sealed = [vout[e["out_off"]: e["out_off"] + e["len"] + 16].tobytes() for e in d]
        bad = [i for i, (r, s) in enumerate(zip(recs, sealed)) if s != oracle.seal(*r)]
        assert not bad, f"seal mismatches at {bad[:8]}"
        # ---- open: ct || tag in, plaintext out; one tampered tag ----
        d2, in2, out2, _ = _descs(recs, [L + 16 for L in lens], lens, align)
        g_in2, g_out2 = GuardedBuffer(in2), GuardedBuffer(out2)
        bufs += [g_in2, g_out2]
        vin2, vout2 = g_in2.view(), g_out2.view()
        for s, e in zip(sealed, d2):
            vin2[e["in_off"]: e["in_off"] + len(s)] = np.frombuffer(s, np.uint8)
        d2["aad_off"] = d["aad_off"]  # the AAD buffer is the seal's
        tamper = len(recs) // 2
        vin2[int(d2[tamper]["in_off"]) + lens[tamper] + 3] ^= 0x10
        res = np.zeros(len(recs), dtype=np.uint64)
        pipe.open(ks, d2, g_in2.base, g_aad.base, g_out2.base, res)
        want = [UINT64_MAX if i == tamper else L for i, L in enumerate(lens)]
        assert [int(x) for x in res] == want
        pts = [vout2[e["out_off"]: e["out_off"] + e["len"]].tobytes() for e in d2]
        assert pts == [r[4] for r in recs]
    finally:
        pipe.close()
        ks.close()
        for b in bufs:
            b.close()


@pytest.mark.parametrize("last_mod,align", [(0, 1), (15, 1), (0, 16)])
@pytest.mark.parametrize("kind", ["mid", "long"])
@pytest.mark.parametrize("lanes", [4, 8])
def test_no_access_past_the_last_record_batch_lanes(engine, oracle, lanes, kind, last_mod, align):
    """the guarded buffers through ptls_hip_aesgcm_seal_batch / open_batch at a forced 4 or 8 lanes per record (ADVICE
    r05): the kernels address the registered pages by their device mapping, the last record ends on the last byte"""
    recs = _records(oracle, kind, last_mod, 16, align)
    lens = [len(r[4]) for r in recs]
    ks = ptls_hip.KeySet(engine, 16, 3)
    keys = [oracle.gen_key(900 + k, 16) for k in range(3)]
    ks.set(0, b"".join(k for k, _ in keys), b"".join(v for _, v in keys))
    bufs = []
    try:
        d, in_total, out_total, aad_total = _descs(recs, lens, [L + 16 for L in lens], align)
        g_in, g_aad, g_out = GuardedBuffer(in_total), GuardedBuffer(aad_total), GuardedBuffer(out_total)
        bufs += [g_in, g_aad, g_out]
        vin, vaad, vout = g_in.view(), g_aad.view(), g_out.view()
        for r, e in zip(recs, d):
            vin[e["in_off"]: e["in_off"] + e["len"]] = np.frombuffer(r[4], np.uint8)
            vaad[e["aad_off"]: e["aad_off"] + e["aad_len"]] = np.frombuffer(r[3], np.uint8)
        b = ptls_hip.Batch(engine, d)
        b.set_lanes(lanes)
        assert b.lanes == lanes
        b.seal(ks, _device_ptr(g_in.base), _device_ptr(g_aad.base), _device_ptr(g_out.base))
        torch.cuda.synchronize()
        sealed = [vout[e["out_off"]: e["out_off"] + e["len"] + 16].tobytes() for e in d]
        bad = [i for i, (r, s) in enumerate(zip(recs, sealed)) if s != oracle.seal(*r)]
        assert not bad, f"seal mismatches at {bad[:8]}"
        d2, in2, out2, _ = _descs(recs, [L + 16 for L in lens], lens, align)
        d2["aad_off"] = d["aad_off"]
        g_in2, g_out2 = GuardedBuffer(in2), GuardedBuffer(out2)
        bufs += [g_in2, g_out2]
        vin2, vout2 = g_in2.view(), g_out2.view()
        for s_, e in zip(sealed, d2):
            vin2[e["in_off"]: e["in_off"] + len(s_)] = np.frombuffer(s_, np.uint8)
        tamper = len(recs) // 3
        vin2[int(d2[tamper]["in_off"]) + lens[tamper] + 1] ^= 0x01
        b2 = ptls_hip.Batch(engine, d2)
        b2.set_lanes(lanes)
        res = torch.zeros(len(recs), dtype=torch.int64, device="cuda")
        b2.open(ks, _device_ptr(g_in2.base), _device_ptr(g_aad.base), _device_ptr(g_out2.base), res)
        torch.cuda.synchronize()
        want = [UINT64_MAX if i == tamper else L for i, L in enumerate(lens)]
        assert [int(x) & UINT64_MAX for x in res.cpu().numpy()] == want
        assert [vout2[e["out_off"]: e["out_off"] + e["len"]].tobytes() for e in d2] == [r[4] for r in recs]
        b.close()
        b2.close()
    finally:
        ks.close()
        for g in bufs:
            g.close()
