"""ctypes binding of libptls_hip.so (include/ptls_hip.h) for tests and bench.py.

Device memory and streams come from PyTorch (plumbing only); every byte of crypto runs in the HIP
kernels of libptls_hip.so.  There is no Python or CPU fallback: if the library or a gfx950 device
is missing, the constructors raise.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PRODUCT_LIB = os.path.join(HERE, "libptls_hip.so")
LIB_PATH = os.environ.get("PTLS_HIP_LIB") or PRODUCT_LIB
UINT64_MAX = (1 << 64) - 1

RECORD_DTYPE = np.dtype([("in_off", "<u8"), ("out_off", "<u8"), ("aad_off", "<u8"), ("seq", "<u8"),
                         ("len", "<u4"), ("aad_len", "<u4"), ("key", "<u4"), ("flags", "<u4")])
assert RECORD_DTYPE.itemsize == 48
SUPP_DTYPE = np.dtype([("sample_off", "<u8"), ("mask_off", "<u8"), ("hp_key", "<u4"), ("flags", "<u4")])
assert SUPP_DTYPE.itemsize == 24
SUPP_ENABLE = 1
TLS13_MESSAGE_DTYPE = np.dtype([("in_off", "<u8"), ("out_off", "<u8"), ("seq", "<u8"), ("len", "<u4"), ("key", "<u4"),
                                ("type", "<u4"), ("reserved", "<u4")])
assert TLS13_MESSAGE_DTYPE.itemsize == 40
TLS13_BAD_RECORD_MAC = (1 << 64) - 1
TLS13_NO_CONTENT_TYPE = (1 << 64) - 2
TLS13_DECODE_ERROR = -50
TLS13_SHORT_RECORD = -20  # a complete application-data record shorter than a tag (PTLS_ALERT_BAD_RECORD_MAC)
TRANSPORT_AUTO, TRANSPORT_COPY, TRANSPORT_MAPPED = 0, 1, 2


def record_tls13_type(t):
    return 1 | ((t & 0xFF) << 8)

# every function declared in include/ptls_hip.h: (restype, argtypes)
_vp, _sz, _i, _u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
SIGNATURES = {
    "ptls_hip_last_error": (ctypes.c_char_p, []),
    "ptls_hip_set_default_device": (_i, [_i]),
    "ptls_hip_engine_new": (_vp, [_i]),
    "ptls_hip_engine_free": (None, [_vp]),
    "ptls_hip_engine_device": (_i, [_vp]),
    "ptls_hip_engine_cu_count": (_i, [_vp]),
    "ptls_hip_keyset_new": (_vp, [_vp, _sz, _sz]),
    "ptls_hip_keyset_free": (None, [_vp]),
    "ptls_hip_keyset_size": (_sz, [_vp]),
    "ptls_hip_keyset_set": (_i, [_vp, _sz, _sz, _vp, _vp, _vp]),
    "ptls_hip_keyset_get_iv": (_i, [_vp, _sz, _vp]),
    "ptls_hip_keyset_set_secrets": (_i, [_vp, _sz, _sz, _vp, _sz, _vp]),
    "ptls_hip_keyset_update_secrets": (_i, [_vp, _sz, _sz, _vp, _sz, _vp]),
    "ptls_hip_keyset_set_iv": (_i, [_vp, _sz, _vp, _vp]),
    "ptls_hip_keyset_xor_iv": (_i, [_vp, _sz, _vp, _sz, _vp]),
    "ptls_hip_batch_new": (_vp, [_vp, _vp, _sz, _vp]),
    "ptls_hip_batch_free": (None, [_vp]),
    "ptls_hip_batch_count": (_sz, [_vp]),
    "ptls_hip_batch_set_lanes": (_i, [_vp, _i]),
    "ptls_hip_batch_lanes": (_i, [_vp]),
    "ptls_hip_batch_set_workgroup": (_i, [_vp, _i]),
    "ptls_hip_batch_workgroup": (_i, [_vp]),
    "ptls_hip_batch_set_max_workgroups": (_i, [_vp, _i]),
    "ptls_hip_batch_grid": (_i, [_vp]),
    "ptls_hip_batch_chunks": (_i, [_vp]),
    "ptls_hip_batch_set_clock": (_i, [_vp, _vp, _sz]),
    "ptls_hip_aesecb_init": (_i, [_vp, _i, _vp, _sz, _i]),
    "ptls_hip_aesecb_dispose": (None, [_vp]),
    "ptls_hip_aesecb_encrypt": (None, [_vp, _vp, _vp]),
    "ptls_hip_aesgcm_seal_batch": (_i, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "ptls_hip_aesgcm_open_batch": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "ptls_hip_aesgcm_seal_batch_supp": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "ptls_hip_aesecb_batch": (_i, [_vp, _vp, _vp, _sz, _vp, _vp, _vp]),
    "ptls_hip_fill_records": (_i, [_vp, _vp, _u64, _u64, _vp, _vp]),
    "ptls_hip_device_copy": (_i, [_vp, _vp, _vp, _sz, _vp]),
    "ptls_hip_tls13_wire_size": (_sz, [_sz]),
    "ptls_hip_tls13_frame": (_sz, [_vp, _sz, _vp, _sz]),
    "ptls_hip_tls13_seal_batch": (_i, [_vp, _vp, _vp, _vp, _vp]),
    "ptls_hip_tls13_parse": (_i, [_vp, _sz, _u64, ctypes.c_uint32, _u64, _u64, _vp, _sz, ctypes.POINTER(_sz),
                                  ctypes.POINTER(_sz)]),
    "ptls_hip_tls13_open_batch": (_i, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "ptls_hip_pipeline_new": (_vp, [_vp, _sz]),
    "ptls_hip_is_supported": (_i, []),
    "ptls_hip_aesgcm_new": (_vp, [_vp, _sz, _sz]),
    "ptls_hip_aesgcm_set_capacity": (_vp, [_vp, _sz]),
    "ptls_hip_aesgcm_free": (None, [_vp]),
    "ptls_hip_aesgcm_encrypt": (None, [_vp, _vp, _vp, _sz, _vp, _vp, _sz, _vp]),
    "ptls_hip_aesgcm_decrypt": (_i, [_vp, _vp, _vp, _sz, _vp, _vp, _sz, _vp]),
    "ptls_hip_pipeline_free": (None, [_vp]),
    "ptls_hip_pipeline_seal": (_i, [_vp, _vp, _vp, _sz, _vp, _vp, _vp]),
    "ptls_hip_pipeline_open": (_i, [_vp, _vp, _vp, _sz, _vp, _vp, _vp, _vp]),
    "ptls_hip_pipeline_tls13_seal": (_i, [_vp, _vp, _vp, _sz, _vp, _vp]),
    "ptls_hip_pipeline_seal_supp": (_i, [_vp, _vp, _vp, _vp, _vp, _sz, _vp, _vp, _vp, _vp]),
    "ptls_hip_pipeline_tls13_open": (_i, [_vp, _vp, _vp, _sz, _vp, _vp, _vp]),
    "ptls_hip_pipeline_set_transport": (_i, [_vp, _i]),
    "ptls_hip_pipeline_last_transport": (_i, [_vp]),
    "ptls_hip_host_register": (_i, [_vp, _sz]),
    "ptls_hip_host_unregister": (_i, [_vp]),
    "ptls_hip_partition_bytes": (_i, [_vp, _sz, _sz, _vp]),
    "ptls_hip_node_new": (_vp, [_vp, _sz, _sz, _sz, _sz]),
    "ptls_hip_node_free": (None, [_vp]),
    "ptls_hip_node_size": (_sz, [_vp]),
    "ptls_hip_node_keyset_set": (_i, [_vp, _sz, _sz, _vp, _vp]),
    "ptls_hip_node_set_transport": (_i, [_vp, _i]),
    "ptls_hip_node_seal": (_i, [_vp, _vp, _sz, _vp, _vp, _vp]),
    "ptls_hip_node_open": (_i, [_vp, _vp, _sz, _vp, _vp, _vp, _vp]),
    "ptls_hip_node_last_split": (_i, [_vp, _vp, _vp]),
    "ptls_hip_device_numa_node": (_i, [_i]),
    "ptls_hip_node_numa": (_i, [_vp, _vp]),
    "ptls_hip_node_host_alloc": (_vp, [_vp, _sz, _vp]),
    "ptls_hip_node_host_free": (None, [_vp, _sz]),
    "ptls_hip_host_page_nodes": (_sz, [_vp, _sz, _sz, _vp, _sz]),
}
DATA_SYMBOLS = ("ptls_hip_aes128ctr", "ptls_hip_aes128gcm", "ptls_hip_aes256ctr", "ptls_hip_aes256gcm",
                "ptls_hip_non_temporal_aes128gcm", "ptls_hip_non_temporal_aes256gcm")

_lib = None


class HipError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HipError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        product = os.path.realpath(LIB_PATH) == os.path.realpath(PRODUCT_LIB)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name, None)
            if f is None:
                if product:  # the product library must export every entry point of include/ptls_hip.h
                    raise HipError(f"{LIB_PATH} does not export {name}: stale or broken build")
                continue  # an older build loaded by an A/B tool (PTLS_HIP_LIB)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def last_error():
    return lib().ptls_hip_last_error().decode()


def _check(rc, what):
    if rc != 0:
        raise HipError(f"{what}: {last_error()} (rc={rc})")


def _ptr(x):
    """device/host pointer of a torch tensor, numpy array, int or None"""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    raise TypeError(type(x))


def _stream(stream):
    if stream is None:
        try:
            import torch
            return torch.cuda.current_stream().cuda_stream
        except Exception:  # noqa: BLE001
            return None
    return stream if isinstance(stream, int) else getattr(stream, "cuda_stream", stream)


class Engine:
    def __init__(self, device=0):
        self.ptr = lib().ptls_hip_engine_new(device)
        if not self.ptr:
            raise HipError(f"ptls_hip_engine_new({device}): {last_error()}")
        self.device = device

    @property
    def cu_count(self):
        return lib().ptls_hip_engine_cu_count(self.ptr)

    def aesecb(self, hp_keyset, supp, src, mask, stream=None):
        """mask[mask_off] = AES-ECB(hp key, src[sample_off:+16]) for every enabled device descriptor"""
        n = supp.numel() // SUPP_DTYPE.itemsize if hasattr(supp, "numel") else len(supp)
        _check(lib().ptls_hip_aesecb_batch(self.ptr, hp_keyset.ptr, _ptr(supp), n, _ptr(src), _ptr(mask), _stream(stream)),
               "aesecb_batch")

    def copy(self, dst, src, nbytes, stream=None):
        """ptls_hip_device_copy: the 16-byte-per-lane streaming copy (bench.py's achievable-HBM reference)"""
        _check(lib().ptls_hip_device_copy(self.ptr, _ptr(dst), _ptr(src), nbytes, _stream(stream)), "device_copy")

    def close(self):
        if self.ptr:
            lib().ptls_hip_engine_free(self.ptr)
            self.ptr = None


class KeySet:
    def __init__(self, engine, key_size, nslots):
        self.engine, self.key_size, self.nslots = engine, key_size, nslots
        self.ptr = lib().ptls_hip_keyset_new(engine.ptr, key_size, nslots)
        if not self.ptr:
            raise HipError(f"ptls_hip_keyset_new: {last_error()}")

    def set(self, first, keys, ivs, stream=None):
        """ivs=None: zero static IVs (header-protection keys)"""
        keys = bytes(keys)
        count = len(keys) // self.key_size
        assert len(keys) == count * self.key_size
        if ivs is not None:
            ivs = bytes(ivs)
            assert len(ivs) == count * 12
        _check(lib().ptls_hip_keyset_set(self.ptr, first, count, keys, ivs, _stream(stream)), "keyset_set")

    def set_secrets(self, first, secrets, hash_size, stream=None):
        """slots [first, first + n) keyed from n TLS 1.3 traffic secrets (HKDF-Expand-Label "key"/"iv" on the GPU)"""
        secrets = bytes(secrets)
        n = len(secrets) // hash_size
        _check(lib().ptls_hip_keyset_set_secrets(self.ptr, first, n, secrets, hash_size, _stream(stream)), "keyset_set_secrets")

    def update_secrets(self, first, secrets, hash_size, stream=None):
        """TLS 1.3 key update of n connections; returns the next secrets"""
        buf = ctypes.create_string_buffer(bytes(secrets), len(secrets))
        n = len(secrets) // hash_size
        _check(lib().ptls_hip_keyset_update_secrets(self.ptr, first, n, buf, hash_size, _stream(stream)),
               "keyset_update_secrets")
        return buf.raw

    def get_iv(self, slot):
        buf = ctypes.create_string_buffer(12)
        _check(lib().ptls_hip_keyset_get_iv(self.ptr, slot, buf), "keyset_get_iv")
        return buf.raw

    def set_iv(self, slot, iv, stream=None):
        _check(lib().ptls_hip_keyset_set_iv(self.ptr, slot, bytes(iv), _stream(stream)), "keyset_set_iv")

    def xor_iv(self, slot, data, stream=None):
        _check(lib().ptls_hip_keyset_xor_iv(self.ptr, slot, bytes(data), len(data), _stream(stream)), "keyset_xor_iv")

    def close(self):
        if self.ptr:
            lib().ptls_hip_keyset_free(self.ptr)
            self.ptr = None


class Batch:
    def __init__(self, engine, recs, stream=None):
        recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
        self.engine, self.recs = engine, recs
        self.ptr = lib().ptls_hip_batch_new(engine.ptr, recs.ctypes.data, len(recs), _stream(stream))
        if not self.ptr:
            raise HipError(f"ptls_hip_batch_new: {last_error()}")

    def __len__(self):
        return len(self.recs)

    @property
    def lanes(self):
        return lib().ptls_hip_batch_lanes(self.ptr)

    def set_lanes(self, lanes):
        _check(lib().ptls_hip_batch_set_lanes(self.ptr, lanes), "batch_set_lanes")

    @property
    def workgroup(self):
        return lib().ptls_hip_batch_workgroup(self.ptr)

    def set_workgroup(self, threads):
        _check(lib().ptls_hip_batch_set_workgroup(self.ptr, threads), "batch_set_workgroup")

    def set_max_workgroups(self, n):
        """cap the launch grid at n workgroups (0 = one per CU); chunks are then planned for n CUs"""
        _check(lib().ptls_hip_batch_set_max_workgroups(self.ptr, n), "batch_set_max_workgroups")

    @property
    def chunks(self):
        """chunks of the launch plan (key-slot runs of at most 32 wave tasks)"""
        return lib().ptls_hip_batch_chunks(self.ptr)

    @property
    def grid(self):
        """workgroups of one launch"""
        return lib().ptls_hip_batch_grid(self.ptr)

    def set_clock(self, buf):
        """diagnostic clock stamps of the following launches into `buf` (device tensor of >= 32 bytes per workgroup;
        None = off): per workgroup {cycles0, ticks0, cycles1, ticks1}, see clock_of()"""
        nbytes = 0 if buf is None else buf.numel() * buf.element_size()
        _check(lib().ptls_hip_batch_set_clock(self.ptr, _ptr(buf), nbytes), "batch_set_clock")

    def seal(self, keyset, inp, aad, out, stream=None):
        _check(lib().ptls_hip_aesgcm_seal_batch(self.ptr, keyset.ptr, _ptr(inp), _ptr(aad), _ptr(out), _stream(stream)),
               "seal_batch")

    def open(self, keyset, inp, aad, out, result, stream=None):
        _check(lib().ptls_hip_aesgcm_open_batch(self.ptr, keyset.ptr, _ptr(inp), _ptr(aad), _ptr(out), _ptr(result),
                                                _stream(stream)), "open_batch")

    def seal_supp(self, keyset, hp_keyset, supp, inp, aad, out, mask, stream=None):
        """seal + QUIC header-protection masks in one launch; supp: device array of SUPP_DTYPE, one per record"""
        _check(lib().ptls_hip_aesgcm_seal_batch_supp(self.ptr, keyset.ptr, hp_keyset.ptr, _ptr(supp), _ptr(inp), _ptr(aad),
                                                     _ptr(out), _ptr(mask), _stream(stream)), "seal_batch_supp")

    def tls13_seal(self, keyset, inp, out, stream=None):
        """records from tls13_frame(): writes headers into `out`, then seals with them as AAD"""
        _check(lib().ptls_hip_tls13_seal_batch(self.ptr, keyset.ptr, _ptr(inp), _ptr(out), _stream(stream)), "tls13_seal_batch")

    def tls13_open(self, keyset, inp, out, result, stream=None):
        """records from tls13_parse(): result = content length | type << 56, or TLS13_BAD_RECORD_MAC / NO_CONTENT_TYPE"""
        _check(lib().ptls_hip_tls13_open_batch(self.ptr, keyset.ptr, _ptr(inp), _ptr(out), _ptr(result), _stream(stream)),
               "tls13_open_batch")

    def fill(self, buf, seed, index_base=0, index=None, stream=None):
        """index: optional device tensor (int64/uint64) of per-descriptor generator indices"""
        _check(lib().ptls_hip_fill_records(self.ptr, _ptr(buf), seed, index_base, _ptr(index), _stream(stream)),
               "fill_records")

    def close(self):
        if self.ptr:
            lib().ptls_hip_batch_free(self.ptr)
            self.ptr = None


def partition_bytes(recs, parts):
    """ptls_hip_partition_bytes: record ranges of about equal payload bytes (host-only, no device needed)"""
    recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
    b = np.zeros(parts + 1, dtype=np.uint64)
    _check(lib().ptls_hip_partition_bytes(recs.ctypes.data, len(recs), parts, b.ctypes.data), "partition_bytes")
    return [int(x) for x in b]


class Node:
    """one batch over several devices (ptls_hip_node_*): byte-balanced contiguous ranges, one host thread + pipeline per
    device; buffers are host memory (pinned for the zero-copy transport)"""

    def __init__(self, devices, key_size, nslots, slice_bytes=64 << 20, transport=TRANSPORT_AUTO):
        arr = (ctypes.c_int * len(devices))(*devices)
        self.ndev, self.key_size = len(devices), key_size
        self.ptr = lib().ptls_hip_node_new(arr, len(devices), key_size, nslots, slice_bytes)
        if not self.ptr:
            raise HipError(f"ptls_hip_node_new: {last_error()}")
        _check(lib().ptls_hip_node_set_transport(self.ptr, transport), "node_set_transport")

    def set_keys(self, first, keys, ivs):
        """the same keys into every device's keyset: slots [first, first + len(keys) / key_size)"""
        keys = bytes(keys)
        ivs = None if ivs is None else bytes(ivs)
        n = len(keys) // self.key_size
        _check(lib().ptls_hip_node_keyset_set(self.ptr, first, n, keys, ivs), "node_keyset_set")

    def seal(self, recs, h_in, h_aad, h_out):
        recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
        _check(lib().ptls_hip_node_seal(self.ptr, recs.ctypes.data, len(recs), _ptr(h_in), _ptr(h_aad), _ptr(h_out)), "node_seal")

    def open(self, recs, h_in, h_aad, h_out, h_result):
        recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
        _check(lib().ptls_hip_node_open(self.ptr, recs.ctypes.data, len(recs), _ptr(h_in), _ptr(h_aad), _ptr(h_out),
                                        _ptr(h_result)), "node_open")

    def last_split(self):
        """(per-device seconds, record bounds) of the last call"""
        sec = np.zeros(self.ndev, dtype=np.float64)
        b = np.zeros(self.ndev + 1, dtype=np.uint64)
        _check(lib().ptls_hip_node_last_split(self.ptr, sec.ctypes.data, b.ctypes.data), "node_last_split")
        return sec.tolist(), [int(x) for x in b]

    def numa_nodes(self):
        """each device's NUMA node (-1: unknown)"""
        out = np.zeros(self.ndev, dtype=np.int32)
        _check(lib().ptls_hip_node_numa(self.ptr, out.ctypes.data), "node_numa")
        return [int(x) for x in out]

    def host_alloc(self, nbytes, splits):
        """a uint8 numpy array over `nbytes` of host memory whose byte range [splits[d], splits[d + 1]) lives on device d's
        NUMA node, registered with every device (ptls_hip_node_host_alloc); free it with host_free"""
        sp = np.ascontiguousarray(splits, dtype=np.uint64)
        p = lib().ptls_hip_node_host_alloc(self.ptr, nbytes, sp.ctypes.data)
        if not p:
            raise HipError(f"ptls_hip_node_host_alloc: {last_error()}")
        return np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))

    @staticmethod
    def host_free(arr):
        lib().ptls_hip_node_host_free(arr.ctypes.data, arr.nbytes)

    def close(self):
        if self.ptr:
            lib().ptls_hip_node_free(self.ptr)
            self.ptr = None


def page_nodes(arr, stride=1, cap=1 << 16):
    """the NUMA node of every stride-th page of a host array (move_pages)"""
    out = np.zeros(cap, dtype=np.int32)
    n = lib().ptls_hip_host_page_nodes(arr.ctypes.data, arr.nbytes, stride, out.ctypes.data, cap)
    return out[:n]


def clock_of(stamps, grid):
    """the clock one launch ran at, from its stamps (Batch.set_clock; array of >= 4 * grid uint64): per workgroup
    delta(shader cycles) / delta(100 MHz ticks) x 100 MHz.  Returns (median GHz over workgroups, min, max, the launch's
    span in ms from the first start to the last end on the 100 MHz counter)"""
    d = clock_detail(stamps, grid)
    return d["ghz_median"], d["ghz_min"], d["ghz_max"], d["span_ms"]


def clock_detail(stamps, grid):
    """clock_of plus how the launch ended across workgroups: every workgroup's start and end on the
    100 MHz counter and its XCD (HW_REG_XCC_ID, in the top byte of the start stamp).
      finish_spread = (last end - median end) / span: the share of the launch that only its slowest workgroups ran;
      per_xcd = median GHz and median end (ms after the first start) of the workgroups of each XCD"""
    u = np.asarray(stamps, dtype=np.uint64).reshape(-1, 4)[:grid]
    xcc = (u[:, 1] >> np.uint64(56)).astype(np.int64)
    a = u.astype(np.float64)
    a[:, 1] = (u[:, 1] & np.uint64((1 << 56) - 1)).astype(np.float64)
    dt, dr = a[:, 2] - a[:, 0], a[:, 3] - a[:, 1]
    ok = dr > 0
    ghz = np.where(ok, dt / np.where(ok, dr, 1) * 0.1, np.nan)
    t0 = a[:, 1].min()
    ends = (a[:, 3] - t0) / 1e5  # ms after the first start
    starts = (a[:, 1] - t0) / 1e5
    span_ms = float(ends.max())
    med_end = float(np.median(ends))
    per_xcd = {}
    for x in sorted(set(xcc.tolist())):
        m = xcc == x
        per_xcd[int(x)] = {"workgroups": int(m.sum()), "ghz_median": round(float(np.nanmedian(ghz[m])), 3),
                           "end_ms_median": round(float(np.median(ends[m])), 4), "end_ms_max": round(float(ends[m].max()), 4)}
    g = ghz[ok]
    return {"ghz_median": float(np.median(g)), "ghz_min": float(g.min()), "ghz_max": float(g.max()), "span_ms": span_ms,
            "end_ms_median": med_end, "end_ms_min": float(ends.min()), "start_ms_max": float(starts.max()),
            "finish_spread": (span_ms - med_end) / span_ms if span_ms > 0 else 0.0,
            "finish_spread_min_to_max": (span_ms - float(ends.min())) / span_ms if span_ms > 0 else 0.0,
            "per_xcd": per_xcd}


def is_supported():
    """True when a gfx950 device is visible (ptls_hip_is_supported, ~ ptls_fusion_is_supported_by_cpu)"""
    return bool(lib().ptls_hip_is_supported())


class AesGcm:
    """fusion-style low-level single-record context (ptls_hip_aesgcm_*, ~ ptls_fusion_aesgcm_*,
    include/picotls/fusion.h:56-96); `nonce` is the 12-byte GCM nonce fusion passes as its counter block"""

    def __init__(self, key, capacity=0):
        self.ptr = lib().ptls_hip_aesgcm_new(key, len(key), capacity)
        if not self.ptr:
            raise HipError(f"ptls_hip_aesgcm_new: {last_error()}")

    def set_capacity(self, capacity):
        self.ptr = lib().ptls_hip_aesgcm_set_capacity(self.ptr, capacity)

    class Supp(ctypes.Structure):  # ptls_aead_supplementary_encryption_t, include/picotls.h:421-436
        _fields_ = [("ctx", ctypes.c_void_p), ("input", ctypes.c_void_p), ("output", ctypes.c_uint8 * 16)]

    def encrypt(self, data, nonce, aad, supp_cipher=None, sample_off=0):
        """ciphertext || tag; with supp_cipher (a ptls_cipher_context_t address) also the supplementary
        block AES-ECB(output[sample_off:sample_off+16]): returns (output, block)"""
        out = ctypes.create_string_buffer(len(data) + 16)
        supp = None
        if supp_cipher is not None:
            supp = self.Supp(supp_cipher, ctypes.addressof(out) + sample_off)
        lib().ptls_hip_aesgcm_encrypt(self.ptr, out, data, len(data), nonce, aad, len(aad),
                                      None if supp is None else ctypes.addressof(supp))
        return out.raw if supp is None else (out.raw, bytes(supp.output))

    def decrypt(self, data, nonce, aad, tag):
        """(ok, plaintext): the plaintext is written whether or not the tag matches, as fusion's"""
        out = ctypes.create_string_buffer(max(len(data), 1))
        ok = lib().ptls_hip_aesgcm_decrypt(self.ptr, out, data, len(data), nonce, aad, len(aad), tag)
        return bool(ok), out.raw[:len(data)]

    def close(self):
        if self.ptr:
            lib().ptls_hip_aesgcm_free(self.ptr)
            self.ptr = None


class AesEcb:
    """fusion's one-block ECB API (ptls_hip_aesecb_*, ~ ptls_fusion_aesecb_*, include/picotls/fusion.h:52-54)"""

    class Ctx(ctypes.Structure):  # ptls_hip_aesecb_context_t
        _fields_ = [("state", ctypes.c_void_p), ("rounds", ctypes.c_uint)]

    def __init__(self, key, is_enc=1):
        self.ctx = self.Ctx()
        _check(lib().ptls_hip_aesecb_init(ctypes.addressof(self.ctx), is_enc, bytes(key), len(key), 0), "aesecb_init")

    @property
    def rounds(self):
        return self.ctx.rounds

    def encrypt(self, block):
        assert len(block) == 16
        out = ctypes.create_string_buffer(16)
        lib().ptls_hip_aesecb_encrypt(ctypes.addressof(self.ctx), out, bytes(block))
        return out.raw

    def close(self):
        if self.ctx.state:
            lib().ptls_hip_aesecb_dispose(ctypes.addressof(self.ctx))


class Pipeline:
    """host-resident seal/open: pinned H2D -> kernel -> D2H overlapped over three streams"""

    def __init__(self, engine, slice_bytes=64 << 20, transport=None):
        self.engine = engine
        self.ptr = lib().ptls_hip_pipeline_new(engine.ptr, slice_bytes)
        if not self.ptr:
            raise HipError(f"ptls_hip_pipeline_new: {last_error()}")
        if transport is not None:
            self.set_transport(transport)

    def set_transport(self, transport):
        """TRANSPORT_AUTO / TRANSPORT_COPY (copy engines + device staging) / TRANSPORT_MAPPED (kernels on the pinned host buffers)"""
        _check(lib().ptls_hip_pipeline_set_transport(self.ptr, transport), "pipeline_set_transport")

    @property
    def last_transport(self):
        return lib().ptls_hip_pipeline_last_transport(self.ptr)

    def seal(self, keyset, recs, h_in, h_aad, h_out):
        recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
        _check(lib().ptls_hip_pipeline_seal(self.ptr, keyset.ptr, recs.ctypes.data, len(recs), _ptr(h_in), _ptr(h_aad),
                                            _ptr(h_out)), "pipeline_seal")

    def open(self, keyset, recs, h_in, h_aad, h_out, h_result):
        recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
        _check(lib().ptls_hip_pipeline_open(self.ptr, keyset.ptr, recs.ctypes.data, len(recs), _ptr(h_in), _ptr(h_aad),
                                            _ptr(h_out), _ptr(h_result)), "pipeline_open")

    def seal_supp(self, keyset, hp_keyset, recs, supp, h_in, h_aad, h_out, h_mask):
        """seal + QUIC header-protection masks; supp = host numpy array (SUPP_DTYPE) indexed like recs"""
        recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
        supp = np.ascontiguousarray(supp, dtype=SUPP_DTYPE)
        _check(lib().ptls_hip_pipeline_seal_supp(self.ptr, keyset.ptr, hp_keyset.ptr, recs.ctypes.data, supp.ctypes.data,
                                                 len(recs), _ptr(h_in), _ptr(h_aad), _ptr(h_out), _ptr(h_mask)),
               "pipeline_seal_supp")

    def tls13_seal(self, keyset, recs, h_in, h_wire):
        """recs from tls13_frame: messages in h_in -> header + ciphertext + tag of every record in h_wire"""
        recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
        _check(lib().ptls_hip_pipeline_tls13_seal(self.ptr, keyset.ptr, recs.ctypes.data, len(recs), _ptr(h_in), _ptr(h_wire)),
               "pipeline_tls13_seal")

    def tls13_open(self, keyset, recs, h_wire, h_out, h_result):
        """recs from tls13_parse: received stream h_wire -> inner content in h_out, length | type << 56 in h_result"""
        recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
        _check(lib().ptls_hip_pipeline_tls13_open(self.ptr, keyset.ptr, recs.ctypes.data, len(recs), _ptr(h_wire), _ptr(h_out),
                                                  _ptr(h_result)), "pipeline_tls13_open")

    def close(self):
        if self.ptr:
            lib().ptls_hip_pipeline_free(self.ptr)
            self.ptr = None


def tls13_frame(msgs):
    """messages (TLS13_MESSAGE_DTYPE) -> record descriptors, picotls's 16384-byte chunking"""
    msgs = np.ascontiguousarray(msgs, dtype=TLS13_MESSAGE_DTYPE)
    n = lib().ptls_hip_tls13_frame(msgs.ctypes.data, len(msgs), None, 0)
    recs = np.zeros(n, dtype=RECORD_DTYPE)
    assert lib().ptls_hip_tls13_frame(msgs.ctypes.data, len(msgs), recs.ctypes.data, n) == n
    return recs


def tls13_parse(wire, wire_off=0, key=0, seq=0, out_base=0, cap=1 << 20, with_rc=False):
    """(recs, consumed) for the complete application-data records at the start of `wire` (bytes); a non-zero return
    raises HipError, or with_rc=True gives (rc, recs, consumed) (the records before the error are kept)"""
    recs = np.zeros(max(cap, 1), dtype=RECORD_DTYPE)
    nrecs, consumed = ctypes.c_size_t(), ctypes.c_size_t()
    rc = lib().ptls_hip_tls13_parse(bytes(wire), len(wire), wire_off, key, seq, out_base, recs.ctypes.data, cap,
                                    ctypes.byref(nrecs), ctypes.byref(consumed))
    if with_rc:
        return rc, recs[: nrecs.value].copy(), consumed.value
    if rc != 0:
        raise HipError(f"tls13_parse: {last_error()} (rc={rc})")
    return recs[: nrecs.value].copy(), consumed.value


def layout_records(lens, aad_lens, keys, seqs, align=16, tag_in_input=False):
    """Pack records into in / out / aad buffers with `align`-byte aligned offsets.

    Returns (recs, in_bytes, out_bytes, aad_bytes).  in holds L (+16 if tag_in_input) per record,
    out holds L + 16 (seal output: ct || tag)."""
    lens = np.asarray(lens, dtype=np.uint64)
    aad_lens = np.asarray(aad_lens, dtype=np.uint64)
    n = len(lens)
    a = np.uint64(align)

    def offsets(sizes):
        padded = (sizes + a - np.uint64(1)) // a * a
        off = np.zeros(n, dtype=np.uint64)
        if n > 1:
            np.cumsum(padded[:-1], out=off[1:])
        total = int(off[-1] + padded[-1]) if n else 0
        return off, total

    recs = np.zeros(n, dtype=RECORD_DTYPE)
    recs["in_off"], in_total = offsets(lens + (np.uint64(16) if tag_in_input else np.uint64(0)))
    recs["out_off"], out_total = offsets(lens + np.uint64(16))
    recs["aad_off"], aad_total = offsets(aad_lens)
    recs["len"] = lens
    recs["aad_len"] = aad_lens
    recs["key"] = keys
    recs["seq"] = seqs
    return recs, in_total, out_total, max(aad_total, 16)
