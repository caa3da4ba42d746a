#!/usr/bin/env python3
"""Where a plugin call through the resident worker spends its time: the DIAGNOSTIC build
hsig-picotls_amd/diag/libptls_hip_wstamps.so (Makefile `diag`, sparse_kernel.hip WORKER_STAMPS) has the worker stamp the
100 MHz counter when it sees a request (after the poll), after the system-scope acquire, after the request's loads, after
the record and after the release fence; the engine times the call on the host.  The host's part (detection of the request
by the polls + the completion word's trip back + the host's own work) = call - (released - seen).  Median microseconds
over 300 calls per shape, fusion-style low-level context (ptls_hip_aesgcm_encrypt) and the one-block ECB.  One JSON line."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PTLS_HIP_LIB"] = os.path.join(ROOT, "hsig-picotls_amd", "diag", "libptls_hip_wstamps.so")
os.environ["PTLS_HIP_PLUGIN_WORKER"] = "1"
for p in (ROOT, os.path.join(ROOT, "hsig-picotls_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402,F401
import ptls_hip  # noqa: E402

L = ptls_hip.lib()
L.ptls_hip_diag_worker_stamps.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
st = np.zeros(15, dtype=np.uint64)
cu = ctypes.c_double()


def sample(call):
    rows = []
    for it in range(320):
        call()
        assert L.ptls_hip_diag_worker_stamps(st.ctypes.data, ctypes.byref(cu)) == 0
        if it >= 20:
            f = st.astype(np.float64)
            d = np.diff(f[:5]) / 100.0  # us
            ghz = (f[14] - f[6]) / ((f[3] - f[2]) * 10.0) if f[3] > f[2] else 2.4  # shader cycles / ns over the record
            ph = np.diff(f[6:15]) / ghz / 1e3 if f[7] else np.zeros(8)
            rows.append([cu.value, *d, *ph])
    a = np.median(np.array(rows), axis=0)
    gpu = float(a[1] + a[2] + a[3] + a[4])
    r = {"call_us": round(float(a[0]), 2), "acquire_inv": round(float(a[1]), 2), "request_loads": round(float(a[2]), 2),
         "record": round(float(a[3]), 2), "release": round(float(a[4]), 2), "host_and_link": round(float(a[0]) - gpu, 2)}
    names = ["ctr_const", "h64_table", "head_elems", "stretch", "tail_elems", "combine", "tag_store", "supp_to_end"]
    r["record_phases"] = {n: round(float(x), 2) for n, x in zip(names, a[5:13])}
    return r


out = {"lib": os.environ["PTLS_HIP_LIB"]}
for key_len in (16, 32):
    g = ptls_hip.AesGcm(bytes(range(key_len)), 1 << 15)
    for n in (0, 1500, 16384):
        pt = bytes((i * 7) & 0xFF for i in range(n))
        out[f"aes{key_len * 8}_L{n}"] = sample(lambda: g.encrypt(pt, bytes(12), b"\x17\x03\x03\x05\xdc"))
    g.close()
ecb = ptls_hip.AesEcb(bytes(range(16)))
out["ecb"] = sample(lambda: ecb.encrypt(bytes(16)))
ecb.close()
print(json.dumps(out), flush=True)
