#!/usr/bin/env python3
"""The plugin under a server's load, through the reference's own picotls (oracle/_ref):
  calls   t/ptlsbench.c's loop (1500-B records, encrypt + decrypt) on 1 / 2 / 4 / 8 / 16 threads at once, each thread with
          its own contexts (ref_ptlsbench_mt): calls per second for ptls_hip_aes128gcm and lib/fusion.c
  life    ptls_aead_new_direct / one seal / ptls_aead_free, 300 rounds (ref_aead_lifecycle): median and p90 microseconds
  beside  a 1 GiB batch seal (65 536 x 16 KiB, AES-128) timed alone and while 4 threads make plugin calls
  free    hipMalloc + hipFree of 1 MiB, and a 1-slot batch keyset new + free, while plugin calls keep the worker resident
One JSON object on stdout."""
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np
import torch

torch.zeros(1, device="cuda")  # torch's HIP runtime first (bench.py's order): initialised after the plugin's, it finds no GPU
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "hsig-picotls_amd"), ROOT]
import ptls_hip  # noqa: E402
from oracle_lib import REF_SO, Ref  # noqa: E402

c = ctypes
R = c.CDLL(REF_SO)
R.ref_ptlsbench_mt.restype = c.c_double
R.ref_ptlsbench_mt.argtypes = [c.c_void_p, c.c_int, c.c_size_t, c.c_size_t]
R.ref_aead_lifecycle.restype = c.c_int
R.ref_aead_lifecycle.argtypes = [c.c_void_p, c.c_size_t, c.c_size_t] + [c.POINTER(c.c_double)] * 3
hip_algo = c.addressof(c.c_char.in_dll(ptls_hip.lib(), "ptls_hip_aes128gcm"))
fus_algo = Ref().algo("ptls_fusion_aes128gcm")
out = {"workers": int(os.environ.get("PTLS_HIP_PLUGIN_WORKERS", "16")),
       "worker": os.environ.get("PTLS_HIP_PLUGIN_WORKER", "1")}


def stats(a):
    a = np.asarray(a)
    return {"median": round(float(np.median(a)), 2), "p90": round(float(np.percentile(a, 90)), 2),
            "max": round(float(a.max()), 2)}


# calls per second
R.ref_ptlsbench_mt(hip_algo, 1, 200, 1500)  # warm-up: module load, pools
calls = {}
for t in (1, 2, 4, 8, 16):
    h = R.ref_ptlsbench_mt(hip_algo, t, 3000, 1500)
    f = R.ref_ptlsbench_mt(fus_algo, t, 20000, 1500)
    calls[t] = {"hip_calls_per_s": round(h), "fusion_calls_per_s": round(f), "hip_us_per_call_per_thread": round(t / h * 1e6, 2)}
    print(f"threads {t}: hip {h:,.0f} calls/s, fusion {f:,.0f}", file=sys.stderr, flush=True)
out["calls_1500B"] = calls
out["hip_scaling_4_over_1"] = round(calls[4]["hip_calls_per_s"] / calls[1]["hip_calls_per_s"], 2)

# context lifecycle
n = 300
arrs = [(c.c_double * n)() for _ in range(3)]
assert R.ref_aead_lifecycle(hip_algo, n, 1500, *arrs) == 0
out["lifecycle_us"] = {k: stats(list(a)[10:]) for k, a in zip(("new", "seal", "free"), arrs)}
assert R.ref_aead_lifecycle(fus_algo, n, 1500, *arrs) == 0
out["lifecycle_us_fusion"] = {k: stats(list(a)[10:]) for k, a in zip(("new", "seal", "free"), arrs)}

# background plugin traffic for the next two measurements
stop = threading.Event()


def traffic():
    while not stop.is_set():
        R.ref_ptlsbench_mt(hip_algo, 4, 500, 1500)


eng = ptls_hip.Engine(0)
nrec, L = 65536, 16384
recs = np.zeros(nrec, dtype=ptls_hip.RECORD_DTYPE)
recs["in_off"] = np.arange(nrec, dtype=np.uint64) * L
recs["out_off"] = np.arange(nrec, dtype=np.uint64) * (L + 16)
recs["aad_off"] = 0
recs["seq"] = np.arange(nrec, dtype=np.uint64)
recs["len"] = L
recs["aad_len"] = 5
ks = ptls_hip.KeySet(eng, 16, 1)
ks.set(0, b"\x11" * 16, b"\x22" * 12)
b = ptls_hip.Batch(eng, recs)
d_pt = torch.zeros(nrec * L + 64, dtype=torch.uint8, device="cuda")
d_ct = torch.zeros(nrec * (L + 16) + 64, dtype=torch.uint8, device="cuda")
d_aad = torch.zeros(64, dtype=torch.uint8, device="cuda")
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]


def time_seal(reps=6):
    ts = []
    for _ in range(reps):
        ev[0].record()
        b.seal(ks, d_pt, d_aad, d_ct)
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    return round(float(np.median(ts[1:])), 3), round(float(max(ts[1:])), 3)


alone = time_seal()
th = threading.Thread(target=traffic)
th.start()
time.sleep(0.05)
beside = time_seal()
hip = c.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [c.POINTER(c.c_void_p), c.c_size_t]
hip.hipFree.argtypes = [c.c_void_p]
tf, tk = [], []
for _ in range(30):
    p = c.c_void_p()
    t0 = time.perf_counter()
    assert hip.hipMalloc(c.byref(p), 1 << 20) == 0
    assert hip.hipFree(p) == 0
    tf.append((time.perf_counter() - t0) * 1e6)
    t0 = time.perf_counter()
    k2 = ptls_hip.KeySet(eng, 16, 1)
    k2.close()
    tk.append((time.perf_counter() - t0) * 1e6)
    time.sleep(0.001)
stop.set()
th.join()
out["batch_1GiB_seal_ms"] = {"alone_median_max": alone, "beside_4_plugin_threads_median_max": beside}
out["with_worker_resident_us"] = {"hipMalloc_hipFree_1MiB": stats(tf), "batch_keyset_new_free": stats(tk)}
b.close()
ks.close()
eng.close()
print(json.dumps(out))
