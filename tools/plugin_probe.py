#!/usr/bin/env python3
"""Per-call latency of the drop-in plugin path (ptls_aead_encrypt / decrypt through the reference's picotls, one
synchronous single-record launch per call) at several record sizes, for the library PTLS_HIP_LIB names, next to
the round trip of an empty torch kernel launch + synchronize on the same device.  Timing only; one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "hsig-picotls_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402  (torch's HIP runtime first)
import ctypes  # noqa: E402
import ptls_hip  # noqa: E402
from oracle_lib import ref_ptlsbench  # noqa: E402

assert torch.cuda.is_available()
x = torch.zeros(1, device="cuda")
for _ in range(100):
    x.add_(1)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(2000):
    x.add_(1)
    torch.cuda.synchronize()
noop_us = (time.perf_counter() - t0) / 2000 * 1e6
hip = ctypes.addressof(ctypes.c_char.in_dll(ptls_hip.lib(), "ptls_hip_aes128gcm"))
ref_ptlsbench(hip, 50, 1500)
out = {"lib": os.path.basename(ptls_hip.LIB_PATH), "torch_noop_launch_sync_us": round(noop_us, 2)}
for L in (0, 16, 1500, 16384):
    r = ref_ptlsbench(hip, 1000, L)
    out[f"L{L}"] = {"enc_us": r["enc_us_per_call"], "dec_us": r["dec_us_per_call"]}
ecb = ptls_hip.AesEcb(bytes(range(16)))
blk = bytes(16)
for _ in range(50):
    blk = ecb.encrypt(blk)
t0 = time.perf_counter()
for _ in range(1000):
    blk = ecb.encrypt(blk)
out["aesecb_encrypt_us"] = round((time.perf_counter() - t0) / 1000 * 1e6, 2)  # one block per call (CTR do_init, HP mask)
ecb.close()
print(json.dumps(out), flush=True)
