#!/usr/bin/env python3
"""Per-call latency of the drop-in plugin path at the shapes VERDICT r05 item 3 names: t/ptlsbench.c's bench_run_one
(:88-173) through the reference's picotls (oracle/_ref) on ptls_hip_aes128gcm and on lib/fusion.c's ptls_fusion_aes128gcm,
N calls of L = 0 / 1 500 / 16 384 bytes, wall-clock microseconds per call.  One JSON line.
Usage: python tools/plugin_calls.py [N]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "hsig-picotls_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402,F401  (the HIP runtime torch loads, before libptls_hip.so)
import ptls_hip  # noqa: E402
from oracle_lib import Ref, ref_ptlsbench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
hip = ctypes.addressof(ctypes.c_char.in_dll(ptls_hip.lib(), "ptls_hip_aes128gcm"))
fus = Ref().algo("ptls_fusion_aes128gcm")
ref_ptlsbench(hip, 50, 1500)  # warm-up: context creation, module load, the worker's first dispatch
out = {"lib": ptls_hip.LIB_PATH, "n": n}
for L in (0, 1500, 16384):
    h = ref_ptlsbench(hip, n, L)
    f = ref_ptlsbench(fus, n, L)
    out[f"L{L}"] = {"hip_enc_us": h["enc_us_per_call"], "hip_dec_us": h["dec_us_per_call"],
                    "fusion_enc_us": f["enc_us_per_call"], "fusion_dec_us": f["dec_us_per_call"]}
print(json.dumps(out), flush=True)
