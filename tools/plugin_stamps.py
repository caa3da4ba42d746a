#!/usr/bin/env python3
"""Where a plugin call's kernel spends its time: the DIAGNOSTIC build
hsig-picotls_amd/diag/libptls_hip_stamps.so (Makefile `diag`, sparse_kernel.hip STAMP_PHASES) stamps the shader clock at
the phase boundaries of the single-record launch; this drives records through the fusion-style low-level context
(ptls_hip_aesgcm_encrypt: the plugin's one-record path) and prints the median microseconds of each phase.  The stamps
drain LDS reads, so the build's run time is not quoted: read the shares.  One JSON line."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "hsig-picotls_amd", "diag", "libptls_hip_stamps.so")
os.environ["PTLS_HIP_LIB"] = LIB
for p in (ROOT, os.path.join(ROOT, "hsig-picotls_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402  (torch's HIP runtime first)
import ptls_hip  # noqa: E402

PHASES = ["aes_tables+barrier", "ctr_const", "h64_table", "head_elems", "stretch", "tail_elems", "valu_combine",
          "tag_store", "supp", "release_fence", "done_store"]
assert torch.cuda.is_available()
L = ptls_hip.lib()
L.ptls_hip_diag_plugin_stamps.argtypes = [ctypes.c_void_p]
st = np.zeros(16, dtype=np.uint64)
out = {"lib": LIB}
for key_len in (16, 32):
    g = ptls_hip.AesGcm(bytes(range(key_len)), 1 << 15)
    for n in (0, 1500, 16384):
        pt = bytes((i * 7) & 0xFF for i in range(n))
        rows = []
        for it in range(220):
            g.encrypt(pt, bytes(12), b"\x17\x03\x03\x05\xdc")
            assert L.ptls_hip_diag_plugin_stamps(st.ctypes.data) == 0
            if it >= 20:
                rows.append(st.astype(np.float64).copy())
        a = np.array(rows)
        ghz = (a[:, 11] - a[:, 0]) / (a[:, 15] - a[:, 14]) * 0.1
        d = np.diff(a[:, :12], axis=1) / ghz[:, None] / 1e3  # us
        out[f"aes{key_len * 8}_L{n}"] = {"clock_ghz": round(float(np.median(ghz)), 3),
                                         "kernel_us": round(float(np.median((a[:, 11] - a[:, 0]) / ghz / 1e3)), 2),
                                         **{p: round(float(np.median(d[:, i])), 2) for i, p in enumerate(PHASES)}}
    g.close()
print(json.dumps(out), flush=True)
