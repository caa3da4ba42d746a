#!/usr/bin/env python3
"""Seal + QUIC header protection in one launch (ptls_hip_aesgcm_seal_batch_supp) on configs[2]'s
shape (4M x 1350 B, AES-128, 13-B AAD), every record with a header-protection mask (sample = 16 bytes at ciphertext
offset 4, RFC 9001 §5.4.2 with a 1-byte packet number: pn_offset + 4), against plain seal of the same batch, for each
library given (PTLS_HIP_LIB A/B).  Timing only (parity: tests/test_gpu_parity.py).  One line per library."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hsig-picotls_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("lib")
ap.add_argument("--records", type=int, default=4 << 20)
args = ap.parse_args()
os.environ["PTLS_HIP_LIB"] = args.lib
import torch  # noqa: E402
import bench  # noqa: E402
import ptls_hip  # noqa: E402

cfg = dict(bench.CONFIGS["c3"], n=args.records)
eng = ptls_hip.Engine(0)
idx, recs, in_total, out_total, lens = bench.make_workload(cfg, 0)
keys, ivs = bench.make_keys(cfg)
ks = ptls_hip.KeySet(eng, 16, 1)
ks.set(0, keys, ivs)
hp = ptls_hip.KeySet(eng, 16, 1)
hp.set(0, bytes(range(16)), None)
n = len(recs)
supp = np.zeros(n, dtype=ptls_hip.SUPP_DTYPE)
supp["sample_off"] = recs["out_off"] + np.uint64(4)
supp["mask_off"] = np.arange(n, dtype=np.uint64) * np.uint64(16)
supp["flags"] = ptls_hip.SUPP_ENABLE
d_supp = torch.from_numpy(supp.view(np.uint8)).cuda()
b = ptls_hip.Batch(eng, recs)
d_pt = torch.zeros(in_total + 64, dtype=torch.uint8, device="cuda")
b.fill(d_pt, bench.SEED_DATA, index=torch.from_numpy(idx.astype(np.int64)).cuda())
d_ct = torch.zeros(out_total + 64, dtype=torch.uint8, device="cuda")
d_aad = torch.from_numpy(bench.build_aad(cfg, idx, lens)).cuda()
d_mask = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
ts = []
for i in range(8):
    ev[0].record()
    b.seal(ks, d_pt, d_aad, d_ct)
    ev[1].record()
    b.seal_supp(ks, hp, d_supp, d_pt, d_aad, d_ct, d_mask)
    ev[2].record()
    torch.cuda.synchronize()
    if i:
        ts.append((ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])))
s, p = np.median(np.array(ts), axis=0)
gib = float(lens.sum()) / 2 ** 30
print(f"{args.lib}: {n} x 1350 B seal {s:.3f} ms ({gib / s * 1e3:.1f} GiB/s)  seal+header protection {p:.3f} ms "
      f"({gib / p * 1e3:.1f} GiB/s)", flush=True)
