#!/usr/bin/env python3
"""Timing-only probe (no parity checks): median seal kernel time of each library given on the command
line over the c2 workload (1M x 16 KiB unless --records).  For ablation builds whose output is wrong."""
import argparse, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--records", type=int, default=1 << 20)
ap.add_argument("--L", type=int, default=16384)
args = ap.parse_args()
import torch
res = {}
for lib in args.libs:
    os.environ["PTLS_HIP_LIB"] = lib
    for m in [m for m in sys.modules if m.startswith("ptls_hip")]:
        del sys.modules[m]
    sys.path.insert(0, os.path.join(ROOT, "hsig-picotls_amd"))
    import ptls_hip
    ptls_hip._lib = None
    n, L = args.records, args.L
    eng = ptls_hip.Engine(0)
    recs, it, ot, _ = ptls_hip.layout_records(np.full(n, L), np.full(n, 5), np.zeros(n), np.arange(n))
    recs["aad_off"] = np.arange(n, dtype=np.uint64) * 16
    ks = ptls_hip.KeySet(eng, 16, 1); ks.set(0, b"k" * 16, b"i" * 12)
    b = ptls_hip.Batch(eng, recs)
    d_in = torch.zeros(it, dtype=torch.uint8, device="cuda"); d_out = torch.empty(ot, dtype=torch.uint8, device="cuda")
    d_aad = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for i in range(6):
        ev[0].record(); b.seal(ks, d_in, d_aad, d_out); ev[1].record(); torch.cuda.synchronize()
        if i: ts.append(ev[0].elapsed_time(ev[1]))
    ms = float(np.median(ts))
    print(f"{os.path.basename(lib)}: seal {ms:.3f} ms  {n * L / ms / 1e6 / 1.073741824:.1f} GiB/s", flush=True)
    b.close(); ks.close(); eng.close()
    del d_in, d_out
