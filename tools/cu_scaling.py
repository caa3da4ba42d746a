#!/usr/bin/env python3
"""Per-CU seal rate of one bench config with the batch kernel's grid capped at N workgroups (one per CU):
if the chip ran at a fixed clock, an LDS-bound kernel would deliver the same GiB/s per CU at every N; a per-CU rate
that rises as N falls shows the clock rising as fewer CUs draw power.  Timing only."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hsig-picotls_amd"))
import torch  # noqa: E402  (torch's HIP runtime first)
assert torch.cuda.is_available()
import bench  # noqa: E402
import ptls_hip  # noqa: E402

GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--cus", default="32,64,128,192,256")
    ap.add_argument("--hold", type=float, default=0.0, help="also keep sealing this many seconds per N (for power sampling)")
    args = ap.parse_args()
    cfg = dict(bench.CONFIGS[args.config])
    eng = ptls_hip.Engine(0)
    idx, recs, in_total, out_total, lens = bench.make_workload(cfg, 0)
    keys, ivs = bench.make_keys(cfg)
    ks = ptls_hip.KeySet(eng, cfg["key_len"], cfg["keys"])
    ks.set(0, keys, ivs)
    b = ptls_hip.Batch(eng, recs)
    aad = torch.from_numpy(bench.build_aad(cfg, idx, lens)).cuda()
    d_in = torch.zeros(in_total + 64, dtype=torch.uint8, device="cuda")
    d_out = torch.zeros(out_total + 64, dtype=torch.uint8, device="cuda")
    b.fill(d_in, bench.SEED_DATA)
    sum_L = float(lens.sum())
    for n in [int(x) for x in args.cus.split(",")]:
        b.set_max_workgroups(n)
        ts = []
        for r in range(4):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            b.seal(ks, d_in, aad, d_out)
            e1.record()
            torch.cuda.synchronize()
            if r:
                ts.append(e0.elapsed_time(e1))
        ms = float(np.median(ts))
        g = sum_L / (ms * 1e-3) / GIB
        print(f"{args.config} workgroups={n}: seal {ms:.3f} ms  {g:.1f} GiB/s  {g / n:.3f} GiB/s per CU", flush=True)
        if args.hold:
            import time
            t0 = time.time()
            print(f"hold start {t0:.1f} workgroups={n}", flush=True)
            while time.time() - t0 < args.hold:
                for _ in range(20):
                    b.seal(ks, d_in, aad, d_out)
                torch.cuda.synchronize()
            print(f"hold end {time.time():.1f}", flush=True)
    b.close()
    ks.close()
    eng.close()


if __name__ == "__main__":
    main()
