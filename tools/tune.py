#!/usr/bin/env python3
"""Same-process tuning sweep: seal kernel time for every (lanes, workgroup) on each config's workload.
Timing only (parity is the tests' job); all variants share one process, box and clock state."""
import argparse, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "hsig-picotls_amd"))
import torch
import bench, ptls_hip
ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="c2,c3,c4")
ap.add_argument("--lanes", default="1,2,4,8")
ap.add_argument("--wg", default="512,768")
ap.add_argument("--reps", type=int, default=4)
ap.add_argument("--pack", type=int, default=0, help="re-lay records out at this byte alignment (1 = packed)")
args = ap.parse_args()
eng = ptls_hip.Engine(0)
for name in args.configs.split(","):
    cfg = bench.CONFIGS[name]
    idx, recs, in_total, out_total, lens = bench.make_workload(cfg, 0)
    if args.pack:
        aad_len = 5 if cfg["aad"] == "tls" else 13
        r2, in_total, out_total, _ = ptls_hip.layout_records(recs["len"], recs["aad_len"], recs["key"], recs["seq"], align=args.pack)
        r2["aad_off"] = recs["aad_off"]
        recs = r2
    n = len(recs); sumL = int(lens.sum())
    ks = ptls_hip.KeySet(eng, cfg["key_len"], cfg["keys"]); ks.set(0, *bench.make_keys(cfg))
    b = ptls_hip.Batch(eng, recs)
    auto = (b.lanes, b.workgroup)
    d_in = torch.zeros(in_total + 64, dtype=torch.uint8, device="cuda")
    d_out = torch.empty(out_total + 64, dtype=torch.uint8, device="cuda")
    d_aad = torch.from_numpy(bench.build_aad(cfg, idx, lens)).cuda()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    rows = []
    for lanes in [int(x) for x in args.lanes.split(",")]:
        for wg in [int(x) for x in args.wg.split(",")]:
            b.set_lanes(lanes); b.set_workgroup(wg)
            ts = []
            for i in range(args.reps + 1):
                ev[0].record(); b.seal(ks, d_in, d_aad, d_out); ev[1].record(); torch.cuda.synchronize()
                if i: ts.append(ev[0].elapsed_time(ev[1]))
            ms = float(np.median(ts))
            rows.append((ms, lanes, wg))
            print(f"{name} lanes={lanes} wg={wg}: {ms:.3f} ms  {sumL / ms / 1e6 / 1.073741824:.1f} GiB/s seal", flush=True)
    best = min(rows)
    print(f"{name}: auto={auto} best lanes={best[1]} wg={best[2]} {sumL / best[0] / 1e6 / 1.073741824:.1f} GiB/s", flush=True)
    b.close(); ks.close(); del d_in, d_out, d_aad; torch.cuda.empty_cache()
