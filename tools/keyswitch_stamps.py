#!/usr/bin/env python3
"""Where a batch launch's wave time goes (task phases added in round 5), from a DIAGNOSTIC build
(EXTRA=-DKS_STAMPS=1 tools/build_variant.sh ksstamps): every wave sums the shader cycles it spends waiting at the key
switch's first barrier (the other waves finishing the old key run's tasks), building the new key's GHASH tables, and
waiting at the second barrier, and inside its tasks: drawing the next task (and finding the chunk's end), setup
(descriptors, AAD elements, counter-mode constants), the branch-free stretch, the generic rest (partial, length and
leftover blocks), the combination + tag; against its total.  One seal launch of the config; prints shares over all
waves.  (The stamps themselves cost cycles: compare shares, not absolute times, with an unstamped build.)"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hsig-picotls_amd")]
ap = argparse.ArgumentParser()
ap.add_argument("lib")
ap.add_argument("--config", default="c4")
ap.add_argument("--lanes", type=int, default=0)
ap.add_argument("--records", type=int, default=0)
args = ap.parse_args()
os.environ["PTLS_HIP_LIB"] = args.lib
import torch  # noqa: E402

torch.zeros(1, device="cuda")
import bench  # noqa: E402
import ptls_hip  # noqa: E402

cfg = dict(bench.CONFIGS[args.config])
if args.records:
    cfg["n"] = args.records
eng = ptls_hip.Engine(0)
idx, recs, in_total, out_total, lens = bench.make_workload(cfg, 0)
keys, ivs = bench.make_keys(cfg)
ks = ptls_hip.KeySet(eng, cfg["key_len"], cfg["keys"])
ks.set(0, keys, ivs)
b = ptls_hip.Batch(eng, recs)
if args.lanes:
    b.set_lanes(args.lanes)
d_pt = torch.zeros(in_total + 64, dtype=torch.uint8, device="cuda")
d_ct = torch.zeros(out_total + 64, dtype=torch.uint8, device="cuda")
d_aad = torch.zeros(len(recs) * 16, dtype=torch.uint8, device="cuda")
NW = b.workgroup // 64
grid = b.grid
clk = torch.zeros(4 * grid + 16 * grid * NW, dtype=torch.int64, device="cuda")
for rep in range(3):
    b.set_clock(clk if rep == 2 else None)
    b.seal(ks, d_pt, d_aad, d_ct)
    torch.cuda.synchronize()
a = clk.cpu().numpy().view(np.uint64)[4 * grid:].reshape(grid, NW, 16).astype(np.float64)
tot = a[:, :, 0].sum()
b1, build, b2, nsw = (a[:, :, k].sum() for k in (1, 2, 3, 4))
print(f"{args.config} lanes={b.lanes} grid={grid} waves={grid * NW}: switches per wave {nsw / (grid * NW):.1f}; "
      f"share of wave cycles: barrier-1 wait {b1 / tot:.4f}, table build {build / tot:.4f}, barrier-2 wait {b2 / tot:.4f}, "
      f"tasks + dealing {(tot - b1 - build - b2) / tot:.4f}; cycles per switch per wave: barrier-1 {b1 / max(nsw, 1):.0f}, "
      f"build {build / max(nsw, 1):.0f}, barrier-2 {b2 / max(nsw, 1):.0f}")
ph = {name: a[:, :, k].sum() / tot for k, name in ((5, "draw"), (6, "setup"), (7, "stretch"), (8, "rest"), (9, "combine+tag"),
                                                   (10, "  rest: loads issued + wave max"), (11, "  rest: AES"),
                                                   (12, "  rest: finish (loads back, stores)"), (13, "  rest: GHASH"))}
print("task phases, share of wave cycles: " + ", ".join(f"{k} {v:.4f}" for k, v in ph.items()) +
      f"")
