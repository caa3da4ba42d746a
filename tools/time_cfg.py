#!/usr/bin/env python3
"""Timing-only probe (no parity checks) over one of bench.py's workloads: median seal and open kernel
times of each library given on the command line.  For ablation builds whose output is wrong."""
import argparse, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hsig-picotls_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--config", default="c4")
ap.add_argument("--lanes", type=int, default=0)
ap.add_argument("--records", type=int, default=0, help="override the config's record count")
ap.add_argument("--key-len", type=int, default=0, help="override the key size (16 / 32)")
ap.add_argument("--fixed-len", type=int, default=0, help="every record this many bytes (instead of the config's lengths)")
ap.add_argument("--keys", type=int, default=0, help="override the number of keys")
ap.add_argument("--wg", type=int, default=0, help="workgroup size (512 / 768; 0 = the planner's)")
ap.add_argument("--clock", action="store_true", help="one more seal + open with the kernels' clock stamps (builds that have them)")
ap.add_argument("--reps", type=int, default=6, help="timed repetitions (the first is dropped)")
ap.add_argument("--zeros", action="store_true", help="all-zero plaintext (default: bench.py's splitmix64 records; zero data "
                "runs at a higher clock, MI355X_MICROARCH.md DVFS)")
args = ap.parse_args()
import torch
import bench
cfg = dict(bench.CONFIGS[args.config])
if args.records:
    cfg["n"] = args.records
if args.key_len:
    cfg["key_len"] = args.key_len
if args.fixed_len:
    cfg["L"] = args.fixed_len
if args.keys:
    cfg["keys"] = args.keys
for lib in args.libs:
    os.environ["PTLS_HIP_LIB"] = lib
    import ptls_hip
    ptls_hip.LIB_PATH = lib
    ptls_hip._lib = None
    eng = ptls_hip.Engine(0)
    idx, recs, in_total, out_total, lens = bench.make_workload(cfg, 0)
    keys, ivs = bench.make_keys(cfg)
    ks = ptls_hip.KeySet(eng, cfg["key_len"], cfg["keys"])
    ks.set(0, keys, ivs)
    sb = ptls_hip.Batch(eng, recs)
    if args.lanes:
        sb.set_lanes(args.lanes)
    if args.wg:
        sb.set_workgroup(args.wg)
    ro = recs.copy()
    ro["in_off"], ro["out_off"] = recs["out_off"], recs["in_off"]
    ob = ptls_hip.Batch(eng, ro)
    ob.set_lanes(sb.lanes)
    if args.wg:
        ob.set_workgroup(args.wg)
    d_pt = torch.zeros(in_total + 64, dtype=torch.uint8, device="cuda")
    if not args.zeros:
        d_idx = torch.from_numpy(idx.astype(np.int64)).cuda()
        sb.fill(d_pt, bench.SEED_DATA, index=d_idx)
        torch.cuda.synchronize()
        del d_idx
    d_ct = torch.zeros(out_total + 64, dtype=torch.uint8, device="cuda")
    d_out = torch.empty(in_total + 64, dtype=torch.uint8, device="cuda")
    d_aad = torch.zeros(len(recs) * 16, dtype=torch.uint8, device="cuda")
    d_res = torch.zeros(len(recs), dtype=torch.int64, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ts = []
    for i in range(args.reps):
        ev[0].record(); sb.seal(ks, d_pt, d_aad, d_ct); ev[1].record(); ob.open(ks, d_ct, d_aad, d_out, d_res); ev[2].record()
        torch.cuda.synchronize()
        if i:
            ts.append((ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])))
    s, o = np.median(np.array(ts), axis=0)
    gib = float(lens.sum()) / 2 ** 30
    clk = ""
    if args.clock and hasattr(ptls_hip.lib(), "ptls_hip_batch_set_clock"):
        cs = torch.zeros(4 * sb.grid, dtype=torch.int64, device="cuda")
        co = torch.zeros(4 * ob.grid, dtype=torch.int64, device="cuda")
        sb.set_clock(cs); ob.set_clock(co)
        ev[0].record(); sb.seal(ks, d_pt, d_aad, d_ct); ev[1].record(); ob.open(ks, d_ct, d_aad, d_out, d_res); ev[2].record()
        torch.cuda.synchronize()
        sc = ptls_hip.clock_of(cs.cpu().numpy().view(np.uint64), sb.grid)
        oc = ptls_hip.clock_of(co.cpu().numpy().view(np.uint64), ob.grid)
        sd = ptls_hip.clock_detail(cs.cpu().numpy().view(np.uint64), sb.grid)
        xc = " ".join(f"x{x}:{v['ghz_median']:.2f}/{v['end_ms_median']:.2f}/{v['end_ms_max']:.2f}" for x, v in sd["per_xcd"].items())
        clk = (f"  clock seal {sc[0]:.3f} GHz (wg {sc[1]:.3f}-{sc[2]:.3f}, span {sc[3]:.3f} ms, event {ev[0].elapsed_time(ev[1]):.3f} ms)"
               f" open {oc[0]:.3f} GHz  finish spread {sd['finish_spread']:.4f} (first end {sd['end_ms_min']:.3f}, median "
               f"{sd['end_ms_median']:.3f}, last start {sd['start_ms_max']:.3f} ms)  xcd ghz/end med/end max: {xc}")
        sb.set_clock(None); ob.set_clock(None)
    print(f"{os.path.basename(os.path.dirname(os.path.dirname(lib))) or '.'}/{os.path.basename(lib)} {args.config} lanes={sb.lanes} "
          f"wg={sb.workgroup}: seal {s:.3f} ms ({gib / s * 1e3:.1f} GiB/s)  open {o:.3f} ms ({gib / o * 1e3:.1f} GiB/s){clk}",
          flush=True)
    sb.close(); ob.close(); ks.close(); eng.close()
    del d_pt, d_ct, d_out
    torch.cuda.empty_cache()
