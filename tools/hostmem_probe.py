#!/usr/bin/env python3
"""Host-resident AES-GCM: copy engines (SDMA) against the batch kernel reading and writing pinned host memory
directly (zero-copy), VERDICT r1 item 6.

Measures, on 1 GiB of c2-shaped records (16 KiB, AES-128, one key):
  * SDMA: pinned H2D alone, D2H alone, both at once on two streams (the current pipeline's transport);
  * the seal kernel with its input and/or output in pinned host memory (device pointers of the mappings from
    hipHostGetDevicePointer), for host memory from hipHostMalloc (coherent / non-coherent) -- seal+open with
    both ends in host memory is the zero-copy end-to-end rate.
Prints one JSON line.  Timing only (the bytes are checked by the pipeline tests, not here)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hsig-picotls_amd"))

import torch  # noqa: E402  (torch's HIP runtime first)
assert torch.cuda.is_available()
import bench  # noqa: E402
import ptls_hip  # noqa: E402

GIB = float(1 << 30)
hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipHostFree.argtypes = [ctypes.c_void_p]
hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
FLAGS = {"coherent": 0x40000000, "noncoherent": 0x80000000}


def host_alloc(n, flags):
    p = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p), n, flags) == 0, "hipHostMalloc"
    d = ctypes.c_void_p()
    assert hip.hipHostGetDevicePointer(ctypes.byref(d), p, 0) == 0, "hipHostGetDevicePointer"
    ctypes.memset(p, 0, n)
    return p.value, d.value


def timed(f, reps=3):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--records", type=int, default=0)
    ap.add_argument("--lanes", default="0", help="comma-separated lanes-per-record values for the zero-copy runs (0 = planner)")
    ap.add_argument("--kinds", default="coherent,noncoherent")
    args = ap.parse_args()
    cfg = dict(bench.CONFIGS[args.config])
    cfg["n"] = args.records or max(1, int((1 << 30) / (cfg["L"] or 8224)))
    out = {"config": args.config, "records": cfg["n"], "record_bytes": cfg["L"]}
    eng = ptls_hip.Engine(0)
    idx, recs, in_total, out_total, lens = bench.make_workload(cfg, 0)
    sum_L = float(lens.sum())
    keys, ivs = bench.make_keys(cfg)
    ks = ptls_hip.KeySet(eng, cfg["key_len"], cfg["keys"])
    ks.set(0, keys, ivs)
    seal_b = ptls_hip.Batch(eng, recs)
    ro = recs.copy()
    ro["in_off"], ro["out_off"] = recs["out_off"], recs["in_off"]
    open_b = ptls_hip.Batch(eng, ro)
    open_b.set_lanes(seal_b.lanes)
    aad = torch.from_numpy(bench.build_aad(cfg, idx, lens)).cuda()
    res = torch.zeros(cfg["n"], dtype=torch.int64, device="cuda")
    d_in = torch.zeros(in_total + 64, dtype=torch.uint8, device="cuda")
    d_out = torch.zeros(out_total + 64, dtype=torch.uint8, device="cuda")
    seal_b.fill(d_in, bench.SEED_DATA)

    # SDMA transport
    h1 = torch.empty(in_total, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(in_total, dtype=torch.uint8).pin_memory()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def h2d():
        with torch.cuda.stream(s1):
            d_in[:in_total].copy_(h1, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            h2.copy_(d_out[:in_total], non_blocking=True)
    a, b, c = timed(h2d), timed(d2h), timed(lambda: (h2d(), d2h()))
    out["sdma"] = {"h2d_gbs": round(in_total / a / 1e9, 1), "d2h_gbs": round(in_total / b / 1e9, 1),
                   "both_aggregate_gbs": round(2 * in_total / c / 1e9, 1)}
    del h1, h2
    seal_b.fill(d_in, bench.SEED_DATA)

    out["device_seal_gibps"] = round(sum_L / timed(lambda: seal_b.seal(ks, d_in, aad, d_out)) / GIB, 1)
    runs = [(k, FLAGS[k], int(l)) for k in args.kinds.split(",") for l in args.lanes.split(",")]
    for kind, fl, lanes in runs:
        seal_b.set_lanes(lanes)
        open_b.set_lanes(seal_b.lanes)
        hin, hin_d = host_alloc(in_total + 64, fl)
        hout, hout_d = host_alloc(out_total + 64, fl)
        hpt, hpt_d = host_alloc(in_total + 64, fl)
        torch.cuda.synchronize()
        # the plaintext into host memory once (SDMA), so the zero-copy seal reads real records
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        assert hip.hipMemcpy(hin, d_in.data_ptr(), in_total, 2) == 0
        r = {}
        r["seal_host_in_gibps"] = round(sum_L / timed(lambda: seal_b.seal(ks, hin_d, aad, d_out)) / GIB, 2)
        r["seal_host_out_gibps"] = round(sum_L / timed(lambda: seal_b.seal(ks, d_in, aad, hout_d)) / GIB, 2)
        t_s = timed(lambda: seal_b.seal(ks, hin_d, aad, hout_d))
        t_o = timed(lambda: open_b.open(ks, hout_d, aad, hpt_d, res))
        r["seal_host_host_gibps"] = round(sum_L / t_s / GIB, 2)
        r["open_host_host_gibps"] = round(sum_L / t_o / GIB, 2)
        r["seal_open_host_host_gibps"] = round(2 * sum_L / (t_s + t_o) / GIB, 2)
        r["open_all_ok"] = bool((res == torch.from_numpy(lens.astype(np.int64)).cuda()).all())
        r["pcie_bytes_per_s_gbs"] = round((2 * sum_L + 16 * cfg["n"]) / t_s / 1e9, 1)
        r["lanes"] = seal_b.lanes
        out[f"zero_copy_{kind}_lanes{seal_b.lanes}"] = r
        for p in (hin, hout, hpt):
            hip.hipHostFree(p)
    print(json.dumps(out), flush=True)
    for o in (seal_b, open_b, ks, eng):
        o.close()


if __name__ == "__main__":
    main()
