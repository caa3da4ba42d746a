#!/usr/bin/env python3
"""Can the host-resident path use the copy engines and the compute units' own PCIe traffic at the same time?

On 1 GiB of c2-shaped records in pinned host memory: ptls_hip_pipeline_seal/open over the MAPPED transport (the
kernels read and write host memory) alone, over the COPY transport (SDMA slices) alone, and the batch split between
the two, each part on its own pipeline driven from its own host thread (ctypes releases the GIL), for several
split fractions (usage: transport_mix_probe.py [config] [fractions, e.g. 0,0.25,1] [pipeline slice MiB, default 64]).  Reports seal+open GiB/s of the whole batch.  Timing plus a round-trip check; one JSON line."""
import json
import os
import sys
import threading
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


def main():
    cfg = dict(bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"])
    cfg["n"] = max(1, int((1 << 30) / (cfg["L"] or 8224)))
    eng = ptls_hip.Engine(0)
    idx, recs, in_total, out_total, lens = bench.make_workload(cfg, 0)
    keys, ivs = bench.make_keys(cfg)
    ks = ptls_hip.KeySet(eng, cfg["key_len"], cfg["keys"])
    ks.set(0, keys, ivs)
    n = len(recs)
    recs["aad_off"] = np.arange(n, dtype=np.uint64) * np.uint64(16)
    h_in = torch.empty(in_total + 64, dtype=torch.uint8).pin_memory()
    d_tmp = torch.zeros(in_total + 64, dtype=torch.uint8, device="cuda")
    b = ptls_hip.Batch(eng, recs)
    b.fill(d_tmp, bench.SEED_DATA, index=torch.from_numpy(idx.astype(np.int64)).cuda())
    torch.cuda.synchronize()
    h_in.copy_(d_tmp)
    b.close()
    del d_tmp
    h_aad = torch.from_numpy(bench.build_aad(cfg, idx, lens)).pin_memory()
    h_ct = torch.empty(out_total + 64, dtype=torch.uint8).pin_memory()
    h_pt = torch.empty(in_total + 64, dtype=torch.uint8).pin_memory()
    h_res = torch.zeros(n, dtype=torch.int64).pin_memory()
    ro = recs.copy()
    ro["in_off"], ro["out_off"] = recs["out_off"], recs["in_off"]
    sumL = float(lens.sum())
    slice_mib = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    pipes = {t: ptls_hip.Pipeline(eng, slice_mib << 20, transport=t) for t in (ptls_hip.TRANSPORT_MAPPED, ptls_hip.TRANSPORT_COPY)}
    res_np = h_res.numpy()

    def run(split, reps=3):
        """records [0, k) over MAPPED, [k, n) over COPY, concurrently; k = (1 - split) * n"""
        k = int(round((1.0 - split) * n))
        parts = [(pipes[ptls_hip.TRANSPORT_MAPPED], 0, k), (pipes[ptls_hip.TRANSPORT_COPY], k, n)]
        parts = [p for p in parts if p[2] > p[1]]

        def go(op):
            ths = []
            for p, lo, hi in parts:
                if op == "seal":
                    f = lambda p=p, lo=lo, hi=hi: p.seal(ks, recs[lo:hi], h_in, h_aad, h_ct)  # noqa: E731
                else:
                    f = lambda p=p, lo=lo, hi=hi: p.open(ks, ro[lo:hi], h_ct, h_aad, h_pt, h_res[lo:hi])  # noqa: E731
                ths.append(threading.Thread(target=f))
            t0 = time.perf_counter()
            for t in ths:
                t.start()
            for t in ths:
                t.join()
            return time.perf_counter() - t0
        go("seal")
        go("open")
        ts, to = [], []
        for _ in range(reps):
            ts.append(go("seal"))
            res_np[:] = 0
            to.append(go("open"))
        ok = bool((res_np == lens.astype(np.int64)).all())
        t_s, t_o = float(np.median(ts)), float(np.median(to))
        return {"copy_fraction": split, "seal_gibps": round(sumL / t_s / GIB, 2), "open_gibps": round(sumL / t_o / GIB, 2),
                "seal_open_gibps": round(2 * sumL / (t_s + t_o) / GIB, 2), "roundtrip_ok": ok}

    out = {"config": cfg["desc"], "records": n, "slice_mib": slice_mib, "runs": []}
    splits = [float(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0.0, 1.0, 0.15, 0.25, 0.35, 0.5]
    for split in splits:
        r = run(split)
        out["runs"].append(r)
        print(dict(r, slice_mib=slice_mib), flush=True)
    print(json.dumps(out), flush=True)
    for p in pipes.values():
        p.close()
    ks.close()
    eng.close()


if __name__ == "__main__":
    main()
