#!/usr/bin/env python3
"""Where the sparse-key kernel's time goes on c4s: the DIAGNOSTIC build
hsig-picotls_amd/diag/libptls_hip_stamps.so (sparse_kernel.hip STAMP_PHASES) has wave 0 of workgroup 0 sum the shader
cycles of each phase of its records; this runs bench.py's c4s workload (65 536 AES-256 records, one per key) once
sealed and once opened and prints the average microseconds per record of each phase.  The stamps drain the LDS reads at
every phase boundary, so the build's own run time is not quoted: read the shares.  One JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "hsig-picotls_amd", "diag", "libptls_hip_stamps.so")
os.environ["PTLS_HIP_LIB"] = LIB
for p in (ROOT, os.path.join(ROOT, "hsig-picotls_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402
import bench  # noqa: E402
import ptls_hip  # noqa: E402

PHASES = {2: "record_setup+ctr_const", 3: "h64_table", 4: "head_elems", 5: "stretch", 6: "tail_elems", 7: "valu_combine",
          8: "tag"}
cfg = dict(bench.CONFIGS["c4s"])
eng = ptls_hip.Engine(0)
idx, recs, in_total, out_total, lens = bench.make_workload(cfg, 0)
keys, ivs = bench.make_keys(cfg)
ks = ptls_hip.KeySet(eng, cfg["key_len"], cfg["keys"])
ks.set(0, keys, ivs)
sb = ptls_hip.Batch(eng, recs)
ro = recs.copy()
ro["in_off"], ro["out_off"] = recs["out_off"], recs["in_off"]
ob = ptls_hip.Batch(eng, ro)
d_pt = torch.zeros(in_total + 64, dtype=torch.uint8, device="cuda")
sb.fill(d_pt, bench.SEED_DATA, index=torch.from_numpy(idx.astype(np.int64)).cuda())
d_ct = torch.zeros(out_total + 64, dtype=torch.uint8, device="cuda")
d_out = torch.zeros(in_total + 64, dtype=torch.uint8, device="cuda")
d_aad = torch.zeros(len(recs) * 16, dtype=torch.uint8, device="cuda")
d_res = torch.zeros(len(recs), dtype=torch.int64, device="cuda")
out = {"lib": LIB, "records": len(recs), "lanes": sb.lanes}
for name, b, run in (("seal", sb, lambda: sb.seal(ks, d_pt, d_aad, d_ct)), ("open", ob, lambda: ob.open(ks, d_ct, d_aad, d_out, d_res))):
    for _ in range(3):
        run()  # warm-up (and the ciphertext open reads)
    clk = torch.zeros(max(64, 4 * b.grid), dtype=torch.int64, device="cuda")
    b.set_clock(clk)
    run()
    torch.cuda.synchronize()
    c = clk.cpu().numpy().view(np.uint64).astype(np.float64)
    b.set_clock(None)
    n = c[25]
    ghz = (c[28] - c[29]) / (c[27] - c[26]) * 0.1
    per = {v: round(c[16 + k] / n / ghz / 1e3, 3) for k, v in PHASES.items()}
    total = sum(per.values())
    out[name] = {"records_of_wave0": int(n), "clock_ghz": round(ghz, 3), "us_per_record": round(total, 3), **per,
                 "shares": {v: round(x / total, 3) for v, x in per.items()}}
print(json.dumps(out), flush=True)
