#!/usr/bin/env python3
"""Per-launch durations of the bench's batch-kernel dispatches from a rocprofv3 --kernel-trace CSV: small dispatches (an
engine's start-up self-check) dropped (< 5 % of the longest), the rest alternating seal / open in dispatch order (each
bench step seals then opens).  rocprofv3's own run_kernel_stats.csv averages every dispatch of the (truncated) kernel
name together, seal, open and the self-check alike.  usage: trace_summary.py <run_kernel_trace.csv>  -> one JSON line"""
import csv
import json
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"].startswith(("aesgcm_batch_kernel", "aesgcm_sparse_kernel"))]
rows.sort(key=lambda r: int(r["Dispatch_Id"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Kernel_Name"]) for r in rows]
top = max(d for d, _ in dur)
big = [d for d, _ in dur if d >= 0.05 * top]
kept = sorted({n for d, n in dur if d >= 0.05 * top})
seal, opn = big[0::2], big[1::2]
med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
print(json.dumps({"source": sys.argv[1], "kernel": "/".join(kept), "dispatches": len(dur), "small_dropped": len(dur) - len(big),
                  "seal_launches": len(seal), "seal_avg_ms": round(sum(seal) / len(seal) / 1e6, 3), "seal_median_ms": round(med(seal) / 1e6, 3),
                  "open_launches": len(opn), "open_avg_ms": round(sum(opn) / len(opn) / 1e6, 3), "open_median_ms": round(med(opn) / 1e6, 3)}))
