#!/usr/bin/env python3
"""HBM traffic per batch-kernel launch from tools/profile_round.sh output (FETCH_SIZE / WRITE_SIZE passes).
Dispatches of aesgcm_batch_kernel alternate seal, open (bench.py step); corrections per
MI355X_MICROARCH.md: FETCH_SIZE is in KiB and counts half of the wide coalesced reads on gfx950 (x2),
WRITE_SIZE is in KiB."""
import csv, glob, json, sys

out, cfg = sys.argv[1], sys.argv[2]


def per_launch(counter):
    """average counter value per seal and per open launch of the bench's own dispatches (tools/bench_dispatches.py)"""
    sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
    from bench_dispatches import bench_dispatches
    f = glob.glob(f"{out}/pmc_{counter}/**/run_counter_collection.csv", recursive=True)
    seal, opn = bench_dispatches(f[0], counter)
    return sum(v[counter] for v in seal) / len(seal), sum(v[counter] for v in opn) / len(opn)


def bench_line(log):
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no bench JSON line in {log}")


fs, fo = per_launch("FETCH_SIZE")
ws, wo = per_launch("WRITE_SIZE")
b = bench_line(f"{out}/trace.log")
alg = b["roofline"]["algorithmic_bytes_per_launch"]
fetch, write = int(fs * 1024 * 2), int(ws * 1024)
stats = glob.glob(f"{out}/trace/**/run_kernel_stats.csv", recursive=True)
avg_ns = None
if stats:  # the bench's kernel: the row with the largest total time (not a start-up self-check's tiny dispatches)
    rows = [r for r in csv.DictReader(open(stats[0])) if r["Name"].startswith(("aesgcm_batch_kernel", "aesgcm_sparse_kernel"))]
    if rows:
        avg_ns = float(max(rows, key=lambda r: float(r["TotalDurationNs"]))["AverageNs"])
print(json.dumps({
    "config": cfg,
    "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes (tools/profile_round.sh)",
    "correction": "FETCH_SIZE[KB]*1024*2 (gfx950 reports half of wide coalesced reads), WRITE_SIZE[KB]*1024",
    "fetch_bytes_per_seal_launch": fetch,
    "write_bytes_per_seal_launch": write,
    "hbm_bytes_per_seal_launch": fetch + write,
    "algorithmic_bytes_per_seal_launch": alg,
    "traffic_over_algorithmic": round((fetch + write) / alg, 4),
    "open": {"fetch_bytes": int(fo * 1024 * 2), "write_bytes": int(wo * 1024)},
    "bench_seal_ms_hip_events": b["seal_ms"], "bench_open_ms_hip_events": b["open_ms"],
    "rocprof_avg_ms_seal_and_open_launches": None if avg_ns is None else round(avg_ns / 1e6, 3),
}, indent=1))
