#!/usr/bin/env python3
"""Summarise tools/pmc_passes.sh output: per-dispatch counter values of the batch kernel (first dispatch
of each bench step = seal), averaged."""
import csv
import glob
import sys
from collections import defaultdict

out = sys.argv[1]
vals = defaultdict(list)
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from bench_dispatches import bench_dispatches  # noqa: E402
for f in sorted(glob.glob(f"{out}/pass*/run_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    names = {r["Counter_Name"] for r in rows}
    key = "GRBM_GUI_ACTIVE" if "GRBM_GUI_ACTIVE" in names else sorted(names)[0] if names else None
    if key is None:
        continue
    seal, _ = bench_dispatches(f, key)
    for v in seal:
        for c, x in v.items():
            vals[c].append(x)
avg = {k: sum(v) / len(v) for k, v in vals.items()}
for k in sorted(avg):
    print(f"{k:28s} {avg[k]:18.1f}")
if "SQ_WAVE_CYCLES" in avg and "SQ_BUSY_CYCLES" in avg:
    wc = avg["SQ_WAVE_CYCLES"]
    print("--- shares of wave-cycles: wait_any %.3f wait_inst_any %.3f active_any %.3f valu %.3f lds %.3f" % (
        avg["SQ_WAIT_ANY"] / wc, avg["SQ_WAIT_INST_ANY"] / wc, avg["SQ_ACTIVE_INST_ANY"] / wc,
        avg["SQ_ACTIVE_INST_VALU"] / wc, avg["SQ_ACTIVE_INST_LDS"] / wc))

# LDS-array occupancy of the seal launch (per CU), for bench.py's roofline block: --json <path>
if "--json" in sys.argv and "SQ_LDS_IDX_ACTIVE" in avg and "GRBM_GUI_ACTIVE" in avg:
    import json
    cyc = avg["GRBM_GUI_ACTIVE"] / 8  # GRBM_GUI_ACTIVE sums the 8 XCDs
    busy = avg["SQ_LDS_IDX_ACTIVE"] / 256 / cyc
    out = {"lds_array_busy_frac": round(busy, 4), "lds_idx_active_cycles_per_cu": round(avg["SQ_LDS_IDX_ACTIVE"] / 256),
           "kernel_cycles_per_xcd": round(cyc),
           "source": "rocprofv3 --pmc SQ_LDS_IDX_ACTIVE / GRBM_GUI_ACTIVE, separate pass (tools/pmc_passes.sh), seal launch"}
    if "SQ_INSTS_VALU" in avg:
        # a wave64 VALU instruction occupies its SIMD-32 for 2 cycles (MI355X_MICROARCH.md); 1024 SIMDs
        out["valu_insts_per_seal_launch"] = round(avg["SQ_INSTS_VALU"])
        out["valu_issue_busy_frac"] = round(avg["SQ_INSTS_VALU"] * 2 / 1024 / cyc, 4)
        out["valu_source"] = "SQ_INSTS_VALU x 2 cycles / 1024 SIMDs / GRBM_GUI_ACTIVE per XCD (another pass of the same bench command)"
    with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
        json.dump(out, f, indent=1)
