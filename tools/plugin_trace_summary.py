#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of tools/plugin_probe.py: median kernel duration and median start-to-start
interval of the plugin's single-record launches per record size (encrypt = sparse kernel seal instantiation,
decrypt = open), of the one-block ECB launches, and of the key setups (one per context).

usage: tools/plugin_trace_summary.py <..._kernel_trace.csv>"""
import csv
import sys

import numpy as np

SIZES = (0, 16, 1500, 16384)  # plugin_probe.py's order, after a 50-call warm-up at 1500 B
WARM = 50


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    out = []

    def stats(rs):
        st = np.array([int(r["Start_Timestamp"]) for r in rs], dtype=np.float64)
        du = np.array([int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs], dtype=np.float64)
        gap = np.median(np.diff(st)) / 1e3 if len(st) > 1 else float("nan")
        return np.median(du) / 1e3, gap

    for kind, tag in (("encrypt", "false"), ("decrypt", "true")):
        ks = [r for r in rows if "aesgcm_sparse_kernel" in r["Kernel_Name"] and f", {tag}," in r["Kernel_Name"]]
        ks = ks[WARM:]
        for i, L in enumerate(SIZES):
            seg = ks[1000 * i:1000 * (i + 1)]
            if len(seg) == 1000:
                d, g = stats(seg)
                out.append(f"{kind:8s} {L:6d} B  kernel {d:7.2f} us  (launches {len(seg)})")
    ecb = [r for r in rows if "aesecb_batch_kernel" in r["Kernel_Name"]][WARM:]
    if ecb:
        d, g = stats(ecb)
        out.append(f"ecb      16 B      kernel {d:7.2f} us  start-to-start {g:7.2f} us  (launches {len(ecb)})")
    ks = [r for r in rows if "keysetup" in r["Kernel_Name"]]
    if ks:
        d, _ = stats(ks)
        name = ks[0]["Kernel_Name"].split("(")[0]
        out.append(f"keysetup one slot  kernel {d:7.2f} us  ({name}, {len(ks)} contexts)")
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1])
