#!/usr/bin/env python3
"""Calibrate FETCH_SIZE / WRITE_SIZE on line-offset (16-byte packed) streams, the access the c3 packed-record traffic
figure rests on.  MI355X_MICROARCH.md calibrates the counters for line-aligned 16-B-per-lane streams only (FETCH_SIZE
counts half of them: x2) and calls other widths uncalibrated.

  run:    python3 tools/copy_calib.py run             (under rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE)
  parse:  python3 tools/copy_calib.py parse OUTDIR    (OUTDIR/pmc_FETCH_SIZE/..., OUTDIR/pmc_WRITE_SIZE/...)

`run` copies NBYTES with ptls_hip_device_copy (one 16-byte load and store per thread) REPS times for each
(source offset, destination offset) in CASES, in that order, so the copy16_kernel dispatches of the counter CSV are the
cases in order after the bench-independent start-up dispatches.  `parse` prints, per case, the counted bytes over the
bytes the copy reads and writes: an offset stream that reads back 1.00 (after the same x2) is measured as exactly as
an aligned one; more than that is what the counter adds for a stream that is not line aligned."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

NBYTES = 1 << 30
REPS = 3
CASES = [(0, 0), (16, 0), (0, 16), (48, 80), (64, 64)]


def run():
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "hsig-picotls_amd"))
    import torch
    assert torch.cuda.is_available()
    import ptls_hip
    eng = ptls_hip.Engine(0)
    src = torch.randint(0, 256, (NBYTES + 256,), dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    stream = torch.cuda.current_stream()
    for so, do in CASES:
        for _ in range(REPS):
            eng.copy(dst.data_ptr() + do, src.data_ptr() + so, NBYTES, stream)
        torch.cuda.synchronize()
        assert torch.equal(dst[do:do + NBYTES], src[so:so + NBYTES]), (so, do)
    eng.close()
    print(json.dumps({"cases": CASES, "reps": REPS, "nbytes": NBYTES}))


def per_dispatch(out, counter):
    f = glob.glob(f"{out}/pmc_{counter}/**/run_counter_collection.csv", recursive=True)
    by = defaultdict(float)
    for r in csv.DictReader(open(f[0])):
        if "copy16_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            by[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    vals = [by[d] for d in sorted(by)]
    return vals[-len(CASES) * REPS:]  # the calibration's own dispatches (bench-style device_copy warm-ups are not run)


def parse(out):
    fetch = per_dispatch(out, "FETCH_SIZE")
    write = per_dispatch(out, "WRITE_SIZE")
    rows = []
    for i, (so, do) in enumerate(CASES):
        f = sum(fetch[i * REPS:(i + 1) * REPS]) / REPS * 1024 * 2
        w = sum(write[i * REPS:(i + 1) * REPS]) / REPS * 1024
        rows.append({"src_offset": so, "dst_offset": do, "fetch_x2_over_bytes": round(f / NBYTES, 4),
                     "write_over_bytes": round(w / NBYTES, 4)})
    print(json.dumps({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, tools/copy_calib.py",
                      "kernel": "copy16_kernel (ptls_hip_device_copy)", "bytes_per_launch": NBYTES, "reps": REPS,
                      "cases": rows}, indent=1))


if __name__ == "__main__":
    run() if sys.argv[1] == "run" else parse(sys.argv[2])
