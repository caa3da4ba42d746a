#!/usr/bin/env python3
"""Per-call latency of the drop-in plugin path at t/ptlsbench.c's shape (bench.py's plugin_ptlsbench), for
profiling: run under `rocprofv3 --kernel-trace --stats` to split a call into kernel time and host/launch time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "hsig-picotls_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402,F401  (torch's HIP runtime first)
import bench  # noqa: E402

if __name__ == "__main__":
    r = bench.plugin_ptlsbench()
    print({k: (v if not isinstance(v, dict) else {kk: v[kk] for kk in ("enc_us_per_call", "dec_us_per_call")}) for k, v in r.items()})
