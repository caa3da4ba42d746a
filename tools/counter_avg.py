#!/usr/bin/env python3
"""Average of one counter over the big batch / sparse kernel dispatches of a rocprofv3 --pmc run (start-up self-checks
dropped, tools/bench_dispatches.py), seal and open alike: usage counter_avg.py <pmc output dir> <counter> [scale]."""
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_dispatches import bench_dispatches  # noqa: E402

d, counter = sys.argv[1], sys.argv[2]
scale = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
f = glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True)
s, o = bench_dispatches(f[0], counter)
v = [x[counter] for x in s + o]
print(f"{counter} dispatches {len(v)} mean {sum(v) / len(v) * scale:.0f} min {min(v) * scale:.0f} max {max(v) * scale:.0f}")
