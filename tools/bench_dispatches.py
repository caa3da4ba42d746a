"""The bench's own batch-kernel dispatches in a rocprofv3 counter CSV.  Small dispatches (an engine's start-up
self-check) are dropped: a dispatch counts when its key counter is at least 5 % of the largest one.  The rest alternate
seal, open in dispatch order (each bench step seals then opens; rocprofv3 truncates the names to the kernel's base name,
so the OPEN template argument cannot tell them apart)."""
import csv
from collections import defaultdict


def bench_dispatches(path, key_counter, counters=None):
    """(seal dispatches, open dispatches): lists of {counter: value summed over the dispatch's rows}"""
    by = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(path)):
        if not r["Kernel_Name"].startswith(("aesgcm_batch_kernel", "aesgcm_sparse_kernel")):
            continue
        if counters is not None and r["Counter_Name"] not in counters:
            continue
        by[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    top = max((v.get(key_counter, 0.0) for v in by.values()), default=0.0)
    big = [by[d] for d in sorted(by) if by[d].get(key_counter, 0.0) >= 0.05 * top]
    return big[0::2], big[1::2]
