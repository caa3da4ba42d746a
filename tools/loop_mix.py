#!/usr/bin/env python3
"""Instruction mix of the loops of one kernel in a `hipcc --cuda-device-only -S` listing.
usage: loop_mix.py file.s <kernel-symbol-substring> [min_instructions]"""
import re, sys
from collections import Counter
src, pat = sys.argv[1], sys.argv[2]
minn = int(sys.argv[3]) if len(sys.argv) > 3 else 200
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and pat in l)
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB[^:\s]+):", l)
    if m:
        labels[m.group(1)] = i
for i, l in enumerate(body):
    m = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\S+)|\s+s_branch\s+(\.LBB\S+)", l)
    if not m:
        continue
    tgt = m.group(1) or m.group(2)
    if tgt in labels and labels[tgt] < i:
        ins = [x.split()[0] for x in body[labels[tgt]:i + 1] if x.startswith("\t") and not x.strip().startswith((".", ";"))]
        if len(ins) < minn:
            continue
        c = Counter()
        for op in ins:
            if op.startswith("ds_"): c["lds:" + op] += 1
            elif op.startswith(("global_", "buffer_")): c["vmem:" + op] += 1
            elif op.startswith("s_waitcnt"): c["waitcnt"] += 1
            elif op.startswith("v_"): c["valu"] += 1; c["v:" + op] += 1
            elif op.startswith("s_"): c["salu"] += 1
            else: c[op] += 1
        print(f"loop {tgt} lines {labels[tgt]}-{i}: {len(ins)} instructions")
        for k, v in sorted(c.items(), key=lambda kv: -kv[1])[:40]:
            print(f"   {v:6d} {k}")
