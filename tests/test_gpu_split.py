"""Parity of split records, a measurement switch kept off in the product (batch_kernel.h / internal.h SPLIT_TASKS,
DESIGN.md §4.7): tests/split_case.py runs its cases on the TEST-ONLY alternate build alt/libptls_hip_split.so in a fresh
process.  Every case must plan split tasks and every record must equal the oracle (oracle/, pinned by lib/fusion.c),
open back, fail on a flipped tag byte and carry the oracle's header-protection mask.  The product plans none."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ALT = os.path.join(os.path.dirname(HERE), "hsig-picotls_amd", "alt", "libptls_hip_split.so")


@pytest.mark.parametrize("which,pct,ncases", [("runs", None, 5), ("chunks", "20", 2)])
def test_split_records_parity_on_the_alternate_build(which, pct, ncases):
    if not os.path.exists(ALT):
        pytest.fail(f"{ALT} missing: build it with `make -C hsig-picotls_amd alts` (part of __graft_entry__.build())")
    env = dict(os.environ, PTLS_HIP_LIB=ALT)
    if pct is not None:
        env["PTLS_HIP_SPLIT_PCT"] = pct
    out = subprocess.run([sys.executable, os.path.join(HERE, "split_case.py"), which], env=env, capture_output=True, text=True,
                         timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("MISMATCHES")]
    assert len(lines) == ncases and f"DONE lib={ALT}" in out.stdout, out.stdout[-2000:]
    for ln in lines:
        assert int(re.search(r"split_tasks=(\d+)", ln).group(1)) > 0, ln
        assert ln.endswith("seal=0 open=0"), ln


def test_product_plans_no_split_tasks(engine, oracle):
    """the product build keeps every task whole, on configs[3]'s shape too"""
    import ptls_hip
    import split_case
    recs = split_case.c4_like(oracle, 32, runs=2, per_run=64, seed=1)
    lens = [len(r[4]) for r in recs]
    r, *_ = ptls_hip.layout_records(lens, [5] * len(lens), [i // 64 for i in range(len(lens))], np.arange(len(lens)))
    b = ptls_hip.Batch(engine, r)
    b.set_lanes(16)
    assert b.split_tasks == 0
    b.close()
