"""The multi-rank bench path on hardware (never run on a GPU before round 3): `bench.py --gpus 2` starts
its own two ranks (torch.distributed.run, gloo for the barriers and the timing summary, no RCCL), here both on device 0
(--device 0), each sealing / opening its own shard of configs[4] and checking its sealed records against the
lib/fusion.c digests of tests/golden/configs.json."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=300):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True, text=True,
                       timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, [json.loads(ln) for ln in lines], r.stderr


def test_bench_two_ranks_on_one_device():
    rc, lines, err = _bench("--gpus", "2", "--device", "0", "--config", "c5", "--records", "65536", "--steps", "2",
                            "--warmup", "1", "--no-cpu-baseline", "--no-e2e", "--no-plugin")
    assert rc == 0, err[-4000:]
    assert len(lines) == 1
    r = lines[0]
    assert r["n_gpus"] == 2 and len(r["per_rank"]) == 2 and r["scaling"] == "weak"
    assert [x["records"] for x in r["per_rank"]] == [[0, 65536], [4 << 20, (4 << 20) + 65536]]
    # every rank checked its own sealed records against lib/fusion.c (first 64 of its 4M shard, +1 seam record)
    assert all(x["golden_records_checked"] >= 64 for x in r["per_rank"]), r["per_rank"]
    assert r["parity"]["open_all_ok"] and r["parity"]["roundtrip_bytes_equal"]
    assert r["value"] > 0 and all(x["seal_gibps"] > 0 for x in r["per_rank"])
    assert r["clock_in_run"]["seal_ghz"] > 0.5
