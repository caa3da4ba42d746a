"""The multi-rank bench path on hardware (never run on a GPU before round 3): `bench.py --gpus 2` starts
its own two ranks (torch.distributed.run, gloo for the barriers and the timing summary, no RCCL), here both on device 0
(--device 0), each sealing / opening its own shard of configs[4] and checking its sealed records against the
lib/fusion.c digests of tests/golden/configs.json; rank 0 then times the reference's CPU engines with the GPUs idle, so
the N > 1 line carries its cpu_baseline too."""
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
                            "--warmup", "1", "--cpu-sample-mib", "64", "--e2e-records", "20000", "--no-plugin")
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
    # the whole node's host-resident figure, driven by rank 0 through the node API over both ranks' devices
    e = r["host_e2e_node"]
    assert e["devices"] == [0, 0] and len(e["per_device"]) == 2 and e["seal_open_gibps"] > 0
    assert e["parity"]["open_all_ok"] and e["parity"]["roundtrip_bytes_equal"] and e["parity"]["golden_records_checked"] >= 64
    # an N > 1 line carries its own CPU baseline (rank 0, GPUs idle), with the labelled whole-host extrapolation
    c = r["cpu_baseline"]
    assert c["kind"] == "reference" and c["cores"] >= 1 and c["value"] > 0, c
    x = c["full_host_extrapolation"]
    assert x["kind"].startswith("extrapolation") and x["physical_cores"] >= c["cores"] and x["gibps"] > c["single_core"]


def test_bench_node_e2e_device_listed_twice():
    """bench.py --node-e2e: the host-resident path over a node's devices in one process (ptls_hip_node_*), each device's
    records in host memory bound to its NUMA node; here device 0 listed twice (two engines, two host threads).  Reports the
    NUMA node every device's range went to, and the share of its input pages found there (move_pages)."""
    rc, lines, err = _bench("--node-e2e", "0,0", "--config", "c4", "--e2e-records", "30000")
    assert rc == 0, err[-4000:]
    r = lines[-1]
    assert r["devices"] == [0, 0] and r["records"] == 30000 and len(r["per_device"]) == 2
    assert r["parity"]["open_all_ok"] and r["parity"]["roundtrip_bytes_equal"]
    assert r["parity"]["golden_records_checked"] >= 64  # configs[3]'s first 64 records against lib/fusion.c
    assert all(isinstance(x, int) for x in r["numa_nodes"]) and r["numa_nodes"][0] == r["numa_nodes"][1]
    for d in r["per_device"]:
        assert d["seal_s"] > 0 and d["records"][1] > d["records"][0]
        if d["numa_node"] >= 0:  # a known node: the range's pages were bound there
            assert d["input_pages_on_its_node"] == 1.0, d
    print(json.dumps({k: r[k] for k in ("seal_open_gibps", "numa_nodes", "per_device")}))
