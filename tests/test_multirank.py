"""world_size-2 gloo test of bench.py's multi-GPU logic on CPU: record shards are disjoint and cover the
job, keys/seq stay globally consistent, and the reported time is the max over ranks."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, cfg, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "hsig-picotls_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    idx, recs, in_total, out_total, lens = bench.make_workload(cfg, rank)
    t = bench.max_over_ranks(1.0 + rank, world)
    q.put((rank, idx.copy(), recs["key"].copy(), recs["seq"].copy(), lens.copy(), t))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cfg, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return out


def test_single_key_shards():
    cfg = dict(n=4096, L=1350, key_len=16, keys=1, aad="quic")
    out = _run(cfg)
    all_idx = np.concatenate([o[1] for o in out])
    assert np.array_equal(np.sort(all_idx), np.arange(2 * 4096, dtype=np.uint64))  # disjoint, complete
    for rank, idx, key, seq, lens, t in out:
        assert np.array_equal(idx, np.arange(rank * 4096, (rank + 1) * 4096, dtype=np.uint64))
        assert np.array_equal(seq, idx) and not key.any()
        assert t == 2.0  # max over ranks (1.0, 2.0)


def test_multi_key_shards_key_major():
    K = 64
    cfg = dict(n=K * 8, L=None, key_len=32, keys=K, aad="tls")
    out = _run(cfg)
    all_idx = np.concatenate([o[1] for o in out])
    assert np.array_equal(np.sort(all_idx), np.arange(2 * K * 8, dtype=np.uint64))
    for rank, idx, key, seq, lens, t in out:
        assert np.array_equal(key, (idx % K).astype(np.uint32))  # record i uses key i mod K
        assert np.array_equal(seq, idx // K)                       # per-key sequence number
        assert np.all(np.diff(key.astype(np.int64)) >= 0)          # same-key records adjacent
        assert lens.min() >= 64 and lens.max() <= 16384


def _bench(*extra, env=None, config="c3", records=2048):
    import json
    import subprocess
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--config", config, "--records", str(records),
                          "--steps", "3", "--warmup", "1", *extra], env=e, capture_output=True, text=True, timeout=240)
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    return out.returncode, [json.loads(ln) for ln in lines], out.stderr


def test_bench_launches_its_own_ranks():
    """`bench.py --gpus 2` with no launcher around it starts 2 ranks itself (torch.distributed.run, 127.0.0.1), as the
    driver's plain `bench.py --gpus N` would on an 8-GPU node; rank 0 alone prints one line with n_gpus 2, both
    ranks' own rates, and a whole-node rate of the ranks' bytes over the slowest rank's time"""
    rc, lines, err = _bench("--gpus", "2")
    assert rc == 0, err[-3000:]
    assert len(lines) == 1, lines
    r = lines[0]
    assert r["n_gpus"] == 2 and len(r["per_rank"]) == 2
    # disjoint record ranges: the first 2048 records of each rank's 4M-record shard (configs[2] per GPU), so every rank
    # holds records with lib/fusion.c digests (tests/golden/configs.json) for its parity check
    assert [x[0] for x in r["first_index_per_rank"]] == [0.0, float(4 << 20)]
    assert [x["records"] for x in r["per_rank"]] == [[0, 2048], [4 << 20, (4 << 20) + 2048]]
    assert all(x["golden_records_checked"] >= 64 for x in r["per_rank"])
    slow = max(x["seconds"] for x in r["per_rank"])
    assert r["per_rank"][1]["seconds"] > r["per_rank"][0]["seconds"]  # rank 1 sleeps twice as long
    total = 2 * 2 * 2048 * 1350 * 3 / (1 << 30)  # ranks x (seal + open) x bytes x steps
    assert abs(r["value"] - total / (r["ms_per_step"] * 3 / 1e3)) / r["value"] < 0.02
    assert r["ms_per_step"] * 3 / 1e3 >= slow - 1e-3  # the max over ranks (JSON fields are rounded)


def test_bench_rejects_a_world_size_mismatch():
    rc, lines, err = _bench("--gpus", "2", env={"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc == 2 and not lines and "WORLD_SIZE=3" in err


def test_partition_bytes_balances_payload():
    """contiguous ranges of about equal payload bytes (prefix sum of L) on configs[3]'s lengths"""
    sys.path.insert(0, ROOT)
    import bench
    cfg = dict(bench.CONFIGS["c4"])
    lens = bench.record_lengths(cfg, np.arange(1 << 16, dtype=np.uint64))
    for parts in (1, 2, 3, 8):
        b = bench.partition_bytes(lens, parts)
        assert b[0] == 0 and b[-1] == len(lens) and all(x <= y for x, y in zip(b, b[1:]))
        share = [int(lens[b[r]:b[r + 1]].sum()) for r in range(parts)]
        assert sum(share) == int(lens.sum())
        assert max(share) - min(share) <= 2 * 16384  # within one record's bytes of the mean on both sides
    # equal counts for fixed L
    assert bench.partition_bytes(np.full(4096, 1350, dtype=np.uint64), 4) == [0, 1024, 2048, 3072, 4096]
    assert bench.partition_bytes(np.zeros(0, dtype=np.uint64), 2) == [0, 0, 0]


def test_bench_strong_scaling_splits_by_bytes():
    """--scaling strong: ONE batch of configs[3]'s records split over 2 ranks by payload bytes, not by count"""
    rc, lines, err = _bench("--gpus", "2", "--scaling", "strong", config="c4", records=1 << 16)
    assert rc == 0, err[-3000:]
    r = lines[0]
    assert r["scaling"] == "strong"
    (a0, a1), (b0, b1) = (x["records"] for x in r["per_rank"])
    assert a0 == 0 and a1 == b0 and b1 == 1 << 16  # contiguous, complete
    p0, p1 = (x["payload_bytes"] for x in r["per_rank"])
    assert abs(p0 - p1) <= 2 * 16384


def test_every_rank_of_the_weak_c2_split_has_golden_records():
    """bench.py checks sealed records against lib/fusion.c digests on EVERY rank: the fixture holds the first and last
    64 records of each rank's 1M-record shard of configs[1] at up to 8 GPUs (and configs[4]'s 8 shards)"""
    sys.path.insert(0, ROOT)
    import bench
    for name in ("c2", "c3", "c4", "c5"):
        g = bench.golden_digests(name)
        n = bench.CONFIGS[name]["n"]
        for rank in range(8):
            lo, hi = bench.rank_range(bench.CONFIGS[name], rank, 8, "weak")
            head = np.arange(lo, lo + 64, dtype=np.uint64)
            tail = np.arange(hi - 64, hi, dtype=np.uint64)
            assert len(bench.golden_positions(head, g)) == 64 and len(bench.golden_positions(tail, g)) == 64, (name, rank)
            assert hi - lo == n
