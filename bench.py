#!/usr/bin/env python3
"""bench.py -- device-resident AES-GCM seal+open throughput of the MI355X engine (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c4s|c5]

--gpus N > 1 without a launcher starts N rank processes itself (torch.distributed.run on 127.0.0.1, before
any GPU call); under a launcher WORLD_SIZE must equal N.  Ranks meet only over gloo (CPU): barriers and the timing
summary; RCCL is not used anywhere (the records need no exchange).  --device D puts every rank on device D (a
rehearsal of the N-rank path on a one-GPU box).  --scaling strong splits ONE batch of the config's records over the
ranks in contiguous ranges of equal payload bytes (prefix sum of L); the default (weak) gives every
rank its own shard of the config's size.

One step = seal of the whole per-GPU batch followed by open of the sealed batch (the BASELINE metric is
"seal+open"), inputs already resident in HBM.  Default workload = BASELINE.json configs[1]
("c2": 1M x 16 KiB TLS records, AES-128-GCM, one key) on every GPU: records are sharded by range,
each rank owns its own 1M records (weak scaling), no collective touches the data path; ranks only
meet at the barriers and the max-over-ranks of the timed region.

Rank 0 prints ONE JSON line.  value = whole-job GiB/s = sum over ranks of 2 * sum(L) per step / the slowest
rank's time; per_rank lists every rank's own rate.
Extra fields: roofline (seal kernel vs the 8 TB/s HBM peak), cpu_baseline (lib/fusion.c on this host's
cores, oracle/_ref), parity (sampled records vs the golden digests of lib/fusion.c + full open check).
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hsig-picotls_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md chip table

SEED_DATA = 0x70746C7300000001
SEED_KEY = 0x6B65790000000000
SEED_AAD = 0x6161640000000000
SEED_LEN = 0x00000000006C656E
GAMMA = np.uint64(0x9E3779B97F4A7C15)

CONFIGS = {  # SURVEY.md §8(d); n = records per GPU
    "c2": dict(n=1 << 20, L=16384, key_len=16, keys=1, aad="tls",
               desc="AES-128-GCM, 1M x 16 KiB TLS records, single key, per GPU (BASELINE configs[1])"),
    "c3": dict(n=4 << 20, L=1350, key_len=16, keys=1, aad="quic",
               desc="AES-128-GCM, 4M x 1350 B QUIC records, 13 B AAD, single key (configs[2])"),
    "c4": dict(n=4 << 20, L=None, key_len=32, keys=1 << 16, aad="tls",
               desc="AES-256-GCM, 4M mixed 64 B-16 KiB records, 64K keys (configs[3])"),
    "c4s": dict(n=1 << 16, L=None, key_len=32, keys=1 << 16, aad="tls",
                desc="AES-256-GCM, 64K mixed 64 B-16 KiB records, ONE per key over 64K keys (a server batch of one "
                     "record per connection; configs[3]'s first 64K records; sparse-key kernel)"),
    "c5": dict(n=4 << 20, L=1350, key_len=16, keys=1, aad="quic",
               desc="AES-128-GCM, 32M x 1350 B records sharded 4M per GPU over 8 GPUs (configs[4])"),
}


def splitmix_at(seed, k):
    """k-th output of the splitmix64 stream seeded with `seed` (vectorised over seed and/or k)"""
    with np.errstate(over="ignore"):
        z = np.asarray(seed, dtype=np.uint64) + (np.asarray(k, dtype=np.uint64) + np.uint64(1)) * GAMMA
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def stream_bytes(seeds, nbytes):
    """[len(seeds), nbytes] uint8: the first nbytes of each seed's stream"""
    seeds = np.asarray(seeds, dtype=np.uint64)
    words = (nbytes + 7) // 8
    w = splitmix_at(seeds[:, None], np.arange(words, dtype=np.uint64)[None, :])
    return w.astype("<u8").view(np.uint8).reshape(len(seeds), words * 8)[:, :nbytes]


def record_lengths(cfg, idx):
    """payload bytes of records idx (fixed L, or 64 + splitmix64(0x6C656E ^ i) mod 16321)"""
    idx = np.asarray(idx, dtype=np.uint64)
    if cfg["L"] is None:
        return (np.uint64(64) + splitmix_at(np.uint64(SEED_LEN) ^ idx, 0) % np.uint64(16321)).astype(np.uint64)
    return np.full(len(idx), cfg["L"], dtype=np.uint64)


def partition_bytes(lens, parts):
    """contiguous ranges [b[r], b[r + 1]) of records with about equal payload bytes each (prefix sum
    of L): range r ends at the first record whose prefix sum reaches (r + 1) / parts of the total.  The same rule as
    ptls_hip_partition_bytes (node.cpp)."""
    lens = np.asarray(lens, dtype=np.uint64)
    csum = np.cumsum(lens, dtype=np.uint64)
    total = int(csum[-1]) if len(csum) else 0
    b = [0]
    for r in range(1, parts):
        target = (total * r + parts - 1) // parts  # ceil(total * r / parts)
        b.append(max(b[-1], int(np.searchsorted(csum, np.uint64(target), side="left")) + 1 if total else 0))
    b.append(len(lens))
    return [min(x, len(lens)) for x in b]


def rank_range(cfg, rank, world, scaling, n_total=None):
    """global record indices [lo, hi) of this rank: weak = its own shard of the config's per-GPU size (cfg["n"],
    truncated to --records), strong = its byte-balanced part of one batch of cfg["n"] records"""
    if scaling == "weak":
        base = rank * (n_total or cfg["n"])
        return base, base + cfg["n"]
    b = partition_bytes(record_lengths(cfg, np.arange(cfg["n"], dtype=np.uint64)), world)
    return b[rank], b[rank + 1]


def record_align(align=None):
    """the byte alignment of each record's offsets: --align, else PTLS_BENCH_ALIGN (environment, the tools' knob), else 128"""
    return int(align or os.environ.get("PTLS_BENCH_ALIGN", "128"))


def make_workload(cfg, rank, world=1, scaling="weak", n_full=None, align=None):
    """per-rank record descriptors, in key-major order (records of one key adjacent), each record's input and output at
    a multiple of `align` bytes (record_align)"""
    import ptls_hip
    lo, hi = rank_range(cfg, rank, world, scaling, n_full)
    n = hi - lo
    base = lo
    if cfg["keys"] == 1:
        idx = np.arange(base, base + n, dtype=np.uint64)
        keyslot = np.zeros(n, dtype=np.uint32)
        seq = idx.copy()
    else:  # record i uses key i % K, per-key seq i // K; order records by key (any n, not only multiples of K)
        K = np.uint64(cfg["keys"])
        allidx = np.arange(base, base + n, dtype=np.uint64)
        idx = allidx[np.argsort(allidx % K, kind="stable")]
        keyslot = (idx % K).astype(np.uint32)
        seq = (idx // K).astype(np.uint64)
    lens = record_lengths(cfg, idx)
    aad_len = 5 if cfg["aad"] == "tls" else 13
    # records at 128-byte (L2 line) aligned offsets by default: no line holds the end of one record and the start of the
    # next, which different waves write at different times.  --align 16 packs them as a QUIC stack's datagram buffers
    # would (c3: 1.11x the algorithmic HBM bytes against 1.05x at 128, profiles/traffic_c3_packed.json)
    align = record_align(align)
    recs, in_total, out_total, _ = ptls_hip.layout_records(lens, np.full(n, aad_len), keyslot, seq, align=align)
    recs["aad_off"] = np.arange(n, dtype=np.uint64) * np.uint64(16)
    return idx, recs, in_total, out_total, lens


def build_aad(cfg, idx, lens):
    n = len(idx)
    aad = np.zeros((n, 16), dtype=np.uint8)
    if cfg["aad"] == "tls":  # 17 03 03 len16(L + 16): build_aad, lib/picotls.c:696-703
        reclen = lens + np.uint64(16)
        aad[:, 0], aad[:, 1], aad[:, 2] = 0x17, 0x03, 0x03
        aad[:, 3] = (reclen >> np.uint64(8)).astype(np.uint8)
        aad[:, 4] = (reclen & np.uint64(0xFF)).astype(np.uint8)
    else:
        for s in range(0, n, 1 << 20):
            aad[s:s + (1 << 20), :13] = stream_bytes(np.uint64(SEED_AAD) ^ idx[s:s + (1 << 20)], 13)
    return aad.reshape(-1)


def make_keys(cfg):
    K, kl = cfg["keys"], cfg["key_len"]
    s = stream_bytes(np.uint64(SEED_KEY) ^ np.arange(K, dtype=np.uint64), kl + 12)
    return s[:, :kl].tobytes(), s[:, kl:kl + 12].tobytes()


def cpu_share():
    """(cpus to use, cpus in the affinity mask, cgroup CPU quota or None): every CPU this process may run on,
    bounded by the container's CPU quota (a GPU box shows the whole machine in its mask but grants a share)"""
    try:
        aff = sorted(os.sched_getaffinity(0))
    except AttributeError:
        aff = list(range(os.cpu_count() or 1))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:  # cgroup v2: "<quota> <period>" or "max <period>"
            q, per = f.read().split()
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f1, open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f2:
                q, per = int(f1.read()), int(f2.read())
                if q > 0:
                    quota = q / per
        except (OSError, ValueError):
            pass
    n = len(aff) if quota is None else max(1, min(len(aff), int(quota + 1e-9)))
    return aff[:n], len(aff), quota


def gpu_local_cpus(dev, cpus):
    """order `cpus` for a CPU baseline that stands beside GPU `dev`: physical cores (one hardware thread per core) of the
    GPU's NUMA node first, then the other physical cores, then SMT siblings.  Returns (ordered cpus, NUMA node or None,
    the node's cpus).  The node comes from the GPU's PCI device in sysfs (hipDeviceGetPCIBusId)."""
    import ctypes
    node, node_cpus = None, set()
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, dev) == 0:
            with open(f"/sys/bus/pci/devices/{buf.value.decode().lower()}/numa_node") as f:
                node = int(f.read())
            if node >= 0:
                with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
                    node_cpus = set(_cpulist(f.read()))
            else:
                node = None
    except (OSError, ValueError):
        node = None

    def primary(c):  # the first hardware thread of its core
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                return min(_cpulist(f.read())) == c
        except (OSError, ValueError):
            return True
    rank = {c: (0 if c in node_cpus else 1) + (0 if primary(c) else 2) for c in cpus}
    return sorted(cpus, key=lambda c: (rank[c], c)), node, sorted(node_cpus)


def _cpulist(text):
    out = []
    for part in text.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        elif part:
            out.append(int(part))
    return out


def host_topology():
    """sockets and physical cores of the whole host from sysfs (every CPU present, not only this process's share):
    a core = a distinct (physical_package_id, core_id)"""
    cores, sockets = set(), set()
    base = "/sys/devices/system/cpu"
    try:
        names = [d for d in os.listdir(base) if d.startswith("cpu") and d[3:].isdigit()]
    except OSError:
        names = []
    for d in names:
        try:
            with open(f"{base}/{d}/topology/physical_package_id") as f1, open(f"{base}/{d}/topology/core_id") as f2:
                pkg, core = int(f1.read()), int(f2.read())
        except (OSError, ValueError):
            continue
        sockets.add(pkg)
        cores.add((pkg, core))
    return dict(sockets=len(sockets) or None, physical_cores=len(cores) or None, logical_cpus=len(names) or None)


def _steady(run_rep, min_reps=5, min_s=3.0, max_s=20.0, tol=0.10):
    """repeat run_rep() (-> GiB/s of one rep) until the last min_reps agree within tol of their median, or max_s;
    "noisy" says the spread bar was not met (a shared host: the GPU box grants a CPU share of a larger machine)"""
    rates, t0 = [], time.time()
    while True:
        rates.append(run_rep())
        last = rates[-min_reps:]
        spread = (max(last) - min(last)) / float(np.median(last))
        el = time.time() - t0
        if len(rates) >= min_reps and ((spread <= tol and el >= min_s) or el >= max_s):
            return dict(median=round(float(np.median(last)), 3), min=round(min(last), 3), max=round(max(last), 3),
                        spread=round(spread, 4), reps=len(rates), reps_used=len(last), noisy=bool(spread > tol))


def cpu_baseline(cfg_name, cfg, dev=0, sample_bytes=1 << 30):
    """The reference's CPU engines (oracle/_ref, built unmodified from lib/fusion.c) on this host's cores: distinct record
    buffers of the config's shape (about 1 GiB, larger than the CPU caches, like the GPU's HBM-resident batch), the
    config's AAD form, one ptls_aead_context_t per pinned thread.  Two engines, the same bytes:
      fusion        ptls_fusion_aes{128,256}gcm (lib/fusion.c:400-844, 128-bit AES-NI / PCLMUL)
      non_temporal  ptls_non_temporal_aes{128,256}gcm (lib/fusion.c:1258-2179: 256-bit VAES / VPCLMULQDQ encrypt when the
                    CPU has them, ptls_fusion_can_aesni256; what ptls_send uses with fusion)
    `value` is the faster of the two.  Threads go to physical cores of the GPU's NUMA node first (gpu_local_cpus), as many as
    the host's CPU share grants.  Each rep = one seal pass + one open pass over the sample (repeated inside the rep to last
    >= 0.3 s); reps repeat until five agree within 10 %.  Reported: median of those five, min / max, for 1 thread and for
    every CPU available."""
    import ctypes
    from oracle_lib import Ref, ORACLE_SO
    L = cfg["L"] or 8224
    nrec = max(64, sample_bytes // L)
    stride = (L + 16 + 63) // 64 * 64
    aad_len = 5 if cfg["aad"] == "tls" else 13
    if not Ref.available:
        o = ctypes.CDLL(ORACLE_SO)
        o.oracle_bench_seal.restype = ctypes.c_double
        o.oracle_bench_seal.argtypes = [ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int]
        n = 64
        t = o.oracle_bench_seal(cfg["key_len"], n, L, 1)
        return dict(value=n * L / t / GIB, unit="GiB/s (seal only)", cores=1, kind="port",
                    sample=f"{n} x {L} B records, oracle C port, single thread")
    rng = np.random.default_rng(2024)
    data = np.frombuffer(rng.bytes(nrec * stride), dtype=np.uint8).reshape(nrec, stride).copy()
    idx = np.arange(nrec, dtype=np.uint64)
    aad = build_aad(cfg, idx, np.full(nrec, L, dtype=np.uint64)).reshape(nrec, 16)[:, :aad_len].copy()
    key, iv = (b"\x11" * cfg["key_len"]), b"\x22" * 12
    share, n_aff, quota = cpu_share()
    try:
        aff = sorted(os.sched_getaffinity(0))
    except AttributeError:
        aff = share
    ordered, node, node_cpus = gpu_local_cpus(dev, aff)
    cpus = ordered[:len(share)]
    threads = len(cpus)
    ref = Ref()
    ref.lib.ref_bench_algo.restype = ctypes.c_double
    ref.lib.ref_bench_algo.argtypes = [ctypes.c_int] + list(ref.lib.ref_bench.argtypes)
    ct = np.zeros_like(data)
    pt = np.zeros_like(data)

    def run(nt, do_open, src, dst, nthreads, passes, aad_arr, alen):
        arr = (ctypes.c_int * nthreads)(*cpus[:nthreads])
        return ref.lib.ref_bench_algo(nt, cfg["key_len"] * 8, do_open, key, iv, src.ctypes.data, dst.ctypes.data, nrec, L, stride,
                                      aad_arr.ctypes.data, alen, nthreads, arr, passes)

    def measure(nt, nthreads, aad_arr, alen):
        run(nt, 0, data, ct, nthreads, 1, aad_arr, alen)  # warm-up, and valid ciphertext for open
        t1 = run(nt, 0, data, ct, nthreads, 1, aad_arr, alen) + run(nt, 1, ct, pt, nthreads, 1, aad_arr, alen)
        passes = max(1, int(np.ceil(0.3 / max(t1, 1e-6))))
        st = _steady(lambda: 2 * passes * nrec * L / (run(nt, 0, data, ct, nthreads, passes, aad_arr, alen) +
                                                      run(nt, 1, ct, pt, nthreads, passes, aad_arr, alen)) / GIB)
        assert np.array_equal(pt[:, :L], data[:, :L]), "reference round trip failed"
        st["passes_per_rep"] = passes
        return st

    engines = {"fusion": 0, "non_temporal": 1}
    out = {name: {n: measure(nt, n, aad, aad_len) for n in sorted({1, threads})} for name, nt in engines.items()}
    best_name = max(out, key=lambda k: out[k][threads]["median"])
    # BASELINE configs[0]'s shape: 4K x 16 KiB with t/ptlsbench.c's 32-byte AAD uint64_t h[4], h[0] = seq (:129-141)
    h = np.zeros((nrec, 4), dtype="<u8")
    h[:, 0] = np.arange(1, nrec + 1, dtype=np.uint64)
    h8 = h.view(np.uint8).reshape(nrec, 32).copy()
    conf1 = None
    if L == 16384:
        saved = nrec
        nrec = 4096
        conf1 = {n: measure(engines[best_name], n, h8, 32) for n in sorted({1, threads})}
        nrec = saved
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    best = out[best_name][threads]
    on_node = sum(1 for c in cpus if c in set(node_cpus))
    res = dict(value=best["median"], unit="GiB/s seal+open", cores=threads, kind="reference", engine=best_name,
               min=best["min"], max=best["max"], spread=best["spread"], reps=best["reps"], noisy=best["noisy"],
               spread_target=0.10,
               single_core=out[best_name][1]["median"], single_core_min=out[best_name][1]["min"],
               single_core_spread=out[best_name][1]["spread"],
               engines={name: dict(all_cores=o[threads]["median"], all_cores_spread=o[threads]["spread"],
                                   single_core=o[1]["median"]) for name, o in out.items()},
               cpus_used=cpus, gpu_numa_node=node, cpus_on_gpu_node=on_node,
               cpus_in_affinity=n_aff, cgroup_cpu_quota=quota,
               fusion_can_aesni256=bool(ref.lib.ref_fusion_can_aesni256()), cpu=cpu_model,
               sample=f"{nrec} x {L} B distinct records ({nrec * L / GIB:.2f} GiB, {cfg_name} shape, {aad_len} B AAD), "
                      f"lib/fusion.c's {best_name} engine (the faster of ptls_fusion_aes*gcm and ptls_non_temporal_aes*gcm) "
                      f"via ptls_aead_encrypt/decrypt, one context per thread pinned to a physical core "
                      f"({on_node} of {threads} on the GPU's NUMA node {node}); median of 5 reps within "
                      f"{best['spread'] * 100:.1f} %, {threads} threads"
                      + (f" (the host's cgroup grants {quota:g} CPUs of the {n_aff} in the affinity mask)" if quota else ""))
    topo = host_topology()
    if topo["physical_cores"]:
        # the measured value is the box's CPU share; what the whole host could do is only estimated here
        res["full_host_extrapolation"] = dict(
            gibps=round(res["single_core"] * topo["physical_cores"], 1), single_core=res["single_core"],
            physical_cores=topo["physical_cores"], sockets=topo["sockets"], logical_cpus=topo["logical_cpus"],
            kind="extrapolation, not a measurement",
            note="one NUMA-local core's rate x every physical core of the host's sockets (sysfs topology); linear in the "
                 "cores, so it ignores the host DRAM bandwidth the records stream through (every byte read once and "
                 "written once per pass) and the clock drop with all cores busy: an upper estimate")
    if conf1 is not None:
        res["config1_ptlsbench_aad"] = dict(
            sample=f"BASELINE configs[0]: 4096 x 16384 B, 32-B AAD h[4] with h[0] = seq (t/ptlsbench.c:129-141), {best_name}",
            single_core=conf1[1]["median"], all_cores=conf1[threads]["median"], all_cores_spread=conf1[threads]["spread"],
            cores=threads, unit="GiB/s seal+open")
    return res


def plugin_ptlsbench():
    """the drop-in plugin path at t/ptlsbench.c's own shape (N = 1000 records of L = 1500 B, bench_run_one
    :88-173): ptls_aead_encrypt / ptls_aead_decrypt through the reference's picotls on lib/fusion.c's
    ptls_fusion_aes128gcm and on ptls_hip_aes128gcm (one synchronous single-record launch per call)"""
    import ctypes
    import ptls_hip
    from oracle_lib import Ref, ref_ptlsbench
    if not Ref.available:
        return None
    hip = ctypes.addressof(ctypes.c_char.in_dll(ptls_hip.lib(), "ptls_hip_aes128gcm"))
    fus = Ref().algo("ptls_fusion_aes128gcm")
    ref_ptlsbench(hip, 50, 1500)  # warm-up: context creation, module load
    return {"fusion_aes128gcm": ref_ptlsbench(fus), "hip_aes128gcm": ref_ptlsbench(hip),
            "note": "Mbps as ptlsbench prints it (8 * N * L / microseconds), wall clock and process CPU time"}


def max_over_ranks(x, world):
    """the slowest rank's time: the whole job is done only when every shard is (gloo, CPU tensors: no RCCL)"""
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_ranks(vals, world):
    """every rank's list of floats (gloo all_gather of the timing summary; nothing of the data path)"""
    if world == 1:
        return [list(vals)]
    import torch
    import torch.distributed as dist
    t = torch.tensor(vals, dtype=torch.float64)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def _free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(args):
    """`bench.py --gpus N` without a launcher around it: start N rank processes (one per GPU) through
    torch.distributed.run on 127.0.0.1, BEFORE this process touches any GPU, relay their output and exit with
    their status.  Under a launcher (WORLD_SIZE set) the world size must equal --gpus."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is not None:
        if int(world_env) != args.gpus:
            sys.stderr.write(f"bench.py: WORLD_SIZE={world_env} but --gpus {args.gpus}\n")
            sys.exit(2)
        return
    if args.gpus <= 1:
        return
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd, env=env))


def golden_digests(cfg_name):
    """{record index: SHA-256 of ct || tag} that lib/fusion.c produced for the config (tests/golden/configs.json: the
    first / last 64 records of every rank's shard at up to 8 ranks)"""
    name = {"c2": "c2_tls16k_aes128", "c3": "c3_quic1350_aes128", "c4": "c4_mixed_aes256_64k", "c4s": "c4_mixed_aes256_64k",
            "c5": "c5_quic1350_aes128_8gpu"}[cfg_name]
    with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
        return {r["i"]: r["sha256"] for r in json.load(f)["configs"][name]["records"]}


def golden_positions(idx, golden):
    """positions in idx of the records that have a golden digest"""
    gi = np.array(sorted(golden), dtype=np.uint64)
    return np.nonzero(np.isin(np.asarray(idx, dtype=np.uint64), gi))[0]


def golden_check(cfg_name, idx, recs, d_ct):
    """compare sampled sealed records with the digests lib/fusion.c produced (tests/golden/configs.json)"""
    golden = golden_digests(cfg_name)
    hit = golden_positions(idx, golden)
    pos = {int(idx[p]): int(p) for p in hit}
    checked = 0
    for i, p in pos.items():
        off, L = int(recs["out_off"][p]), int(recs["len"][p])
        blob = d_ct[off:off + L + 16].cpu().numpy().tobytes()
        if hashlib.sha256(blob).hexdigest() != golden[i]:
            raise AssertionError(f"record {i}: sealed bytes differ from lib/fusion.c")
        checked += 1
    return checked


def device_copy_gbs(eng, nbytes=4 << 30, reps=5):
    """achievable HBM bandwidth in this session (report against the measured device-copy bandwidth too):
    ptls_hip_device_copy, a flat copy kernel with one 16-byte load and store per thread (the shape MI355X_MICROARCH.md
    measures 6.29 TB/s with; tools/copy_probe: 6.19 TB/s, the best of 40 shapes), of nbytes, read + write counted, HIP
    events on the launch stream, median of reps.  The torch
    uint8 copy_ this used until round 4 read ~4.9 TB/s and overstated frac_of_measured_copy; it is kept beside it."""
    import torch
    src = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    stream = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def timed(fn):
        fn()
        ts = []
        for _ in range(reps):
            ev[0].record(stream)
            fn()
            ev[1].record(stream)
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]))
        return round(2 * nbytes / (float(np.median(ts)) * 1e-3) / 1e9, 1)
    kernel = timed(lambda: eng.copy(dst, src, nbytes, stream))
    torch_copy = timed(lambda: dst.copy_(src))
    del src, dst
    return kernel, torch_copy


def lds_issue_ceiling(key_len, clock_ghz):
    """LDS ceiling of the full-block loop: per 16-B block, AES T-table lookups (ds_read_b32, 2 LDS
    cycles per wave instruction) + 16 GHASH window lookups (ds_read_b128, 4 cycles), MI355X_MICROARCH.md LDS table;
    256 CUs at the clock the launches ran at (clock_in_run) and at the 2.4 GHz max clock; plaintext GiB/s of seal."""
    rounds = 10 if key_len == 16 else 14
    lookups = 2 + 8 + 16 * (rounds - 3) + 16  # counter-mode shortcut: round 1 = 2, round 2 = 8 lookups
    cyc_per_block = (lookups * 2 + 16 * 4) / 64.0
    gib = lambda ghz: 256 * ghz * 1e9 / cyc_per_block * 16 / GIB  # noqa: E731
    return dict(aes_lookups_per_block=lookups, ghash_lookups_per_block=16, lds_cycles_per_block_per_cu=round(cyc_per_block, 3),
                clock_ghz=round(clock_ghz, 3), seal_gibps=round(gib(clock_ghz), 1), seal_gibps_at_2_4_ghz=round(gib(2.4), 1))


def host_e2e(args, cfg, eng, ks, recs, lens, d_pt, d_aad, aad_len):
    """Records start and end in pinned host memory (socket-buffer case), through ptls_hip_pipeline_seal/open, timed
    wall-clock around each whole call, for both transports: "copy" (64 MiB slices, H2D -> kernel -> D2H overlapped
    on three streams, copy engines) and "mapped" (the kernels read and write the pinned host buffers over PCIe)."""
    import torch
    import ptls_hip
    L_mean = float(lens.mean())
    n = args.e2e_records or max(1, min(len(recs), int((1 << 30) / L_mean)))
    sub = recs[:n].copy()
    in_lo, out_lo = int(sub["in_off"][0]), int(sub["out_off"][0])
    in_hi = int(sub["in_off"][-1] + sub["len"][-1] + 16)
    out_hi = int(sub["out_off"][-1] + sub["len"][-1] + 16)
    sub["in_off"] -= np.uint64(in_lo)
    sub["out_off"] -= np.uint64(out_lo)
    sub["aad_off"] = np.arange(n, dtype=np.uint64) * np.uint64(16)
    h_in = torch.empty(in_hi - in_lo, dtype=torch.uint8).pin_memory()
    h_in.copy_(d_pt[in_lo:in_hi])
    h_aad = torch.empty(n * 16, dtype=torch.uint8).pin_memory()
    h_aad.copy_(d_aad[: n * 16])
    h_ct = torch.empty(out_hi - out_lo, dtype=torch.uint8).pin_memory()
    h_pt = torch.empty(in_hi - in_lo, dtype=torch.uint8).pin_memory()
    h_res = torch.zeros(n, dtype=torch.int64).pin_memory()
    sub_o = sub.copy()
    sub_o["in_off"], sub_o["out_off"] = sub["out_off"], sub["in_off"]
    # compare record bytes only (gaps between aligned records are never written)
    edge = np.zeros(in_hi - in_lo + 1, dtype=np.int32)
    np.add.at(edge, sub["in_off"].astype(np.int64), 1)
    np.add.at(edge, (sub["in_off"] + sub["len"]).astype(np.int64), -1)
    mask = np.cumsum(edge[:-1]) > 0
    sumL = float(sub["len"].sum())
    out = dict(records=n, bytes_in=int(sumL), note="pinned host buffers; wall clock around ptls_hip_pipeline_seal/open, "
               "every byte crossing PCIe inside the timed call")
    for name, tr in (("copy", ptls_hip.TRANSPORT_COPY), ("mapped", ptls_hip.TRANSPORT_MAPPED)):
        pipe = ptls_hip.Pipeline(eng, 64 << 20, transport=tr)
        pipe.seal(ks, sub, h_in, h_aad, h_ct)  # warm-up
        ts, to = [], []
        for _ in range(3):
            h_pt.zero_()
            h_res.zero_()
            t0 = time.perf_counter()
            pipe.seal(ks, sub, h_in, h_aad, h_ct)
            ts.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            pipe.open(ks, sub_o, h_ct, h_aad, h_pt, h_res)
            to.append(time.perf_counter() - t0)
        used = pipe.last_transport
        pipe.close()
        ok = bool((h_res.numpy() == sub["len"].astype(np.int64)).all()) and \
            bool(np.array_equal(h_pt.numpy()[mask], h_in.numpy()[mask])) and used == tr
        if not ok:
            raise AssertionError(f"host-resident round trip failed ({name})")
        t_s, t_o = float(np.median(ts)), float(np.median(to))
        out[name] = dict(seal_gibps=round(sumL / t_s / GIB, 2), open_gibps=round(sumL / t_o / GIB, 2),
                         seal_open_gibps=round(2 * sumL / (t_s + t_o) / GIB, 2), roundtrip_ok=ok)
    out["copy"].update(slice_bytes=64 << 20, streams=3)
    out["seal_open_gibps"] = max(out["copy"]["seal_open_gibps"], out["mapped"]["seal_open_gibps"])
    return out


def node_e2e(args, cfg, devices):
    """The host-resident path over several devices in ONE process (ptls_hip_node_*): the config's
    records (1 GiB by default) in host memory whose per-device ranges are bound to each device's NUMA node
    (ptls_hip_node_host_alloc), byte-balanced contiguous ranges per device, one host thread per device (pinned to that
    device's node) running its zero-copy pipeline; wall clock around each node seal / open.  Whole node = payload bytes /
    the slowest device's seconds (ptls_hip_node_last_split).  Parity: every record opens to its bytes, and the sealed
    records that have a lib/fusion.c digest in tests/golden/configs.json are compared with it."""
    import torch
    import ptls_hip
    idx, recs, in_total, out_total, lens = make_workload(cfg, 0, 1, "weak", CONFIGS[args.config]["n"], args.align)
    L_mean = float(lens.mean())
    n = args.e2e_records or max(1, min(len(recs), int((1 << 30) / L_mean)))
    sub, idx, lens = recs[:n].copy(), idx[:n], lens[:n]
    in_lo, out_lo = int(sub["in_off"][0]), int(sub["out_off"][0])
    sub["in_off"] -= np.uint64(in_lo)
    sub["out_off"] -= np.uint64(out_lo)
    in_bytes = int(sub["in_off"][-1] + sub["len"][-1] + 16)
    out_bytes = int(sub["out_off"][-1] + sub["len"][-1] + 16)
    aad = build_aad(cfg, idx, lens)
    sub["aad_off"] = np.arange(n, dtype=np.uint64) * np.uint64(16)
    nd = len(devices)
    node = ptls_hip.Node(devices, cfg["key_len"], cfg["keys"], transport=ptls_hip.TRANSPORT_MAPPED)
    keys, ivs = make_keys(cfg)
    node.set_keys(0, keys, ivs)
    bounds = ptls_hip.partition_bytes(sub, nd)

    def splits(field, total):
        return [0] + [int(sub[field][bounds[d]]) if bounds[d] < n else total for d in range(1, nd)] + [total]
    h_in = node.host_alloc(in_bytes, splits("in_off", in_bytes))
    h_pt = node.host_alloc(in_bytes, splits("in_off", in_bytes))
    h_ct = node.host_alloc(out_bytes, splits("out_off", out_bytes))
    h_aad = torch.from_numpy(aad).pin_memory()
    h_res = torch.zeros(n, dtype=torch.int64).pin_memory()
    try:
        # the records' bytes: the same splitmix64 streams as the device-resident run, generated on the first device
        eng = ptls_hip.Engine(devices[0])
        gb = ptls_hip.Batch(eng, sub)
        d_buf = torch.zeros(in_bytes, dtype=torch.uint8, device=f"cuda:{devices[0]}")
        d_idx = torch.from_numpy(idx.astype(np.int64)).to(d_buf.device)
        gb.fill(d_buf, SEED_DATA, index=d_idx)
        torch.cuda.synchronize(d_buf.device)
        torch.from_numpy(h_in).copy_(d_buf.cpu())
        del d_buf, d_idx
        gb.close()
        eng.close()
        sub_o = sub.copy()
        sub_o["in_off"], sub_o["out_off"] = sub["out_off"], sub["in_off"]
        node.seal(sub, h_in, h_aad, h_ct)  # warm-up
        ts, to, dev_s, dev_o = [], [], [], []
        for _ in range(3):
            t0 = time.perf_counter()
            node.seal(sub, h_in, h_aad, h_ct)
            ts.append(time.perf_counter() - t0)
            dev_s.append(node.last_split()[0])
            h_pt[:] = 0
            h_res.zero_()
            t0 = time.perf_counter()
            node.open(sub_o, h_ct, h_aad, h_pt, h_res)
            to.append(time.perf_counter() - t0)
            dev_o.append(node.last_split()[0])
        sumL = float(lens.sum())
        edge = np.zeros(in_bytes + 1, dtype=np.int32)
        np.add.at(edge, sub["in_off"].astype(np.int64), 1)
        np.add.at(edge, (sub["in_off"] + sub["len"]).astype(np.int64), -1)
        mask = np.cumsum(edge[:-1]) > 0
        ok_open = bool((h_res.numpy() == lens.astype(np.int64)).all())
        ok_pt = bool(np.array_equal(h_pt[mask], h_in[mask]))
        d_ct = torch.from_numpy(h_ct).to("cuda")
        golden_n = golden_check(args.config, idx, sub, d_ct)
        del d_ct
        if not (ok_open and ok_pt):
            raise AssertionError(f"node host-resident round trip failed (status ok={ok_open}, bytes ok={ok_pt})")
        numa = node.numa_nodes()
        placement = []
        sp_in = splits("in_off", in_bytes)
        for d in range(nd):
            pages = ptls_hip.page_nodes(h_in[sp_in[d]:sp_in[d + 1]], stride=16)
            placement.append(round(float((pages == numa[d]).mean()), 3) if numa[d] >= 0 and len(pages) else None)
        t_s, t_o = float(np.median(ts)), float(np.median(to))
        per_dev = []
        for d in range(nd):
            share = float(lens[bounds[d]:bounds[d + 1]].sum())
            s_d = float(np.median([x[d] for x in dev_s]))
            o_d = float(np.median([x[d] for x in dev_o]))
            per_dev.append(dict(device=devices[d], numa_node=numa[d], records=[bounds[d], bounds[d + 1]], payload_bytes=int(share),
                                seal_s=round(s_d, 4), open_s=round(o_d, 4),
                                seal_open_gibps=round(2 * share / (s_d + o_d) / GIB, 2) if s_d + o_d > 0 else None,
                                input_pages_on_its_node=placement[d]))
        return dict(devices=devices, records=n, payload_bytes=int(sumL), transport="mapped (zero-copy)",
                    seal_gibps=round(sumL / t_s / GIB, 2), open_gibps=round(sumL / t_o / GIB, 2),
                    seal_open_gibps=round(2 * sumL / (t_s + t_o) / GIB, 2),
                    whole_node_from_slowest_device_gibps=round(2 * sumL / (max(float(np.median([max(x) for x in dev_s])), 1e-9) +
                                                                           max(float(np.median([max(x) for x in dev_o])), 1e-9)) / GIB, 2),
                    per_device=per_dev, numa_nodes=numa,
                    parity=dict(open_all_ok=ok_open, roundtrip_bytes_equal=ok_pt, golden_records_checked=golden_n),
                    note="host buffers from ptls_hip_node_host_alloc: each device's range bound to its NUMA node; "
                         "wall clock around ptls_hip_node_seal / open, every byte crossing PCIe inside the timed call")
    finally:
        for a in (h_in, h_pt, h_ct):
            ptls_hip.Node.host_free(a)
        node.close()


def report_ranks(result, per_rank, world, steps, elapsed):
    """per-rank and whole-node rates from every rank's [seconds, plaintext bytes per step, seal ms, open ms, first record,
    end record, golden records checked]: whole node = sum of all ranks' bytes / the slowest rank's time"""
    total_bytes = sum(r[1] for r in per_rank) * 2 * steps  # seal + open each pass over the plaintext
    result["value"] = round(total_bytes / elapsed / GIB, 2)
    result["per_rank"] = [{"rank": i, "gibps": round(2 * r[1] * steps / r[0] / GIB, 2), "seconds": round(r[0], 4),
                           "seal_gibps": round(r[1] / (r[2] * 1e-3) / GIB, 2) if r[2] > 0 else None,
                           "open_gibps": round(r[1] / (r[3] * 1e-3) / GIB, 2) if r[3] > 0 else None,
                           "records": [int(r[4]), int(r[5])], "payload_bytes": int(r[1]), "golden_records_checked": int(r[6])}
                          for i, r in enumerate(per_rank)]
    result["whole_node_gibps"] = result["value"]


def dry_run(args, cfg, world, rank):
    """CPU rehearsal of the multi-rank path (tests/test_multirank.py): the same launcher, barriers, max-over-ranks
    and per-rank gather over gloo, with a sleep standing in for the GPU work"""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    lo, hi = rank_range(cfg, rank, world, args.scaling, CONFIGS[args.config]["n"])
    idx, recs, in_total, out_total, lens = make_workload(cfg, rank, world, args.scaling, CONFIGS[args.config]["n"], args.align)
    sum_L = int(lens.sum())
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.02 * (rank + 1))
    mine = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(mine, world)
    golden_here = len(golden_positions(idx, golden_digests(args.config)))  # what the GPU run would check on this rank
    per_rank = gather_ranks([mine, float(sum_L), 0.0, 0.0, float(lo), float(hi), float(golden_here)], world)
    result = {"metric": "dry run (no GPU)", "value": None, "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
              "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "dry_run": True,
              "records_per_rank": len(recs), "first_index_per_rank": gather_ranks([float(idx[0]) if len(idx) else -1.0], world),
              "scaling": args.scaling}
    report_ranks(result, per_rank, world, args.steps, elapsed)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=list(CONFIGS))
    ap.add_argument("--lanes", type=int, default=0)
    ap.add_argument("--align", type=int, default=0, choices=[0, 16, 32, 64, 128, 256],
                    help="byte alignment of every record's input and output (default 128, or PTLS_BENCH_ALIGN); 16 packs "
                         "them back to back")
    ap.add_argument("--records", type=int, default=0, help="override records per GPU (smaller runs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-mib", type=int, default=1024, help="records in the CPU baseline's sample (default 1 GiB)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-resident (pinned H2D/D2H) measurement")
    ap.add_argument("--no-plugin", action="store_true", help="skip the ptlsbench-shape plugin timing")
    ap.add_argument("--e2e-records", type=int, default=0, help="records in the host-resident sample (default: 1 GiB)")
    ap.add_argument("--device", type=int, default=-1,
                    help="every rank on this device (default: LOCAL_RANK); rehearses N ranks on a one-GPU box")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: every rank its own shard of the config's size; strong: one batch split by bytes")
    ap.add_argument("--node-e2e", default="",
                    help="only the host-resident path over these devices in one process (ptls_hip_node_*), e.g. 0,1,2,3; "
                         "a device may repeat (one-GPU rehearsal: 0,0)")
    ap.add_argument("--dry-run", action="store_true", help=argparse.SUPPRESS)  # CPU rehearsal of the rank logic (tests)
    args = ap.parse_args()
    launch_ranks(args)  # N > 1 without a launcher: re-run as N ranks, before any GPU call

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cfg = dict(CONFIGS[args.config])
    if args.records:
        cfg["n"] = args.records
    if args.dry_run:
        return dry_run(args, cfg, world, rank)

    import torch
    import torch.distributed as dist
    import ptls_hip
    if args.node_e2e:
        devices = [int(x) for x in args.node_e2e.split(",")]
        res = {"metric": "GiB/s AES-GCM seal+open, host-resident, one process over a node's GPUs (ptls_hip_node_*)",
               "config": {"workload": cfg["desc"], "key_bits": cfg["key_len"] * 8}, "unit": "GiB/s"}
        res.update(node_e2e(args, cfg, devices))
        res["value"] = res["seal_open_gibps"]
        print(json.dumps(res), flush=True)
        return
    dev = local if args.device < 0 else args.device
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("gloo")  # CPU-side coordination only: barriers and the timing summary

    eng = ptls_hip.Engine(dev)
    lo, hi = rank_range(cfg, rank, world, args.scaling, CONFIGS[args.config]["n"])
    idx, recs, in_total, out_total, lens = make_workload(cfg, rank, world, args.scaling, CONFIGS[args.config]["n"], args.align)
    n = len(recs)
    sum_L = int(lens.sum())
    aad = build_aad(cfg, idx, lens)
    aad_len = 5 if cfg["aad"] == "tls" else 13

    keys, ivs = make_keys(cfg)
    ks = ptls_hip.KeySet(eng, cfg["key_len"], cfg["keys"])
    t0 = time.time()
    ks.set(0, keys, ivs)
    setup_s = time.time() - t0
    secrets_s = None
    if cfg["keys"] > 1:
        # the same number of connections keyed from TLS 1.3 traffic secrets on the GPU
        hs = 48 if cfg["key_len"] == 32 else 32
        ks2 = ptls_hip.KeySet(eng, cfg["key_len"], cfg["keys"])
        sec = np.random.default_rng(1).integers(0, 256, cfg["keys"] * hs, dtype=np.uint8).tobytes()
        ks2.set_secrets(0, sec, hs)  # warm-up (module load)
        t0 = time.time()
        ks2.set_secrets(0, sec, hs)
        secrets_s = time.time() - t0
        ks2.close()

    seal_b = ptls_hip.Batch(eng, recs)
    if args.lanes:
        seal_b.set_lanes(args.lanes)
    recs_o = recs.copy()
    recs_o["in_off"], recs_o["out_off"] = recs["out_off"], recs["in_off"]
    open_b = ptls_hip.Batch(eng, recs_o)
    open_b.set_lanes(seal_b.lanes)

    d_pt = torch.empty(in_total + 64, dtype=torch.uint8, device="cuda")
    d_ct = torch.empty(out_total + 64, dtype=torch.uint8, device="cuda")
    d_out = torch.empty(in_total + 64, dtype=torch.uint8, device="cuda")
    d_aad = torch.from_numpy(aad).cuda()
    d_res = torch.zeros(n, dtype=torch.int64, device="cuda")
    # payload of record i = splitmix64 stream of SEED_DATA ^ i (same bytes the CPU side generates)
    d_idx = torch.from_numpy(idx.astype(np.int64)).cuda()
    seal_b.fill(d_pt, SEED_DATA, index=d_idx)
    torch.cuda.synchronize()
    del d_idx

    stream = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]

    def step(times=None):
        ev[0].record(stream)
        seal_b.seal(ks, d_pt, d_aad, d_ct, stream)
        ev[1].record(stream)
        open_b.open(ks, d_ct, d_aad, d_out, d_res, stream)
        ev[2].record(stream)
        if times is not None:
            torch.cuda.synchronize()
            times.append((ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    mine = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = max_over_ranks(time.perf_counter() - t0, world)

    # per-kernel timing (HIP events on the launch stream) and the clock of those same launches, outside the timed
    # region: the kernels' diagnostic stamps (ptls_hip_batch_set_clock) give delta(shader cycles) / delta(100 MHz
    # ticks) per workgroup, so the clock the reported kernel time was measured at is part of this run's record
    clk_s = torch.zeros(4 * seal_b.grid, dtype=torch.int64, device="cuda")
    clk_o = torch.zeros(4 * open_b.grid, dtype=torch.int64, device="cuda")
    seal_b.set_clock(clk_s)
    open_b.set_clock(clk_o)
    ktimes, kclk, kdet = [], [], []
    for _ in range(max(2, min(args.steps, 5))):
        step(ktimes)
        kclk.append((ptls_hip.clock_of(clk_s.cpu().numpy().view(np.uint64), seal_b.grid),
                     ptls_hip.clock_of(clk_o.cpu().numpy().view(np.uint64), open_b.grid)))
        kdet.append(ptls_hip.clock_detail(clk_s.cpu().numpy().view(np.uint64), seal_b.grid))
    seal_b.set_clock(None)
    open_b.set_clock(None)
    seal_ms = float(np.median([a for a, _ in ktimes]))
    open_ms = float(np.median([b for _, b in ktimes]))
    seal_ghz = float(np.median([c[0][0] for c in kclk]))
    open_ghz = float(np.median([c[1][0] for c in kclk]))
    timed_seal_open_ms = elapsed / args.steps * 1e3

    # parity: every record opens to its length and original bytes; sampled records == lib/fusion.c, on every rank
    ok_open = bool((d_res == torch.tensor(lens.astype(np.int64), device="cuda")).all())
    ok_pt = bool(torch.equal(d_out[:in_total], d_pt[:in_total]))
    golden_n = golden_check(args.config, idx, recs, d_ct)
    if not (ok_open and ok_pt):
        raise AssertionError(f"rank {rank}: open round trip failed (status ok={ok_open}, bytes ok={ok_pt})")
    per_rank = gather_ranks([mine, float(sum_L), seal_ms, open_ms, float(lo), float(hi), float(golden_n), seal_ghz], world)

    alg_bytes = int(2 * sum_L + n * (aad_len + 16))  # 2L + A + 16 per record, per launch
    achieved = alg_bytes / (seal_ms * 1e-3) / 1e9
    batch_kernel = seal_b.lanes != 64

    result = {
        "metric": "GiB/s AES-128-GCM seal+open, device-resident, 16KiB records, 1/2/4/8 GPU"
        if args.config == "c2" else f"GiB/s AES-GCM seal+open, device-resident ({args.config})",
        "value": None,
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 records, SURVEY.md §8(d)), generated in HBM",
        "config": {"workload": cfg["desc"], "records_per_gpu": n, "record_bytes": cfg["L"] or "mixed 64-16384",
                   "aad_bytes": aad_len, "keys": cfg["keys"], "key_bits": cfg["key_len"] * 8,
                   "lanes_per_record": seal_b.lanes, "record_align": record_align(args.align),
                   "parallelism": (f"records sharded by range over {world} GPU(s), no collective" if args.scaling == "weak" else
                                   f"one batch of {cfg['n']} records split over {world} GPU(s) in byte-balanced contiguous "
                                   f"ranges, no collective")},
        "seal_gibps": round(sum(r[1] / (r[2] * 1e-3) for r in per_rank) / GIB, 2),
        "open_gibps": round(sum(r[1] / (r[3] * 1e-3) for r in per_rank) / GIB, 2),
        "seal_ms": round(seal_ms, 3),
        "open_ms": round(open_ms, 3),
        "clock_in_run": {"seal_ghz": round(seal_ghz, 3), "open_ghz": round(open_ghz, 3),
                         "seal_ghz_min_max_over_workgroups": [round(min(c[0][1] for c in kclk), 3),
                                                              round(max(c[0][2] for c in kclk), 3)],
                         "seal_span_ms_100mhz": round(float(np.median([c[0][3] for c in kclk])), 3),
                         # how the seal launches ended across workgroups: (last end - median end) / span, median of the
                         # stamped launches, and the median launch's per-XCD clock and end time
                         "seal_finish_spread": round(float(np.median([d["finish_spread"] for d in kdet])), 4),
                         "seal_finish_spread_first_to_last": round(float(np.median([d["finish_spread_min_to_max"]
                                                                                   for d in kdet])), 4),
                         "seal_per_xcd": sorted(kdet, key=lambda d: d["span_ms"])[len(kdet) // 2]["per_xcd"],
                         "seal_mcycles_per_launch": round(seal_ghz * seal_ms, 2),
                         "cycles_note": "clock x kernel time = the launch's length in shader cycles: the work measure that does "
                                        "not move with the box's clock (MI355X_MICROARCH.md DVFS)",
                         "stamped_seal_open_ms": round(seal_ms + open_ms, 3),
                         "timed_loop_seal_open_ms": round(timed_seal_open_ms, 3),
                         "source": "s_memtime / s_memrealtime at each workgroup's start and end, in the launches "
                                   "seal_ms / open_ms were timed on (not in the timed loop)"},
        "key_setup_s": round(setup_s, 4),
        "key_setup_from_secrets_s": None if secrets_s is None else round(secrets_s, 4),
        "roofline": {"bound": "lds" if batch_kernel else "latency", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "frac_note": "achieved HBM bytes / the 8 TB/s HBM peak (the contract's roofline); the unit that binds "
                                  "is named in 'bound' (DESIGN.md §4.1: the batch kernel's T-table and GHASH lookups keep "
                                  "the LDS array busy; the sparse kernel is latency-bound, §4.8)",
                     "kernel": ("aesgcm_sparse_kernel (seal)" if not batch_kernel else "aesgcm_batch_kernel (seal)"),
                     "algorithmic_bytes_per_launch": alg_bytes},
        "parity": {"open_all_ok": ok_open, "roundtrip_bytes_equal": ok_pt, "golden_records_checked": int(sum(r[6] for r in per_rank)),
                   "golden_records_checked_per_rank": [int(r[6]) for r in per_rank]},
    }
    report_ranks(result, per_rank, world, args.steps, elapsed)
    copy_gbs, torch_copy_gbs = device_copy_gbs(eng)
    result["roofline"]["measured_copy_gbs"] = copy_gbs
    result["roofline"]["measured_copy_source"] = ("ptls_hip_device_copy: one 16-B load + store per thread, 4 GiB, read + "
                                                  "write counted, HIP events, median of 5")
    result["roofline"]["torch_uint8_copy_gbs"] = torch_copy_gbs
    result["roofline"]["frac_of_measured_copy"] = round(achieved / copy_gbs, 4)
    if batch_kernel:  # the batch kernel's LDS model (the sparse-key kernel is latency-bound)
        ceil = lds_issue_ceiling(cfg["key_len"], seal_ghz)
        ceil["frac"] = round(seal_ms and (sum_L / (seal_ms * 1e-3) / GIB) / ceil["seal_gibps"], 4)
        result["roofline"]["lds_issue_ceiling"] = ceil
    if not args.no_e2e and world == 1:  # PCIe path is per GPU; at N > 1 the ranks would share the host links
        result["host_e2e"] = host_e2e(args, cfg, eng, ks, recs, lens, d_pt, d_aad, aad_len)
    tfile = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tfile):
        with open(tfile) as f:
            tr = json.load(f)
        result["roofline"]["traffic"] = tr.get("hbm_bytes_per_seal_launch")
        result["roofline"]["traffic_source"] = os.path.relpath(tfile, ROOT)
    lfile = os.path.join(ROOT, "profiles", f"lds_{args.config}.json")
    if os.path.exists(lfile) and "lds_issue_ceiling" in result["roofline"]:  # LDS-array occupancy of the same kernel from its PMC pass (the bound that binds)
        with open(lfile) as f:
            lj = json.load(f)
        ceil = result["roofline"]["lds_issue_ceiling"]
        ceil["lds_array_busy_measured"] = lj["lds_array_busy_frac"]
        ceil["lds_array_busy_source"] = os.path.relpath(lfile, ROOT) + " (PMC pass of the same kernel, another run)"
        if "valu_issue_busy_frac" in lj:  # the other issue port of the same loop
            ceil["valu_issue_busy_measured"] = lj["valu_issue_busy_frac"]
    for o in (seal_b, open_b):
        o.close()
    del d_pt, d_ct, d_out, d_aad, d_res, clk_s, clk_o
    if not args.no_e2e and world > 1:
        # the host-resident figure for the whole node: ONE process (rank 0) drives every rank's device through the node
        # API, each device's records in host memory on its own NUMA node; the other ranks wait (their GPUs idle)
        torch.cuda.empty_cache()
        devs = [int(r[0]) for r in gather_ranks([float(dev)], world)]
        dist.barrier()
        if rank == 0:
            result["host_e2e_node"] = node_e2e(args, cfg, devs)
        dist.barrier()
    if rank == 0 and world == 1 and not args.no_plugin:
        result["plugin_ptlsbench"] = plugin_ptlsbench()
    if not args.no_cpu_baseline:
        # on rank 0 with every GPU idle: at N > 1 the other ranks wait at the barrier (an N > 1 line carries
        # its own CPU baseline)
        if world > 1:
            dist.barrier()
        if rank == 0:
            result["cpu_baseline"] = cpu_baseline(args.config, cfg, dev, args.cpu_sample_mib << 20)
        if world > 1:
            dist.barrier()
    if rank == 0:
        print(json.dumps(result), flush=True)
    for o in (ks, eng):
        o.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
