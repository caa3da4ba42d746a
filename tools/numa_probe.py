#!/usr/bin/env python3
"""Host NUMA placement for the host-resident path ("pin host buffers on the GPU's local NUMA node").

Prints the box's NUMA topology (nodes, their CPUs, this process's affinity, the GPU's node from sysfs), then for
each NUMA node: 1 GiB of c2-shaped records in host memory BOUND to that node (mmap + mbind(MPOL_BIND), pages
touched, verified with move_pages, then hipHostRegister'ed), sealed and opened by the batch kernel in place over
PCIe (zero-copy, as the MAPPED pipeline transport does), and plain SDMA H2D / D2H copies from the same buffers.
Also the default allocation (torch pin_memory / hipHostMalloc: first touch by this thread) for comparison.
Timing only; prints one JSON line."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hsig-picotls_amd"))

import torch  # noqa: E402  (torch's HIP runtime first)
assert torch.cuda.is_available()
import bench  # noqa: E402
import ptls_hip  # noqa: E402

GIB = float(1 << 30)
libc = ctypes.CDLL(None, use_errno=True)
libc.syscall.restype = ctypes.c_long
libc.mmap.restype = ctypes.c_void_p
libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
SYS_mbind, SYS_move_pages = 237, 279
hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
hip.hipDeviceGetPCIBusId.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int]


def read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def topology():
    nodes = []
    online = read("/sys/devices/system/node/online") or ""
    for part in online.split(","):
        if "-" in part:
            a, b = part.split("-")
            nodes += list(range(int(a), int(b) + 1))
        elif part:
            nodes.append(int(part))
    buf = ctypes.create_string_buffer(64)
    bus = None
    if hip.hipDeviceGetPCIBusId(buf, 64, 0) == 0:
        bus = buf.value.decode().lower()
    gpu_node = read(f"/sys/bus/pci/devices/{bus}/numa_node") if bus else None
    aff = sorted(os.sched_getaffinity(0))
    per = {}
    for n in nodes:
        cl = read(f"/sys/devices/system/node/node{n}/cpulist")
        per[n] = cl
    return dict(nodes=nodes, node_cpus=per, gpu_pci=bus, gpu_numa_node=None if gpu_node is None else int(gpu_node),
                affinity_count=len(aff), affinity_first=aff[:4], affinity_last=aff[-4:])


def bound_alloc(nbytes, node):
    """mmap + mbind(MPOL_BIND, node) + touch; returns (ptr, nodes of sampled pages) or raises"""
    PROT_RW, MAP_PRIV_ANON = 0x3, 0x22
    p = libc.mmap(None, nbytes, PROT_RW, MAP_PRIV_ANON, -1, 0)
    assert p not in (None, ctypes.c_void_p(-1).value), "mmap"
    if node is not None:
        mask = (ctypes.c_ulong * 16)()
        mask[node // 64] = 1 << (node % 64)
        r = libc.syscall(SYS_mbind, ctypes.c_void_p(p), ctypes.c_size_t(nbytes), 2, mask, ctypes.c_ulong(1024), 0)
        if r != 0:
            e = ctypes.get_errno()
            libc.munmap(p, nbytes)
            raise OSError(e, f"mbind to node {node} failed: {os.strerror(e)}")
    ctypes.memset(p, 0, nbytes)  # first touch under the policy
    k = 8
    pages = (ctypes.c_void_p * k)(*[p + i * (nbytes // k) for i in range(k)])
    status = (ctypes.c_int * k)()
    libc.syscall(SYS_move_pages, 0, ctypes.c_ulong(k), pages, None, status, 0)
    return p, sorted(set(status))


def main():
    topo = topology()
    out = {"topology": topo}
    cfg = dict(bench.CONFIGS["c2"])
    cfg["n"] = 65536  # 1 GiB of 16 KiB records
    eng = ptls_hip.Engine(0)
    idx, recs, in_total, out_total, lens = bench.make_workload(cfg, 0)
    sum_L = float(lens.sum())
    keys, ivs = bench.make_keys(cfg)
    ks = ptls_hip.KeySet(eng, cfg["key_len"], cfg["keys"])
    ks.set(0, keys, ivs)
    seal_b = ptls_hip.Batch(eng, recs)
    seal_b.set_lanes(64)  # the mapped transport's choice for records of >= 64 GHASH elements
    ro = recs.copy()
    ro["in_off"], ro["out_off"] = recs["out_off"], recs["in_off"]
    open_b = ptls_hip.Batch(eng, ro)
    open_b.set_lanes(64)
    aad = torch.from_numpy(bench.build_aad(cfg, idx, lens)).cuda()
    res = torch.zeros(cfg["n"], dtype=torch.int64, device="cuda")
    d_in = torch.zeros(in_total + 64, dtype=torch.uint8, device="cuda")
    seal_b.fill(d_in, bench.SEED_DATA)
    torch.cuda.synchronize()
    nb_in, nb_out = in_total + 64, out_total + 64

    def timed(f, reps=3):
        f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            f()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    def run(label, node):
        try:
            bufs = [bound_alloc(n, node) for n in (nb_in, nb_out, nb_in)]
        except (OSError, AssertionError) as e:
            out[label] = {"error": str(e)}
            return
        ptrs = [b[0] for b in bufs]
        devs = []
        for p, n in zip(ptrs, (nb_in, nb_out, nb_in)):
            assert hip.hipHostRegister(p, n, 0) == 0, "hipHostRegister"
            d = ctypes.c_void_p()
            assert hip.hipHostGetDevicePointer(ctypes.byref(d), p, 0) == 0
            devs.append(d.value)
        assert hip.hipMemcpy(ptrs[0], d_in.data_ptr(), in_total, 2) == 0
        t_s = timed(lambda: seal_b.seal(ks, devs[0], aad, devs[1]))
        t_o = timed(lambda: open_b.open(ks, devs[1], aad, devs[2], res))
        ok = bool((res == torch.from_numpy(lens.astype(np.int64)).cuda()).all())
        h2d = timed(lambda: hip.hipMemcpy(d_in.data_ptr(), ptrs[0], in_total, 1))
        d2h = timed(lambda: hip.hipMemcpy(ptrs[2], d_in.data_ptr(), in_total, 2))
        out[label] = {"page_nodes": bufs[0][1], "seal_gibps": round(sum_L / t_s / GIB, 2), "open_gibps": round(sum_L / t_o / GIB, 2),
                      "seal_open_gibps": round(2 * sum_L / (t_s + t_o) / GIB, 2), "open_all_ok": ok,
                      "sdma_h2d_gbs": round(in_total / h2d / 1e9, 1), "sdma_d2h_gbs": round(in_total / d2h / 1e9, 1)}
        for p, n in zip(ptrs, (nb_in, nb_out, nb_in)):
            hip.hipHostUnregister(p)
            libc.munmap(p, n)
        print(label, out[label], flush=True)

    run("first_touch", None)
    for n in topo["nodes"]:
        run(f"node{n}", n)
    print(json.dumps(out), flush=True)
    for o in (seal_b, open_b, ks, eng):
        o.close()


if __name__ == "__main__":
    main()
