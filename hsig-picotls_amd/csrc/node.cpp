/*
 * node.cpp -- one batch over several devices: contiguous record ranges of equal payload bytes, one host
 * thread and one pipeline per device, host buffers bound to each device's NUMA node.  No collective: records are
 * independent.
 */
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <thread>

#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "host.h"
/* ---------------------------------------------------------------------------------------------- */
/* one batch over several devices                                                 */
/* ---------------------------------------------------------------------------------------------- */

extern "C" int ptls_hip_partition_bytes(const ptls_hip_record_t *recs, size_t n, size_t parts, size_t *bounds)
{
    if ((recs == nullptr && n != 0) || parts == 0 || bounds == nullptr)
        return fail(PTLS_HIP_EINVAL, "partition_bytes: bad arguments");
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i)
        total += recs[i].len;
    /* range r ends right after the first record whose prefix sum reaches ceil(total * (r + 1) / parts) (bench.py
     * partition_bytes is the same rule) */
    bounds[0] = 0;
    size_t i = 0;
    uint64_t csum = 0;
    for (size_t r = 1; r < parts; ++r) {
        const unsigned __int128 t = ((unsigned __int128)total * r + parts - 1) / parts;
        const uint64_t target = (uint64_t)t;
        if (total == 0) {
            bounds[r] = 0;
            continue;
        }
        while (i < n && csum < target)
            csum += recs[i++].len;
        bounds[r] = std::max(bounds[r - 1], i);
    }
    bounds[parts] = n;
    return 0;
}

struct st_ptls_hip_node_t {
    std::vector<ptls_hip_engine_t *> eng;
    std::vector<ptls_hip_keyset_t *> ks;
    std::vector<ptls_hip_pipeline_t *> pipe;
    std::vector<int> numa;       /* each device's NUMA node (-1: unknown) */
    std::vector<double> seconds; /* per device, last call */
    std::vector<size_t> bounds;  /* record ranges of the last call */
};

/* ---- NUMA placement (host buffers on each GPU's local node) ---- */

static std::vector<int> parse_cpulist(const char *text)
{
    std::vector<int> out;
    const char *p = text;
    while (*p != '\0' && *p != '\n') {
        char *end = nullptr;
        const long a = strtol(p, &end, 10);
        if (end == p)
            break;
        long b = a;
        p = end;
        if (*p == '-') {
            b = strtol(p + 1, &end, 10);
            p = end;
        }
        for (long c = a; c <= b; ++c)
            out.push_back((int)c);
        if (*p == ',')
            ++p;
    }
    return out;
}

static std::string read_small_file(const std::string &path)
{
    FILE *f = fopen(path.c_str(), "r");
    if (f == nullptr)
        return std::string();
    char buf[4096];
    const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
    fclose(f);
    buf[n] = '\0';
    return std::string(buf);
}

extern "C" int ptls_hip_device_numa_node(int device)
{
    char bdf[64] = {0};
    if (hipDeviceGetPCIBusId(bdf, sizeof(bdf), device) != hipSuccess)
        return -1;
    for (char *c = bdf; *c != '\0'; ++c)
        *c = (char)tolower(*c);
    const std::string v = read_small_file(std::string("/sys/bus/pci/devices/") + bdf + "/numa_node");
    return v.empty() ? -1 : atoi(v.c_str());
}

/* the CPUs of NUMA node `node` this process may run on (empty: unknown node, or none allowed) */
static std::vector<int> node_cpus(int node)
{
    std::vector<int> out;
    if (node < 0)
        return out;
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0)
        return out;
    for (int c : parse_cpulist(read_small_file("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist").c_str()))
        if (c >= 0 && c < CPU_SETSIZE && CPU_ISSET(c, &allowed))
            out.push_back(c);
    return out;
}

/* the calling thread runs on `node`'s CPUs (when it has any this process may use) */
static void pin_thread_to_node(int node)
{
    const std::vector<int> cpus = node_cpus(node);
    if (cpus.empty())
        return;
    cpu_set_t s;
    CPU_ZERO(&s);
    for (int c : cpus)
        CPU_SET(c, &s);
    (void)pthread_setaffinity_np(pthread_self(), sizeof(s), &s);
}

static long sys_mbind(void *addr, unsigned long len, int mode, const unsigned long *mask, unsigned long maxnode, unsigned flags)
{
    return syscall(SYS_mbind, addr, len, mode, mask, maxnode, flags);
}

extern "C" void ptls_hip_node_free(ptls_hip_node_t *node)
{
    if (node == nullptr)
        return;
    for (auto *p : node->pipe)
        ptls_hip_pipeline_free(p);
    for (auto *k : node->ks)
        ptls_hip_keyset_free(k);
    for (auto *e : node->eng)
        ptls_hip_engine_free(e);
    delete node;
}

extern "C" ptls_hip_node_t *ptls_hip_node_new(const int *devices, size_t ndev, size_t key_size, size_t nslots, size_t slice_bytes)
{
    if (devices == nullptr || ndev == 0 || ndev > 64) {
        fail(PTLS_HIP_EINVAL, "node_new: 1 to 64 devices");
        return nullptr;
    }
    auto *node = new st_ptls_hip_node_t();
    for (size_t d = 0; d < ndev; ++d) {
        ptls_hip_engine_t *e = ptls_hip_engine_new(devices[d]);
        node->eng.push_back(e);
        ptls_hip_keyset_t *k = e != nullptr ? ptls_hip_keyset_new(e, key_size, nslots) : nullptr;
        node->ks.push_back(k);
        ptls_hip_pipeline_t *p = k != nullptr ? ptls_hip_pipeline_new(e, slice_bytes) : nullptr;
        node->pipe.push_back(p);
        if (p == nullptr) {
            const std::string why = g_err;
            ptls_hip_node_free(node);
            fail(PTLS_HIP_ENODEV, "node_new: device %d: %s", devices[d], why.c_str());
            return nullptr;
        }
    }
    for (size_t d = 0; d < ndev; ++d)
        node->numa.push_back(ptls_hip_device_numa_node(devices[d]));
    node->seconds.assign(ndev, 0.0);
    node->bounds.assign(ndev + 1, 0);
    return node;
}

extern "C" int ptls_hip_node_numa(ptls_hip_node_t *node, int *numa_nodes)
{
    if (node == nullptr || numa_nodes == nullptr)
        return fail(PTLS_HIP_EINVAL, "node_numa: bad arguments");
    std::copy(node->numa.begin(), node->numa.end(), numa_nodes);
    return 0;
}

/* Host memory for a node's records: `bytes` of anonymous memory whose byte range [splits[d], splits[d + 1]) is bound
 * (mbind MPOL_BIND) to device d's NUMA node and faulted in there, then registered with every device (hipHostRegister,
 * mapped + portable) so either transport can use it.  A device whose node is unknown leaves its range to first touch. */
extern "C" void *ptls_hip_node_host_alloc(ptls_hip_node_t *node, size_t bytes, const size_t *splits)
{
    if (node == nullptr || bytes == 0 || splits == nullptr || splits[0] != 0 || splits[node->eng.size()] != bytes) {
        fail(PTLS_HIP_EINVAL, "node_host_alloc: splits must run from 0 to bytes, one range per device");
        return nullptr;
    }
    const size_t pg = (size_t)sysconf(_SC_PAGESIZE), len = (bytes + pg - 1) / pg * pg;
    void *p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) {
        fail(PTLS_HIP_ENOMEM, "node_host_alloc: mmap of %zu bytes failed", bytes);
        return nullptr;
    }
    uint8_t *base = static_cast<uint8_t *>(p);
    for (size_t d = 0; d < node->eng.size(); ++d) {
        if (splits[d + 1] < splits[d]) {
            munmap(p, len);
            fail(PTLS_HIP_EINVAL, "node_host_alloc: splits must not decrease");
            return nullptr;
        }
        /* whole pages: a page shared by two ranges goes with the first */
        const size_t lo = (splits[d] + pg - 1) / pg * pg, hi = d + 1 == node->eng.size() ? len : (splits[d + 1] + pg - 1) / pg * pg;
        const int nd = node->numa[d];
        if (hi > lo && nd >= 0 && nd < 1024) {
            unsigned long mask[1024 / (8 * sizeof(unsigned long))] = {0};
            mask[nd / (8 * sizeof(unsigned long))] |= 1ul << (nd % (8 * sizeof(unsigned long)));
            (void)sys_mbind(base + lo, hi - lo, 2 /* MPOL_BIND */, mask, 1024 + 1, 0);
        }
        if (hi > lo)
            std::memset(base + lo, 0, hi - lo); /* fault the pages in on their node */
    }
    if (hipHostRegister(p, len, hipHostRegisterMapped | hipHostRegisterPortable) != hipSuccess) {
        munmap(p, len);
        fail(PTLS_HIP_ENOMEM, "node_host_alloc: hipHostRegister failed");
        return nullptr;
    }
    return p;
}

extern "C" void ptls_hip_node_host_free(void *ptr, size_t bytes)
{
    if (ptr == nullptr)
        return;
    const size_t pg = (size_t)sysconf(_SC_PAGESIZE), len = (bytes + pg - 1) / pg * pg;
    (void)hipHostUnregister(ptr);
    munmap(ptr, len);
}

/* the NUMA node of every `stride`-th page of [ptr, ptr + bytes) (move_pages query), written to nodes (-errno for a page
 * not present); returns the number of pages written */
extern "C" size_t ptls_hip_host_page_nodes(const void *ptr, size_t bytes, size_t stride, int *nodes, size_t cap)
{
    const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
    std::vector<void *> pages;
    for (size_t off = 0; off < bytes && pages.size() < cap; off += pg * (stride ? stride : 1))
        pages.push_back(const_cast<uint8_t *>(static_cast<const uint8_t *>(ptr)) + off);
    if (pages.empty())
        return 0;
    if (syscall(SYS_move_pages, 0, pages.size(), pages.data(), nullptr, nodes, 0) != 0)
        return 0;
    return pages.size();
}

extern "C" size_t ptls_hip_node_size(ptls_hip_node_t *node)
{
    return node != nullptr ? node->eng.size() : 0;
}

extern "C" int ptls_hip_node_keyset_set(ptls_hip_node_t *node, size_t first, size_t count, const void *keys, const void *ivs)
{
    if (node == nullptr)
        return fail(PTLS_HIP_EINVAL, "node_keyset_set: null node");
    for (auto *k : node->ks) /* replicated: every device holds every connection's key slot */
        if (int rc = ptls_hip_keyset_set(k, first, count, keys, ivs, nullptr))
            return rc;
    return 0;
}

extern "C" int ptls_hip_node_set_transport(ptls_hip_node_t *node, int transport)
{
    if (node == nullptr)
        return fail(PTLS_HIP_EINVAL, "node_set_transport: null node");
    for (auto *p : node->pipe)
        if (int rc = ptls_hip_pipeline_set_transport(p, transport))
            return rc;
    return 0;
}

/* the records split in contiguous ranges of about equal payload bytes, one host thread per device driving its own
 * pipeline over its range (the host buffers are shared: offsets stay relative to them), no data crossing devices */
static int node_run(ptls_hip_node_t *node, const ptls_hip_record_t *recs, size_t n, const void *h_in, const void *h_aad,
                    void *h_out, uint64_t *h_result, bool open)
{
    if (node == nullptr || (n != 0 && (recs == nullptr || h_in == nullptr || h_out == nullptr)) || (open && h_result == nullptr))
        return fail(PTLS_HIP_EINVAL, "node seal/open: bad arguments");
    const size_t nd = node->eng.size();
    if (int rc = ptls_hip_partition_bytes(recs, n, nd, node->bounds.data()))
        return rc;
    std::vector<int> rcs(nd, 0);
    std::vector<std::string> errs(nd);
    std::vector<std::thread> th;
    for (size_t d = 0; d < nd; ++d) {
        th.emplace_back([&, d]() {
            pin_thread_to_node(node->numa[d]); /* the device's host thread plans and stages on the device's own node */
            const size_t lo = node->bounds[d], hi = node->bounds[d + 1];
            const auto t0 = std::chrono::steady_clock::now();
            int rc = 0;
            if (hi > lo)
                rc = open ? ptls_hip_pipeline_open(node->pipe[d], node->ks[d], recs + lo, hi - lo, h_in, h_aad, h_out, h_result + lo)
                          : ptls_hip_pipeline_seal(node->pipe[d], node->ks[d], recs + lo, hi - lo, h_in, h_aad, h_out);
            node->seconds[d] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            rcs[d] = rc;
            if (rc != 0)
                errs[d] = g_err; /* thread_local: carried back to the caller's thread */
        });
    }
    for (auto &t : th)
        t.join();
    for (size_t d = 0; d < nd; ++d)
        if (rcs[d] != 0)
            return fail(rcs[d], "node: device %d: %s", node->eng[d]->device, errs[d].c_str());
    return 0;
}

extern "C" int ptls_hip_node_seal(ptls_hip_node_t *node, const ptls_hip_record_t *recs, size_t n, const void *h_in, const void *h_aad,
                                  void *h_out)
{
    return node_run(node, recs, n, h_in, h_aad, h_out, nullptr, false);
}

extern "C" int ptls_hip_node_open(ptls_hip_node_t *node, const ptls_hip_record_t *recs, size_t n, const void *h_in, const void *h_aad,
                                  void *h_out, uint64_t *h_result)
{
    return node_run(node, recs, n, h_in, h_aad, h_out, h_result, true);
}

extern "C" int ptls_hip_node_last_split(ptls_hip_node_t *node, double *seconds, size_t *bounds)
{
    if (node == nullptr)
        return fail(PTLS_HIP_EINVAL, "node_last_split: null node");
    if (seconds != nullptr)
        std::copy(node->seconds.begin(), node->seconds.end(), seconds);
    if (bounds != nullptr)
        std::copy(node->bounds.begin(), node->bounds.end(), bounds);
    return 0;
}
