/*
 * planner.cpp -- the launch planner of the batch kernels: lanes per record (choose_lanes), key-homogeneous chunks in
 * length order (build_chunks, guided_tail), workgroup size and grid.  Host-only arithmetic over the descriptors; the
 * measurements behind each rule are cited where it is made.
 */
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "host.h"
/* ---------------------------------------------------------------------------------------------- */
/* batches                                                                                         */
/* ---------------------------------------------------------------------------------------------- */

/* lanes per record from the mean GHASH length N = ceil(A/16) + ceil(L/16) + 1: keep >= ~16 Horner
 * steps per lane so the log2(G) reduction tree stays a small fraction of the work.  Many keys with few
 * records each (a server's connections): a workgroup works on one key at a time (its GHASH tables fill
 * the LDS), so with 8 lanes a 64-record key run gives only 8 wave tasks to 12 waves; 16 lanes per
 * record doubles the tasks per key run (measured on the 64K-key BASELINE shape). */
int choose_lanes(const ptls_hip_record_t *recs, size_t n, unsigned ncu)
{
    if (n == 0)
        return 1;
    double sum = 0;
    size_t runs = 1;
    for (size_t i = 0; i < n; ++i) {
        sum += (double)((recs[i].aad_len + 15) / 16 + (recs[i].len + 15) / 16 + 1);
        if (i != 0 && recs[i].key != recs[i - 1].key)
            ++runs;
    }
    const double mean = sum / (double)n;
    const double per_run = (double)n / (double)runs;
    /* round 4 (the windowed lane combination for every G, batch_kernel.h WIN_ALL): G = 4 is as fast as G = 8 or faster at
     * every length with long key runs (seal GiB/s G = 4 / 8, same box, tools/calls_r04/r04_call28.sh: 3 000 B 1 183 / 1 151,
     * 4 096 B 1 220 / 1 188, 8 192 B 1 215 / 1 222, c2's 16 KiB 1 258 / 1 250; 2 000 B 1 154-1 163 / 1 101; c3 G = 2 / 4
     * within 1 %).  Until then G = 8 from 128 GHASH elements (the tree's cost grew with log2 G differently) */
    const int g = mean >= 48 ? 4 : mean >= 16 ? 2 : 1;
    /* key runs too short to amortise the per-key GHASH tables: the key-independent wave-per-record kernel */
    if (per_run < SPARSE_MAX_PER_RUN)
        return SPARSE_LANES;
    /* long records, short key runs: more lanes per record give a key run more wave tasks for the workgroup's 12
     * waves, as long as the run fits one chunk (2 * 16 * 64 / G records): a run spilling into a second chunk costs up to
     * 25 %.  Measured on configs[3]'s lengths (AES-256, 64 B - 16 KiB, 4M records; tools/time_cfg.py), seal
     * GiB/s at 8 / 16 / 32 lanes, round 3 (the G = 32 window combination): 64 records per key 532 / 769 / 803, 96: 748 /
     * 813 / 620, 128: 810 / 827 / 804, 192: 838 / 644 / 806 (tools/calls_r03/r03_call17.sh); round 2 at 16 / 32 lanes
     * (sparse kernel): 8 per key 126 / 258 (503), 16: 260 / 499 (516), 24: 394 / 681 (525), 32: 518 / 715, 48: 717 / 734. */
    if (mean >= 256 && per_run <= 64)
        return 32;
    if (mean >= 256 && per_run <= 128)
        return 16;
    /* a run of up to 320 records is at most 20 wave tasks at G = 4 for 12 waves: G = 8 doubles them.  c4's lengths, seal
     * GiB/s G = 4 / 8 / 16 (tools/calls_r04/r04_call26.sh, r04_call30.sh): ~210 records per key 822 / 893 / 851, ~420 per
     * key 898 / 869 / -, one key 932 / 927 / - */
    if (mean >= 256 && per_run <= 320)
        return 8;
    /* Small batches: a launch gives each CU 12 waves that draw wave tasks of 64/G records, so a batch of fewer than
     * about two tasks per wave leaves most waves idle or waiting for one long last task.  More lanes per record make
     * more, shorter tasks, as long as each lane keeps >= 8 GHASH elements.  Round 5, same box, seal GiB/s at G = 4 / 8 /
     * 16 / 32 (tools/calls_r05/r05_call11.sh): c2's 16 KiB records, 4 096 records (64 MiB) 206 / 321 / 457 / 542,
     * 16 384 573-590 / 682-693 / 872-973 / 885-900, 65 536 981-997 / 983-989 / 974-990 / 938-966, 262 144 1 172-1 176 /
     * 1 179 / 1 173-1 176 / 1 144-1 149; c3's 1 350 B records at G = 2 / 4 / 8: 65 536 records 575 / 655-669 / 700-707,
     * 786 432 893-904 / 906-910 / 860-864. */
    int gs = g;
    const double waves = 12.0 * (double)(ncu ? ncu : 256);
    while (gs < 32 && (double)n * gs / 64.0 < 2.0 * waves && mean / (2.0 * gs) >= 8.0)
        gs *= 2;
    return gs;
}

/* grid of a launch: one workgroup per CU at most (both kernels fill the LDS); the batch kernel takes one
 * workgroup per chunk, the sparse kernel one per 12 records (a record per wave) */
unsigned plan_grid(size_t n, size_t nchunks, int lanes, unsigned ncu)
{
    if (lanes == SPARSE_LANES)
        return (unsigned)std::max<size_t>(1, std::min<size_t>((n + 11) / 12, (size_t)ncu));
    return (unsigned)std::min<size_t>(nchunks, ncu);
}

int plan_wg(const std::vector<Chunk> &ch, int lanes)
{
    /* Measured on MI355X (tools/tune.py, same-process sweep): 768 threads = 3 waves per SIMD at 168 VGPRs
     * (no spills for G <= 4) beats 512 (2 waves, 193 VGPRs) on every BASELINE shape: 1M x 16 KiB 1033 vs
     * 968 GiB/s seal, 4M x 1350 B 864 vs 788, 64K keys 416 vs 415; 1024 threads spills and loses to both. */
    (void)ch;
    (void)lanes;
    return WG_ALT;
}

/* Guided chunk sizes at the end of long key runs (batch_kernel.h QUEUE hands chunks out in plan order).  A workgroup's
 * last chunk ends the launch for it, so the chunks dealt last should be small: a chunk that starts when `rem` wave tasks
 * remain in the batch gets at most rem / (2 ncu) tasks (at least one), like guided self-scheduling.  Only chunks of key
 * runs longer than one full chunk are cut (configs[1], [2], [4]): a short run's pieces would each rebuild the key's GHASH
 * tables on another workgroup, and such batches already balance over many runs.  The records of a chunk stay in their
 * length-sorted order, so each piece is a contiguous, sorted range. */
static void guided_tail(std::vector<Chunk> &ch, uint32_t per_task, unsigned ncu)
{
    static const bool on = [] { /* PTLS_HIP_GUIDED=0 (environment): full-size chunks to the end (A/B measurements) */
        const char *e = getenv("PTLS_HIP_GUIDED");
        return e == nullptr || atoi(e) != 0;
    }();
    if (!on)
        return;
    size_t total = 0;
    for (const Chunk &c : ch)
        total += (c.count + per_task - 1) / per_task;
    std::vector<Chunk> out;
    out.reserve(ch.size() + 4 * (size_t)ncu);
    size_t done = 0;
    for (size_t k = 0; k < ch.size(); ++k) {
        Chunk c = ch[k];
        const bool long_run = (k > 0 && ch[k - 1].key == c.key) || (k + 1 < ch.size() && ch[k + 1].key == c.key);
        size_t tasks = (c.count + per_task - 1) / per_task;
        while (long_run && tasks > 1) {
            const size_t want = std::max<size_t>(1, (total - done) / (2 * (size_t)ncu));
            if (want >= tasks)
                break;
            Chunk piece = c;
            piece.count = (uint32_t)(want * per_task);
            out.push_back(piece);
            c.first += piece.count;
            c.count -= piece.count;
            done += want;
            tasks -= want;
        }
        done += tasks;
        out.push_back(c);
    }
    ch.swap(out);
}

/* chunk = run of records with one key slot, sized to keep all waves of a workgroup busy for a few tasks
 * (at most 32 wave tasks), but small enough that a batch of fewer tasks still spreads over every CU (the
 * grid is one workgroup per chunk up to the CU count).  Inside a chunk the records are ordered by
 * decreasing length, so the 64/lanes records a wave processes together have similar lengths (their
 * branch-free full-block stretch is limited by the shortest). */
void build_chunks(const ptls_hip_record_t *recs, size_t n, int lanes, unsigned ncu, std::vector<Chunk> &ch,
                         std::vector<uint32_t> &order, bool &all_aligned)
{
    ch.clear();
    order.resize(n);
    all_aligned = true;
    if (lanes == SPARSE_LANES) {
        /* the sparse kernel keeps no per-key workgroup state and its waves take records grid-stride: in
         * decreasing length over the whole batch every wave gets a similar share of bytes.  One chunk holds
         * the record count (the kernel reads nothing else from it); its key field names no slot. */
        bool sorted = true;
        uint32_t max_len = 0;
        for (size_t i = 0; i < n; ++i) {
            order[i] = (uint32_t)i;
            if (((recs[i].in_off | recs[i].out_off | recs[i].aad_off) & 15) != 0)
                all_aligned = false;
            if (i != 0 && recs[i].len > recs[i - 1].len)
                sorted = false;
            max_len = std::max(max_len, recs[i].len);
        }
        /* (the host plans every slice of a host-resident pipeline while the device runs the previous one: a comparison
         * sort of ~200K QUIC records per slice took longer than the slice's kernel) */
        if (!sorted && max_len < (1u << 24)) {
            /* stable counting sort by decreasing 16-byte block count: the kernel balances GHASH elements, not bytes */
            const uint32_t nb = (max_len >> 4) + 1;
            std::vector<uint32_t> start(nb + 1, 0);
            for (size_t i = 0; i < n; ++i)
                ++start[nb - 1 - (recs[i].len >> 4) + 1];
            for (uint32_t b = 0; b < nb; ++b)
                start[b + 1] += start[b];
            for (size_t i = 0; i < n; ++i)
                order[start[nb - 1 - (recs[i].len >> 4)]++] = (uint32_t)i;
        } else if (!sorted) {
            std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return recs[x].len > recs[y].len; });
        }
        if (n != 0)
            ch.push_back(Chunk{0, (uint32_t)n, 0xffffffffu, all_aligned ? 1u : 0u});
        return;
    }
    const uint32_t per_task = 64u / (uint32_t)lanes;
    const size_t tasks = (n + per_task - 1) / per_task;
    const size_t spread = (tasks + (ncu ? ncu : 1) - 1) / (ncu ? ncu : 1); /* tasks per chunk for >= ncu chunks */
    const uint32_t max_chunk = per_task * (uint32_t)std::max<size_t>(1, std::min<size_t>((WG_MAX / 64) * 2, spread));
    size_t i = 0;
    while (i < n) {
        Chunk c;
        c.first = (uint32_t)i;
        c.key = recs[i].key;
        c.count = 0;
        c.flags = 1;
        bool sorted = true;
        while (i < n && recs[i].key == c.key && c.count < max_chunk) {
            if (((recs[i].in_off | recs[i].out_off | recs[i].aad_off) & 15) != 0)
                c.flags = 0;
            if (c.count != 0 && recs[i].len > recs[i - 1].len)
                sorted = false;
            order[i] = (uint32_t)i;
            ++c.count;
            ++i;
        }
        if (!sorted)
            std::stable_sort(order.begin() + c.first, order.begin() + c.first + c.count,
                             [&](uint32_t x, uint32_t y) { return recs[x].len > recs[y].len; });
        all_aligned = all_aligned && (c.flags & 1u);
        ch.push_back(c);
    }
    guided_tail(ch, per_task, ncu ? ncu : 1);
}


/* The kernels read the descriptors in plan order (recs_ord).  When the plan keeps the caller's order (records that
 * already come as the planner sorts them: equal lengths, non-increasing lengths within each key run), the caller-order
 * copy serves as both: no host gather and one descriptor upload less per pipeline slice (a 1 GiB slice set of QUIC
 * records is ~800K descriptors; the host plans each slice while the device runs the previous one). */
bool identity_order(const std::vector<uint32_t> &order, size_t n)
{
    for (size_t t = 0; t < n; ++t)
        if (order[t] != (uint32_t)t)
            return false;
    return true;
}
