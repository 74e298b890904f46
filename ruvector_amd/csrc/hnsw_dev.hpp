// hnsw_dev.hpp — device helpers shared by the HNSW search (k_hnsw.hip) and
// build (k_hnsw_build.hip) kernels: exact-order distances, the tagged visited
// hash and wave-parallel sorted inserts.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>

#include "poincare_dev.hpp"
#include "rvx/rvx.h"

namespace rvx {
namespace hnswdev {

constexpr int VCAP_MIN = 32768;  // visited-set slots per query (power of two), grown with ef
constexpr int C_EXTRA = 128; // candidate capacity = ef + C_EXTRA (builder)
constexpr int ID_MASK = 0x7FFFFFFF;  // node ids; bit 31 is the search's expanded flag

// One float4 step of the reference's scalar accumulation (distance.rs:34-85).
template <int METRIC>
__device__ __forceinline__ float acc4(float acc, const float4& q, const float4& v) {
    if (METRIC == RVX_METRIC_L2) {
        float t = q.x - v.x; acc = acc + t * t;
        t = q.y - v.y; acc = acc + t * t;
        t = q.z - v.z; acc = acc + t * t;
        t = q.w - v.w; acc = acc + t * t;
    } else if (METRIC == RVX_METRIC_L1) {
        acc = acc + fabsf(q.x - v.x); acc = acc + fabsf(q.y - v.y);
        acc = acc + fabsf(q.z - v.z); acc = acc + fabsf(q.w - v.w);
    } else {
        acc = acc + q.x * v.x; acc = acc + q.y * v.y; acc = acc + q.z * v.z; acc = acc + q.w * v.w;
    }
    return acc;
}

template <int METRIC>
__device__ __forceinline__ float finish_dist(float acc, float qn, float xn) {
    if (METRIC == RVX_METRIC_L2) return sqrtf(acc);
    if (METRIC == RVX_METRIC_DOT) return -acc;
    if (METRIC == RVX_METRIC_COSINE) return (qn > 1e-8f && xn > 1e-8f) ? 1.0f - acc / (qn * xn) : 1.0f;
    return acc;
}

// One lane's exact-order distance over a stored row, the row streamed in
// 128-B batches with the next batch's loads in flight while the current one
// accumulates (one load at a time would expose a memory round trip per 16 B
// of a 3 KB row). Q_GLOBAL: the other operand is a stored row too (pair_dist)
// and is streamed the same way; otherwise it is read at use (LDS).
#ifndef RVX_ROW_BATCH
#define RVX_ROW_BATCH 8
#endif
constexpr int ROW_BATCH = RVX_ROW_BATCH;  // float4s per batch

template <int METRIC, bool Q_GLOBAL, int RB = ROW_BATCH>
__device__ __forceinline__ float stream_acc(const float* __restrict__ qs, const float* __restrict__ x, int n4) {
    const float4* r = reinterpret_cast<const float4*>(x);
    const float4* qq = reinterpret_cast<const float4*>(qs);
    float acc = 0.0f;
    // Main loop over whole double batches with no branch between a load and its
    // use (a guarded load would sit in its own block and the waitcnt pass would
    // fall back to vmcnt(0), serialising the row again); the last prefetch
    // re-reads a batch already in cache instead of branching.
    const int nfull = n4 / (2 * RB) * (2 * RB);
    if (nfull > 0) {
        float4 xa[RB], xb[RB], qa[Q_GLOBAL ? RB : 1], qb[Q_GLOBAL ? RB : 1];
        auto load = [&](float4* xv, float4* qv, int base) {
#pragma unroll
            for (int j = 0; j < RB; ++j) {
                xv[j] = r[base + j];
                if constexpr (Q_GLOBAL) qv[j] = qq[base + j];
            }
        };
        auto run = [&](const float4* xv, const float4* qv, int base) {
#pragma unroll
            for (int j = 0; j < RB; ++j) acc = acc4<METRIC>(acc, Q_GLOBAL ? qv[j] : qq[base + j], xv[j]);
        };
        load(xa, qa, 0);
        for (int base = 0; base < nfull; base += 2 * RB) {
            load(xb, qb, base + RB);
            run(xa, qa, base);
            load(xa, qa, base + 2 * RB < nfull ? base + 2 * RB : base);
            run(xb, qb, base + RB);
        }
    }
    for (int k = nfull; k < n4; ++k) acc = acc4<METRIC>(acc, qq[k], r[k]);
    return acc;
}

// curv: the Poincaré curvature (RVX_METRIC_POINCARE only: HyperbolicHnsw::distance,
// fused norms + poincare_distance_from_norms, hnsw.rs:173-180)
template <int METRIC, bool Q_GLOBAL = false, int RB = ROW_BATCH>
__device__ __forceinline__ float row_dist(const float* __restrict__ qs, const float* __restrict__ x, int d, float qn,
                                          float xn, float curv = 1.0f) {
    if constexpr (METRIC == RVX_METRIC_POINCARE) return pdev::hyp_dist(qs, x, d, curv);
    if constexpr (METRIC == RVX_METRIC_HYP_L2) return pdev::hyp_l2(qs, x, d);
    float acc = 0.0f;
    if ((d & 3) == 0) {
        acc = stream_acc<METRIC, Q_GLOBAL, RB>(qs, x, d >> 2);
    } else {
        for (int k = 0; k < d; ++k) {
            const float q = qs[k], v = x[k];
            if (METRIC == RVX_METRIC_L2) { const float t = q - v; acc = acc + t * t; }
            else if (METRIC == RVX_METRIC_L1) acc = acc + fabsf(q - v);
            else acc = acc + q * v;
        }
    }
    return finish_dist<METRIC>(acc, qn, xn);
}

// ---- wave-cooperative distances ----------------------------------------------
// dist(q, x[row_lane]) for the 64 rows a wave's lanes name (-1: none, result
// unused), each still ONE lane's sequential chain in the reference order. Rows
// reach LDS by LDS-DMA, 32 dims per chunk: one wave instruction moves 8 rows x
// 128 B, so it touches 8 pages where per-lane streaming touches 64 — beyond a
// few GB of randomly read rows the per-CU translation cache, not HBM, bounds a
// per-lane search (86% UTCL1 misses at 12 GB). Stage layout [64 rows][128 B],
// 16-B slot p ^ ((row >> 1) & 7) (conflict-free for the per-lane ds_read_b128).
// Two stages: the next chunk's DMA is in flight while this one accumulates.
// Requires no other vector-memory op of the wave between a fill and its wait.
// NST stages per wave: 2 keeps the next chunk's DMA in flight; 1 halves the
// wave's LDS so more waves fit a CU (the search takes it past ef 1024, where
// the R list already costs most of the LDS: C3 10M x 768 ef 3200 5.9k -> 8.1k QPS,
// equal at ef 800, -3.5% at ef 100; scripts/exp_wd_stages.sh).
constexpr int WD_CH = 32;                     // dims per chunk
constexpr int WD_STAGE = 64 * WD_CH * 4;      // bytes per stage
constexpr int WD_LDS = 2 * WD_STAGE;          // bytes per wave, two stages
__host__ __device__ constexpr int wd_lds(int nst) { return nst * WD_STAGE; }

__host__ __device__ inline bool wave_dist_ok(int d) { return d % WD_CH == 0; }

template <int METRIC>
__device__ __forceinline__ void wd_fill(const float* __restrict__ x, int d, const int (&rid)[8], int c, int lane,
                                        unsigned char* st) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int j = 8 * i + (lane >> 3);
        const int piece = (lane & 7) ^ ((j >> 1) & 7);
        __builtin_amdgcn_global_load_lds((const void*)(x + (int64_t)rid[i] * d + c * WD_CH + 4 * piece),
                                         (__attribute__((address_space(3))) void*)(st + i * 1024), 16, 0, 0);
    }
}

// QC: qs is the query row in global memory, read through the constant address space, so
// the wave-uniform reads are scalar loads (lgkmcnt, not vmcnt: the DMA accounting below stays
// exact) and the query needs no LDS; else qs is the query staged in LDS.
template <int METRIC, bool QC = false>
__device__ __forceinline__ float wd_chunk(float acc, const float* qs, int c, int lane, const unsigned char* st) {
    const int sw = (lane >> 1) & 7;
    if constexpr (QC) {
        typedef const __attribute__((address_space(4))) float cf;
        cf* qq = (cf*)(qs + c * WD_CH);
        float4 qv[WD_CH / 4];
#pragma unroll
        for (int p = 0; p < WD_CH / 4; ++p) qv[p] = make_float4(qq[4 * p], qq[4 * p + 1], qq[4 * p + 2], qq[4 * p + 3]);
#pragma unroll
        for (int p = 0; p < WD_CH / 4; ++p) {
            const float4 v = *reinterpret_cast<const float4*>(st + lane * (WD_CH * 4) + ((p ^ sw) << 4));
            acc = acc4<METRIC>(acc, qv[p], v);
        }
        return acc;
    }
    const float4* qq = reinterpret_cast<const float4*>(qs + c * WD_CH);
#pragma unroll
    for (int p = 0; p < WD_CH / 4; ++p) {
        const float4 v = *reinterpret_cast<const float4*>(st + lane * (WD_CH * 4) + ((p ^ sw) << 4));
        acc = acc4<METRIC>(acc, qq[p], v);
    }
    return acc;
}

// Ordering is explicit: nothing in the compiler orders a ds_read behind an
// LDS-DMA to the same bytes (only a barrier drains them), so before reading a
// stage the wave waits vmcnt(8) — the 8 DMAs of the next chunk may still be
// in flight, everything older (this chunk) has landed — and before refilling a
// stage it waits lgkmcnt(0) so the stage's reads have returned. The asm
// statements clobber memory, which also keeps the DMA groups in issue order.
// vmcnt(8 * G): at most G chunk groups (8 DMAs each) still in flight
template <int G>
__device__ __forceinline__ void wd_wait_groups() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * G) : "memory");
}
// the ring's tail: `left` (< NST - 1, wave-uniform) younger groups may stay in flight
template <int NST>
__device__ __forceinline__ void wd_wait_left(int left) {
    static_assert(NST <= 8, "vmcnt holds at most 63 outstanding loads");
    switch (left) {
        case 0: wd_wait_groups<0>(); break;
        case 1: wd_wait_groups<1>(); break;
        case 2: wd_wait_groups<2>(); break;
        case 3: wd_wait_groups<3>(); break;
        case 4: wd_wait_groups<4>(); break;
        case 5: wd_wait_groups<5>(); break;
        default: wd_wait_groups<6>(); break;
    }
}

template <int METRIC, int NST = 2, bool QC = false>
__device__ __forceinline__ float wd_run(const float* __restrict__ x, int d, const float* qs, const int (&rid)[8], int lane,
                                        unsigned char* s0, unsigned char* s1) {
    const int nch = d / WD_CH;
    float acc = 0.0f;
    if constexpr (NST >= 3) {
        // a ring of NST stages (s0 .. s0 + (NST-1) * WD_STAGE): NST - 1 chunks in flight
        // while one accumulates — for waves alone on their CU (large ef: R holds most
        // of the LDS), where no other wave hides a chunk's memory round trip
        int fill = 0;  // stage the next fill lands in
        for (; fill < NST - 1 && fill < nch; ++fill) wd_fill<METRIC>(x, d, rid, fill, lane, s0 + fill * WD_STAGE);
        int cur = 0;  // stage chunk c is in
        for (int c = 0; c < nch; ++c) {
            const int nx = c + NST - 1;
            if (nx < nch) {
                // stage `fill` held chunk c - 1, whose reads returned (lgkmcnt(0) below)
                wd_fill<METRIC>(x, d, rid, nx, lane, s0 + fill * WD_STAGE);
                fill = fill + 1 == NST ? 0 : fill + 1;
                wd_wait_groups<NST - 1>();
            } else {
                wd_wait_left<NST>(nch - 1 - c);
            }
            acc = wd_chunk<METRIC, QC>(acc, qs, c, lane, s0 + cur * WD_STAGE);
            cur = cur + 1 == NST ? 0 : cur + 1;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        return acc;
    }
    if constexpr (NST == 1) {
        for (int c = 0; c < nch; ++c) {
            wd_fill<METRIC>(x, d, rid, c, lane, s0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            acc = wd_chunk<METRIC, QC>(acc, qs, c, lane, s0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        return acc;
    }
    wd_fill<METRIC>(x, d, rid, 0, lane, s0);
    for (int c = 0; c < nch; c += 2) {
        if (c + 1 < nch) {
            wd_fill<METRIC>(x, d, rid, c + 1, lane, s1);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        acc = wd_chunk<METRIC, QC>(acc, qs, c, lane, s0);
        if (c + 1 >= nch) break;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (c + 2 < nch) {
            wd_fill<METRIC>(x, d, rid, c + 2, lane, s0);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        acc = wd_chunk<METRIC, QC>(acc, qs, c + 1, lane, s1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    return acc;
}

// All 64 lanes call together. row < 0: no row (the lane's result is garbage).
template <int METRIC, int NST = 2, bool QC = false>
__device__ __forceinline__ float wave_dist(const float* qs, const float* __restrict__ x, int d, int row, float qn,
                                           float xn, unsigned char* stage, int lane) {
    int rid[8];
    const int mine = row < 0 ? 0 : row;
#pragma unroll
    for (int i = 0; i < 8; ++i) rid[i] = __shfl(mine, 8 * i + (lane >> 3));
    const float acc = wd_run<METRIC, NST, QC>(x, d, qs, rid, lane, stage, stage + WD_STAGE);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // stages are refilled by the next call
    return finish_dist<METRIC>(acc, qn, xn);
}

// Claim `node` in a query's visited set: true if it was not visited yet.
// Slots whose tag is another query's are free (the table is zeroed per launch).
// A table that has no free slot left sets *full (the host turns it into an error: the
// node would otherwise be skipped without a trace); visited_capacity sizes tables so this
// cannot happen below 8 ef expansions of full lists, and never for tables of >= 2n slots.
__device__ __forceinline__ bool visit_claim(unsigned long long* vis, unsigned vmask, unsigned long long qtag, int node,
                                            int* full) {
    const unsigned long long key = qtag | (unsigned)(node + 1);
    unsigned h = ((unsigned)node * 2654435761u) & vmask;
    unsigned long long cur = __hip_atomic_load(&vis[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (unsigned probe = 0; probe <= vmask; ++probe) {
        if ((cur & 0xFFFFFFFF00000000ull) == qtag) {
            if (cur == key) return false;
            h = (h + 1) & vmask;
            cur = __hip_atomic_load(&vis[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            continue;
        }
        const unsigned long long prev = atomicCAS(&vis[h], cur, key);
        if (prev == cur) return true;
        cur = prev;
    }
    atomicOr(full, 1);  // table full (every slot probed): reported, never silent
    return false;
}

// visited-table size (a power of two) for a search of width ef over lists of <= max_deg
// neighbours in a graph of n nodes: a search of width ef expands ~ef..2ef nodes of <= max_deg
// neighbours each, so 4 ef max_deg slots keep the load well below 1/2; up to 2^30 slots (8 GiB),
// and never more than the first power of two >= 2n — a query claims each node at most once, so
// such a table is never more than half full. Callers size their slot count by bytes.
inline unsigned visited_capacity(int ef, int max_deg, int64_t n) {
    unsigned v = VCAP_MIN;
    const uint64_t want = (uint64_t)ef * 4u * (uint64_t)std::max(max_deg, 64);
    while (v < want && v < (1u << 30)) v <<= 1;
    const uint64_t all = 2 * (uint64_t)std::max<int64_t>(n, 1);
    while (v > 64 && (uint64_t)(v >> 1) >= all) v >>= 1;
    return v;
}

__device__ __forceinline__ bool lt(float d, int id, float bd, int bid) { return d < bd || (d == bd && id < bid); }

// wave-parallel insert of (d,id) into an array sorted ascending (asc=true) or
// descending by (d,id); size must be < capacity. Returns new size.
__device__ __forceinline__ int sorted_insert(float* ad, int* ai, int size, float d, int id, bool asc, int lane) {
    // position = number of elements that stay in front of the new one
    int cnt = 0;
    for (int i = lane; i < size; i += 64) {
        const bool before = asc ? lt(ad[i], ai[i], d, id) : lt(d, id, ad[i], ai[i]);
        cnt += before ? 1 : 0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    const int pos = cnt;
    // shift [pos, size) right by one, walking chunks from the end so every
    // read of a chunk happens before the writes that could overwrite it
    for (int base = ((size - 1) / 64) * 64; base >= pos - 63 && base >= 0; base -= 64) {
        const int i = base + lane;
        float vd = 0.f; int vi = 0;
        const bool mv = (i >= pos && i < size);
        if (mv) { vd = ad[i]; vi = ai[i]; }
        __builtin_amdgcn_wave_barrier();
        if (mv) { ad[i + 1] = vd; ai[i + 1] = vi; }
        __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0) { ad[pos] = d; ai[pos] = id; }
    __builtin_amdgcn_wave_barrier();
    return size + 1;
}


// ---- batched admission ------------------------------------------------------
// search_layer's neighbour loop (hnsw.rs:1004-1046) admits the fresh neighbours
// of one expansion in list order: e is admitted iff d(e) < d(farthest in R) or
// |R| < ef; admitted e goes into C and R, and R drops its farthest when
// |R| > ef. Only the running farthest makes the order matter, so:
//  1. decisions: walk the fresh lanes in order against a register window
//     holding R's largest <= 64 entries (lane wn-1 = the max): each admission
//     inserts into the window (or below it) and pops the window max when
//     |R| > ef — the exact sequence of farthest values;
//  2. merge: pops only ever remove the current maximum, so the final R is the
//     |R_new| smallest of R ∪ A and C is C ∪ A (both by (d, id)); each array
//     takes ONE in-place merge (ranks by binary search, moves from the back)
//     instead of a wave-wide sorted insert per admitted neighbour.
// A batch that could reach the candidate capacity takes the per-element path
// (its farthest-candidate drop rule depends on the order).
// scratch: LDS [64] floats + [64] ints. Returns false on candidate overflow.

__device__ __forceinline__ bool lt_de(float d, int id, float bd, int bid) { return d < bd || (d == bd && id < bid); }

// number of entries of the sorted array (asc: ascending, else descending by (d,id))
// placed before (d, id); n <= 64 entries, binary search
__device__ __forceinline__ int rank_in(const float* ad, const int* ai, int n, float d, int id, bool asc) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const bool before = asc ? lt_de(ad[mid], ai[mid], d, id) : lt_de(d, id, ad[mid], ai[mid]);
        if (before) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// merge the sorted batch (sd, si)[0..na) into the sorted array (ad, ai)[0..n),
// keeping the first nkeep entries; same order (asc) for both.
__device__ __forceinline__ void merge_sorted(float* ad, int* ai, int n, const float* sd, const int* si, int na, int nkeep,
                                             bool asc, int lane) {
    // batch positions first (they search the array before it moves)
    int bpos = -1;
    float bd = 0.f; int bi = 0;
    if (lane < na) {
        bd = sd[lane]; bi = si[lane];
        bpos = lane + rank_in(ad, ai, n, bd, bi, asc);
    }
    __builtin_amdgcn_wave_barrier();
    // array entries move right by the number of batch entries before them; walk
    // chunks from the back so a chunk is read before anything can overwrite it
    for (int base = ((n - 1) / 64) * 64; base >= 0; base -= 64) {
        const int j = base + lane;
        float vd = 0.f; int vi = 0, pos = -1;
        if (j < n) {
            vd = ad[j]; vi = ai[j];
            pos = j + rank_in(sd, si, na, vd, vi, asc);
        }
        __builtin_amdgcn_wave_barrier();
        if (pos >= 0 && pos < nkeep) { ad[pos] = vd; ai[pos] = vi; }
        __builtin_amdgcn_wave_barrier();
    }
    if (bpos >= 0 && bpos < nkeep) { ad[bpos] = bd; ai[bpos] = bi; }
    __builtin_amdgcn_wave_barrier();
}

// Exact sequential admission decisions of one expansion's fresh neighbours
// (lanes in fmask, in lane order) against a register window of R's largest
// <= 64 entries (lane wn-1 = the max): each admission inserts into the window
// (or below it) and pops the window max when |R| > ef, which reproduces the
// exact sequence of farthest values. Returns the admitted lane mask; r = |R|
// after the batch. R ids may carry the search's expanded flag in bit 31
// (masked off here).
// decide_window: the same decisions from a window already in registers — lane l < wn holds the
// (below + l)-th smallest entry of R (ids masked), `total` = |R| (the buffered HBM R below).
__device__ __forceinline__ unsigned long long decide_window(unsigned long long fmask, float dd, int nid, int ef,
                                                            float wd, int wi, int wn, int below, int total, int& r,
                                                            int lane) {
    r = total;
    unsigned long long adm = 0ull;
    unsigned long long todo = fmask;
    while (todo) {
        const int src = __ffsll((long long)todo) - 1;
        todo &= todo - 1;
        const float ed = __shfl(dd, src);
        const int eid = __shfl(nid, src);
        const float fd = __shfl(wd, wn - 1);  // current farthest of R
        if (!(ed < fd || r < ef)) continue;
        adm |= 1ull << src;
        r += 1;
        const float w0d = __shfl(wd, 0);
        const int w0i = __shfl(wi, 0);
        if (below == 0 || !lt_de(ed, eid, w0d, w0i)) {
            if (wn == 64) {  // keep 64: the smallest window entry moves below
                wd = __shfl_down(wd, 1); wi = __shfl_down(wi, 1);
                if (lane == 63) { wd = INFINITY; wi = INT_MAX; }
                wn = 63; below += 1;
            }
            const int pos = __popcll(__ballot(lane < wn && lt_de(wd, wi, ed, eid)));
            const float ud = __shfl_up(wd, 1);
            const int ui = __shfl_up(wi, 1);
            if (lane > pos && lane <= wn) { wd = ud; wi = ui; }
            if (lane == pos) { wd = ed; wi = eid; }
            wn += 1;
        } else {
            below += 1;
        }
        if (r > ef) {  // pop the farthest
            if (lane == wn - 1) { wd = INFINITY; wi = INT_MAX; }
            wn -= 1; r -= 1;
        }
    }
    return adm;
}

__device__ __forceinline__ unsigned long long decide_batch(unsigned long long fmask, float dd, int nid, int ef,
                                                           const float* rd, const int* ri, int rs, int& r, int lane) {
    const int wn = min(rs, 64);
    const int below = rs - wn;
    float wd = INFINITY; int wi = INT_MAX;
    if (lane < wn) { wd = rd[below + lane]; wi = ri[below + lane] & ID_MASK; }
    return decide_window(fmask, dd, nid, ef, wd, wi, wn, below, rs, r, lane);
}

// The same admissions decided in parallel (R in LDS). Sequentially (hnsw.rs:1004-1046) fresh
// neighbour i enters R iff |R| < ef or it precedes R's farthest. While R is full its farthest
// never grows, and a refused neighbour is at or beyond it, so the refused ones never precede a
// later admitted one: neighbour i enters iff fewer than ef entries of R_0 ∪ {fresh j < i}
// precede it — its rank in R_0 (a binary search in LDS, every lane at once) plus the earlier
// fresh neighbours before it (one pass of wave-uniform lane reads). Same admissions as
// decide_batch for distinct (d, id) pairs (R never holds a fresh node); callers keep
// decide_batch when a distance is NaN. rk: the lane's rank in R_0 (merge_into_r reuses it).
__device__ __forceinline__ int rank_in_r(const float* rd, const int* ri, int n, float d, int id);
__device__ __forceinline__ unsigned long long decide_par(unsigned long long fmask, float dd, int nid, int ef,
                                                         const float* rd, const int* ri, int rs, int& r, int& rk,
                                                         int lane) {
    const bool mine = (fmask >> lane) & 1ull;
    rk = mine ? rank_in_r(rd, ri, rs, dd, nid) : 0;
    int before = 0;
    for (unsigned long long t = fmask; t; t &= t - 1) {
        const int o = __ffsll((long long)t) - 1;
        const float od = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dd), o));
        const int oi = __builtin_amdgcn_readlane(nid, o);
        before += (o < lane && lt_de(od, oi, dd, nid)) ? 1 : 0;
    }
    const unsigned long long adm = __ballot(mine && rk + before < ef);
    r = min(ef, rs + __popcll(adm));
    return adm;
}

// The admitted lanes' (d, id) sorted ascending into the scratch (sd, si)[0..na).
// srk (nullable): also each entry's rank in R (decide_par's rk) at its sorted position.
__device__ __forceinline__ int sort_batch(unsigned long long adm, float dd, int nid, float* sd, int* si, int lane,
                                          int* srk = nullptr, int rk = 0) {
    const int na = __popcll(adm);
    if (na == 0) return 0;
    const bool mine = (adm >> lane) & 1ull;
    int rank = 0;
    for (unsigned long long t = adm; t; t &= t - 1) {
        const int o = __ffsll((long long)t) - 1;
        const float od = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dd), o));
        const int oi = __builtin_amdgcn_readlane(nid, o);
        rank += lt_de(od, oi, dd, nid) ? 1 : 0;
    }
    if (mine) {
        sd[rank] = dd; si[rank] = nid;
        if (srk) srk[rank] = rk;
    }
    __builtin_amdgcn_wave_barrier();
    return na;
}

__device__ bool admit_batch(bool fresh, float dd, int nid, int ef, int ccap, float* rd, int* ri, int& rs, float* cd,
                            int* ci, int& cs, float* sd, int* si, int lane) {
    const unsigned long long fmask = __ballot(fresh);
    if (!fmask) return true;
    const int nf = __popcll(fmask);
    if (cs + nf > ccap) {
        // per-element path (rare: the candidate list is near its capacity)
        unsigned long long todo = fmask;
        while (todo) {
            const int src = __ffsll((long long)todo) - 1;
            todo &= todo - 1;
            const float ed = __shfl(dd, src);
            const int eid = __shfl(nid, src);
            const float fd = rd[rs - 1];
            if (ed < fd || rs < ef) {
                if (cs >= ccap) {
                    if (cd[0] > fd) {  // drop the farthest candidate: it can only terminate the search
                        for (int base = 0; base < cs - 1; base += 64) {
                            const int i = base + lane;
                            float vd = 0.f; int vi = 0;
                            const bool mv = i + 1 < cs;
                            if (mv) { vd = cd[i + 1]; vi = ci[i + 1]; }
                            __builtin_amdgcn_wave_barrier();
                            if (mv) { cd[i] = vd; ci[i] = vi; }
                            __builtin_amdgcn_wave_barrier();
                        }
                        cs -= 1;
                    } else {
                        return false;
                    }
                }
                cs = sorted_insert(cd, ci, cs, ed, eid, /*asc=*/false, lane);
                rs = sorted_insert(rd, ri, rs, ed, eid, /*asc=*/true, lane);
                if (rs > ef) rs -= 1;
            }
        }
        return true;
    }
    int r = rs;
    const unsigned long long adm = decide_batch(fmask, dd, nid, ef, rd, ri, rs, r, lane);
    const int na = sort_batch(adm, dd, nid, sd, si, lane);
    if (na == 0) return true;
    merge_sorted(rd, ri, rs, sd, si, na, r, /*asc=*/true, lane);
    rs = r;
    // C is descending: the same batch reversed
    float xd = 0.f; int xi = 0;
    if (lane < na) { xd = sd[na - 1 - lane]; xi = si[na - 1 - lane]; }
    __builtin_amdgcn_wave_barrier();
    if (lane < na) { sd[lane] = xd; si[lane] = xi; }
    __builtin_amdgcn_wave_barrier();
    merge_sorted(cd, ci, cs, sd, si, na, cs + na, /*asc=*/false, lane);
    cs += na;
    return true;
}

// ---- search: R only ---------------------------------------------------------
// The search keeps no candidate array: a candidate that is not in R is at or
// beyond R's farthest in the (d, id) order and, R's farthest never growing
// once |R| = ef, would end the search when popped, so "pop the nearest
// candidate" is "take the nearest unexpanded entry of R" (bit 31 of its id
// marks it expanded) and "stop" is "none left". That is search_layer's loop
// (hnsw.rs:913-1055) with the stop test comparing (d, id) pairs, which only
// differs from the reference's distance-only test on an exact distance tie
// with R's farthest (the reference's heaps leave tie order unspecified).

// R's rank of (d, id): entries of R (ascending, flagged ids) ordered before it
__device__ __forceinline__ int rank_in_r(const float* rd, const int* ri, int n, float d, int id) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (lt_de(rd[mid], ri[mid] & ID_MASK, d, id)) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// Merge the ascending batch (sd, si)[0..na) into R (rd, ri)[0..n), keeping the
// first nkeep entries. Each batch entry finds its rank in R by binary search;
// R entry j moves right by #{batch entries ranked <= j}, a constant over every
// 64-entry chunk that holds no batch rank, so only chunks at or after the
// first rank move and each costs one ballot. Returns the first batch rank
// (entries before it did not move). Chunks move in groups of MG walking back:
// a group is read whole, then written (entries only move right, so a group's
// writes land at or above its own lowest entry and never on the next group's),
// which keeps MG reads in flight instead of one memory round trip per chunk —
// at ef 12288 a merge walks up to 192 chunks. MG costs 3 VGPRs per chunk: 8 for R
// in HBM, 2 for R in LDS (short round trips; the LDS kernels' occupancy is
// register-bound).
#ifndef RVX_MERGE_LDS_G
#define RVX_MERGE_LDS_G 2
#endif
#ifndef RVX_MERGE_RG_G
#define RVX_MERGE_RG_G 8
#endif
template <int MERGE_GROUP = RVX_MERGE_LDS_G>
__device__ __forceinline__ int merge_into_r(float* rd, int* ri, int n, const float* sd, const int* si, int na, int nkeep,
                                            int lane, const int* srk = nullptr) {
    float bd = 0.f; int bi = 0, rk = INT_MAX;
    if (lane < na) { bd = sd[lane]; bi = si[lane]; rk = srk ? srk[lane] : rank_in_r(rd, ri, n, bd, bi); }
    const int first = __shfl(rk, 0);
    __builtin_amdgcn_wave_barrier();
    for (int top = ((n - 1) / 64) * 64; top >= 0 && top + 63 >= first; top -= 64 * MERGE_GROUP) {
        float vd[MERGE_GROUP];
        int vi[MERGE_GROUP], sh[MERGE_GROUP];
#pragma unroll
        for (int g = 0; g < MERGE_GROUP; ++g) {
            const int base = top - 64 * g;
            const int j = base + lane;
            sh[g] = -1;
            vd[g] = 0.f; vi[g] = 0;
            if (base >= 0 && base + 63 >= first) {  // wave-uniform
                // batch entries ranked at or before the chunk, and those inside it
                int shift = __popcll(__ballot(lane < na && rk <= base));
                unsigned long long in = __ballot(lane < na && rk > base && rk <= base + 63);
                while (in) {
                    const int b = __ffsll((long long)in) - 1;
                    in &= in - 1;
                    shift += (j >= __shfl(rk, b)) ? 1 : 0;
                }
                if (j < n) { vd[g] = rd[j]; vi[g] = ri[j]; sh[g] = shift; }
            }
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int g = 0; g < MERGE_GROUP; ++g) {
            const int j = top - 64 * g + lane;
            if (sh[g] >= 0 && j + sh[g] < nkeep) { rd[j + sh[g]] = vd[g]; ri[j + sh[g]] = vi[g]; }
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (lane < na && lane + rk < nkeep) { rd[lane + rk] = bd; ri[lane + rk] = bi; }
    __builtin_amdgcn_wave_barrier();
    return first;
}

// ---- R in HBM with an LDS buffer (the HBM-resident-R search, k_hnsw.hip RG) ---------------
// R = Rh ∪ B: Rh a sorted array in the slot's HBM row, B a sorted array of <= RB_CAP entries in
// LDS; every (d, id) pair is in one of them. Admissions go into B (an LDS merge); B moves into
// Rh in one walk down Rh when it would overflow (flush_into_r) — instead of one walk, with a
// binary search per admitted entry, over Rh in HBM per admission batch (the HBM-R
// merges were 60-66% of the cycles and doubled the bytes, one merge at ef 12,288 reading and
// rewriting ~98 KB). The search is the same set operations on R, so the same expansions, the
// same admissions and the same result bits.
#ifndef RVX_RB_CAP
#define RVX_RB_CAP 256
#endif
constexpr int RB_CAP = RVX_RB_CAP;
// an expansion's fresh neighbours collected before admission (k_hnsw.hip collect_fresh): whole
// layer-0 lists of up to this many entries (MAX_C0, the builder's cap), longer lists slice by slice
constexpr int FRESH_CAP = 256;

// The union window: lane l < wn gets the (below + l)-th smallest entry of Rh ∪ B (id masked),
// wsrc 1 when it comes from B. The union's largest 64 lie within Rh's largest 64 and B's largest
// 64 (an entry with 63 larger ones in the union has at most 63 larger in its own array). Scratch:
// sd / si / so [64] in LDS.
__device__ __forceinline__ void union_window(const float* rd, const int* ri, int rs, const float* bd, const int* bi,
                                             int nb, float* sd, int* si, int* so, float& wd, int& wi, int& wsrc,
                                             int& wn, int& below, int lane) {
    const int wr = min(rs, 64), wb = min(nb, 64);
    float ed = INFINITY, fd = INFINITY;
    int eid = INT_MAX, fid = INT_MAX;
    if (lane < wr) { ed = rd[rs - wr + lane]; eid = ri[rs - wr + lane] & ID_MASK; }
    if (lane < wb) { fd = bd[nb - wb + lane]; fid = bi[nb - wb + lane] & ID_MASK; }
    int rkr = lane, rkb = lane;  // rank among the wr + wb window entries (pairs are distinct)
    for (int o = 0; o < wb; ++o) {
        const float od = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fd), o));
        rkr += lt_de(od, __builtin_amdgcn_readlane(fid, o), ed, eid) ? 1 : 0;
    }
    for (int o = 0; o < wr; ++o) {
        const float od = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ed), o));
        rkb += lt_de(od, __builtin_amdgcn_readlane(eid, o), fd, fid) ? 1 : 0;
    }
    wn = min(rs + nb, 64);
    below = rs + nb - wn;
    const int cut = wr + wb - wn;
    __builtin_amdgcn_wave_barrier();
    if (lane < wr && rkr >= cut) { sd[rkr - cut] = ed; si[rkr - cut] = eid; so[rkr - cut] = 0; }
    if (lane < wb && rkb >= cut) { sd[rkb - cut] = fd; si[rkb - cut] = fid; so[rkb - cut] = 1; }
    __builtin_amdgcn_wave_barrier();
    wd = INFINITY; wi = INT_MAX; wsrc = 0;
    if (lane < wn) { wd = sd[lane]; wi = si[lane]; wsrc = so[lane]; }
    __builtin_amdgcn_wave_barrier();
}

// After decide_window over the union window (wd, wi, wsrc)[0..wn) and the sorted admitted batch
// (sd, si)[0..na): the union holds total + na entries and keeps the first r, so the
// npop = total + na - r largest go — all within the window and the batch. Counts how many of them
// are Rh's, B's and the batch's (each array loses its own largest).
__device__ __forceinline__ void split_pops(float wd, int wi, int wsrc, int wn, const float* sd, const int* si, int na,
                                           int npop, int& pop_r, int& pop_b, int& pop_a, int lane) {
    pop_r = pop_b = pop_a = 0;
    if (npop <= 0) return;
    float ad = INFINITY; int aid = INT_MAX;
    if (lane < na) { ad = sd[lane]; aid = si[lane]; }
    int rkw = lane, rka = lane;
    for (int o = 0; o < na; ++o) rkw += lt_de(sd[o], si[o], wd, wi) ? 1 : 0;
    for (int o = 0; o < wn; ++o) {
        const float od = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wd), o));
        rka += lt_de(od, __builtin_amdgcn_readlane(wi, o), ad, aid) ? 1 : 0;
    }
    const int cut = wn + na - npop;
    pop_r = __popcll(__ballot(lane < wn && rkw >= cut && wsrc == 0));
    pop_b = __popcll(__ballot(lane < wn && rkw >= cut && wsrc != 0));
    pop_a = __popcll(__ballot(lane < na && rka >= cut));
}

// Move the sorted buffer (bd, bi)[0..nb) (ids may carry the expanded flag) into Rh (rd, ri)[0..rs)
// in global memory, keeping all rs + nb entries: one walk down Rh from the top, MG chunks read
// before any is written (entries only move right, so a group's writes never land on the next
// group's unread entries). Rh entry j moves right by #{B entries before it}; B entry b lands at
// b + #{Rh entries before it}, found while walking the chunk that holds it. The walk stops once
// every B entry is placed. Returns the position of B's smallest entry (nothing below it moved).
template <int MG>
__device__ int flush_into_r(float* rd, int* ri, int rs, const float* bd, const int* bi, int nb, int lane) {
    int pb = nb;  // B entries [pb, nb) are placed
    int low = rs + nb;
    for (int top = ((rs - 1) / 64) * 64; rs > 0 && top >= 0 && pb > 0; top -= 64 * MG) {
        float vd[MG];
        int vi[MG];
#pragma unroll
        for (int g = 0; g < MG; ++g) {
            const int j = top - 64 * g + lane;
            vd[g] = INFINITY; vi[g] = INT_MAX;
            if (top - 64 * g >= 0 && j < rs) { vd[g] = rd[j]; vi[g] = ri[j]; }
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int g = 0; g < MG; ++g) {
            const int base = top - 64 * g;
            if (base < 0 || pb == 0) break;  // wave-uniform
            const int j = base + lane;
            const bool valid = j < rs;
            const int vm = vi[g] & ID_MASK;
            const float c0d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(vd[g]), 0));
            const int c0i = __builtin_amdgcn_readlane(vm, 0);
            int before = 0;  // B entries placed in this chunk that precede my entry
            while (pb > 0) {
                const float b_d = bd[pb - 1];
                const int b_i = bi[pb - 1], b_m = b_i & ID_MASK;
                if (!lt_de(c0d, c0i, b_d, b_m)) break;  // it precedes the chunk's first entry: lower
                const int pos = (pb - 1) + base + __popcll(__ballot(valid && lt_de(vd[g], vm, b_d, b_m)));
                before += (valid && lt_de(b_d, b_m, vd[g], vm)) ? 1 : 0;
                if (lane == 0) { rd[pos] = b_d; ri[pos] = b_i; }
                low = pos;
                --pb;
            }
            const int sh = pb + before;  // every remaining B entry precedes the chunk
            if (valid && sh > 0) { rd[j + sh] = vd[g]; ri[j + sh] = vi[g]; }
        }
        __builtin_amdgcn_wave_barrier();
    }
    for (int b = lane; b < pb; b += 64) { rd[b] = bd[b]; ri[b] = bi[b]; }  // below every Rh entry
    if (pb > 0) low = 0;
    __builtin_amdgcn_wave_barrier();
    return low;
}

// distance between two stored rows, reference scalar order (distance.rs)
template <int METRIC>
__device__ __forceinline__ float pair_dist(const float* __restrict__ a, const float* __restrict__ b, int d, float na,
                                           float nb, float curv = 1.0f) {
    return row_dist<METRIC, true>(a, b, d, na, nb, curv);
}

}  // namespace hnswdev
}  // namespace rvx
