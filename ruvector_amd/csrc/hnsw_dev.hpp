// hnsw_dev.hpp — device helpers shared by the HNSW search (k_hnsw.hip) and
// build (k_hnsw_build.hip) kernels: exact-order distances, the tagged visited
// hash and wave-parallel sorted inserts.
#pragma once
#include <hip/hip_runtime.h>

#include "poincare_dev.hpp"
#include "rvx/rvx.h"

namespace rvx {
namespace hnswdev {

constexpr int VCAP_MIN = 32768;  // visited-set slots per query (power of two), grown with ef
constexpr int C_EXTRA = 128; // candidate capacity = ef + C_EXTRA

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
constexpr int ROW_BATCH = 8;  // float4s per batch

template <int METRIC, bool Q_GLOBAL>
__device__ __forceinline__ float stream_acc(const float* __restrict__ qs, const float* __restrict__ x, int n4) {
    const float4* r = reinterpret_cast<const float4*>(x);
    const float4* qq = reinterpret_cast<const float4*>(qs);
    float acc = 0.0f;
    float4 xa[ROW_BATCH], xb[ROW_BATCH], qa[Q_GLOBAL ? ROW_BATCH : 1], qb[Q_GLOBAL ? ROW_BATCH : 1];
    auto load = [&](float4* xv, float4* qv, int base) {
#pragma unroll
        for (int j = 0; j < ROW_BATCH; ++j)
            if (base + j < n4) {
                xv[j] = r[base + j];
                if constexpr (Q_GLOBAL) qv[j] = qq[base + j];
            }
    };
    auto run = [&](const float4* xv, const float4* qv, int base) {
#pragma unroll
        for (int j = 0; j < ROW_BATCH; ++j)
            if (base + j < n4) acc = acc4<METRIC>(acc, Q_GLOBAL ? qv[j] : qq[base + j], xv[j]);
    };
    load(xa, qa, 0);
    for (int base = 0; base < n4; base += 2 * ROW_BATCH) {
        load(xb, qb, base + ROW_BATCH);
        run(xa, qa, base);
        load(xa, qa, base + 2 * ROW_BATCH);
        run(xb, qb, base + ROW_BATCH);
    }
    return acc;
}

// curv: the Poincaré curvature (RVX_METRIC_POINCARE only: HyperbolicHnsw::distance,
// fused norms + poincare_distance_from_norms, hnsw.rs:173-180)
template <int METRIC, bool Q_GLOBAL = false>
__device__ __forceinline__ float row_dist(const float* __restrict__ qs, const float* __restrict__ x, int d, float qn,
                                          float xn, float curv = 1.0f) {
    if constexpr (METRIC == RVX_METRIC_POINCARE) return pdev::hyp_dist(qs, x, d, curv);
    float acc = 0.0f;
    if ((d & 3) == 0) {
        acc = stream_acc<METRIC, Q_GLOBAL>(qs, x, d >> 2);
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

// Claim `node` in a query's visited set: true if it was not visited yet.
// Slots whose tag is another query's are free (the table is zeroed per launch).
__device__ __forceinline__ bool visit_claim(unsigned long long* vis, unsigned vmask, unsigned long long qtag, int node) {
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
    return false;  // table full: cannot happen below vmask+1 visited nodes
}

// visited-table size for a search of width ef (load factor well below 1/2)
inline unsigned visited_capacity(int ef) {
    unsigned v = VCAP_MIN;
    // a search of width ef expands ~ef..2ef nodes of <= 64 neighbours each
    while (v < (unsigned)ef * 256u && v < (1u << 23)) v <<= 1;
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


// distance between two stored rows, reference scalar order (distance.rs)
template <int METRIC>
__device__ __forceinline__ float pair_dist(const float* __restrict__ a, const float* __restrict__ b, int d, float na,
                                           float nb, float curv = 1.0f) {
    return row_dist<METRIC, true>(a, b, d, na, nb, curv);
}

}  // namespace hnswdev
}  // namespace rvx
