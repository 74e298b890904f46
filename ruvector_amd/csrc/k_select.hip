// k_select.hip — exact top-k of long rows of distances for any k (K12).
//
// FlatIndex::search sorts every (id, distance) pair and truncates to k
// (crates/ruvector-core/src/index/flat.rs:63-64); search_with_pruning sorts its
// candidates by exact distance and truncates (crates/ruvector-hyperbolic-hnsw/src/
// hnsw.rs:476-486). Neither bounds k. The list-based scans (K1, K10) keep a per-query
// list of at most SCAN_MAX_K entries; beyond that the distances of a query batch are
// written out whole (K1's tile loop, k_scan.hip) and this file selects from them:
//
//  1. key(row) = (order-preserving bits of the distance, -0.0 as +0.0) << 32 | position:
//     unique per row and ordered exactly as (distance, id) — the reference's order with
//     ties by id, as K1 and the oracle break them. NaN distances are no candidates
//     (K1 never admits them either).
//  2. Radix select of the k-th smallest key: up to six passes of 11/11/10/11/11/10 bits.
//     Each pass histograms the digit of the rows whose key matches the prefix chosen so
//     far (LDS histogram per block, flushed with one atomic per non-empty bin), and one
//     block per query picks the digit where the running count crosses k. A query is done
//     as soon as the chosen digit's bin holds exactly the rows still needed (usually
//     after the distance bits), or when fewer than k rows are valid (all are taken).
//  3. The rows with key <= the chosen prefix (exactly min(k, valid)) are compacted and
//     sorted: a bitonic sort in LDS for k <= 8192, rocPRIM's segmented radix sort above.
//  4. Output in (distance, position) order: the distance bits re-read from the row (so a
//     -0.0 stays -0.0), the id = position + id_offset or idmap[query][position].
// Bytes per query and pass: 4 B per row read (the passes stop early), plus the
// compaction's read; the distance rows are written once by the producer.
#include <rocprim/device/device_segmented_radix_sort.hpp>

#include "common.hpp"
#include "graph.hpp"
#include "scan.hpp"

namespace rvx {
namespace {

constexpr int SEL_BINS = 2048;
constexpr int SEL_PASSES = 6;
constexpr int SEL_WIDTH[SEL_PASSES] = {11, 11, 10, 11, 11, 10};
constexpr int SEL_LDS_SORT_MAX = 8192;

struct SelState {
    unsigned long long prefix;  // the chosen top `bits` bits of the k-th key
    int bits;
    int need;  // rows still to take among those matching the prefix
    int done;
    int all;   // fewer valid rows than k: every valid row is selected
};

__device__ __forceinline__ uint32_t ord_key(float d) {
    const uint32_t b = __float_as_uint(d == 0.0f ? 0.0f : d);  // -0.0 ties +0.0 (then by id)
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__device__ __forceinline__ unsigned long long row_key(float d, int64_t pos) {
    return ((unsigned long long)ord_key(d) << 32) | (unsigned long long)(uint32_t)pos;
}

__global__ void k_sel_init(SelState* st, int64_t nseg, int k) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s < nseg) st[s] = SelState{0ull, 0, k, 0, 0};
}

__global__ __launch_bounds__(256) void k_sel_hist(const float* __restrict__ D, int64_t len, int64_t ld,
                                                  const SelState* __restrict__ st, unsigned* __restrict__ hist,
                                                  int width, int64_t chunk) {
    __shared__ unsigned lh[SEL_BINS];
    const int64_t seg = blockIdx.y;
    const SelState s = st[seg];
    if (s.done) return;  // uniform over the block
    for (int i = threadIdx.x; i < SEL_BINS; i += 256) lh[i] = 0u;
    __syncthreads();
    const int shift = 64 - s.bits - width;
    const unsigned mask = (1u << width) - 1u;
    const float* row = D + seg * ld;
    const int64_t b = (int64_t)blockIdx.x * chunk, e = min(len, b + chunk);
    for (int64_t i = b + threadIdx.x; i < e; i += 256) {
        const float d = row[i];
        if (d != d) continue;
        const unsigned long long key = row_key(d, i);
        if (s.bits > 0 && (key >> (64 - s.bits)) != s.prefix) continue;
        atomicAdd(&lh[(unsigned)(key >> shift) & mask], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i <= (int)mask; i += 256)
        if (lh[i]) atomicAdd(&hist[seg * SEL_BINS + i], lh[i]);
}

// One block per query: the digit whose bin holds the need-th row of the prefix class.
__global__ __launch_bounds__(256) void k_sel_choose(unsigned* __restrict__ hist, SelState* __restrict__ st, int width,
                                                    int first) {
    __shared__ unsigned sc[256];
    __shared__ unsigned pick[3];  // digit, rows below it, rows in it
    const int64_t seg = blockIdx.x;
    const int tid = threadIdx.x;
    const SelState s = st[seg];
    if (s.done) return;
    unsigned* h = hist + seg * SEL_BINS;
    const int per = (1 << width) / 256;  // 8 or 4 bins per thread
    unsigned loc[8];
    unsigned sum = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        loc[j] = j < per ? h[tid * per + j] : 0u;
        sum += loc[j];
    }
    sc[tid] = sum;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // inclusive scan (Hillis-Steele)
        const unsigned v = tid >= o ? sc[tid - o] : 0u;
        __syncthreads();
        sc[tid] += v;
        __syncthreads();
    }
    const unsigned total = sc[255];
    const unsigned excl = sc[tid] - sum;
    const unsigned need = (unsigned)s.need;
    if (first && total <= need) {  // at most k valid rows: take them all
        if (tid == 0) {
            SelState t = s;
            t.done = 1;
            t.all = 1;
            st[seg] = t;
        }
    } else {
        if (excl < need && need <= excl + sum) {
            unsigned c = excl;
            for (int j = 0; j < per; ++j) {
                if (c + loc[j] >= need) {
                    pick[0] = (unsigned)(tid * per + j);
                    pick[1] = c;
                    pick[2] = loc[j];
                    break;
                }
                c += loc[j];
            }
        }
        __syncthreads();
        if (tid == 0) {
            SelState t = s;
            t.prefix = (t.prefix << width) | pick[0];
            t.bits += width;
            t.need -= (int)pick[1];
            t.done = ((unsigned)t.need == pick[2] || t.bits >= 64) ? 1 : 0;
            st[seg] = t;
        }
    }
    for (int j = 0; j < per; ++j) h[tid * per + j] = 0u;  // ready for the next pass
}

__global__ __launch_bounds__(256) void k_sel_compact(const float* __restrict__ D, int64_t len, int64_t ld,
                                                     const SelState* __restrict__ st, int* __restrict__ cnt,
                                                     unsigned long long* __restrict__ sel, int k, int64_t chunk) {
    const int64_t seg = blockIdx.y;
    const SelState s = st[seg];
    const float* row = D + seg * ld;
    const int64_t b = (int64_t)blockIdx.x * chunk, e = min(len, b + chunk);
    for (int64_t i = b + threadIdx.x; i < e; i += 256) {
        const float d = row[i];
        if (d != d) continue;
        const unsigned long long key = row_key(d, i);
        if (s.all || (key >> (64 - s.bits)) <= s.prefix) {
            const int slot = atomicAdd(&cnt[seg], 1);
            if (slot < k) sel[seg * (int64_t)k + slot] = key;  // (k here: the key stride min(k, len))
        }
    }
}

__device__ __forceinline__ void sel_emit(const float* D, int64_t len, int64_t ld, const int64_t* idmap, int64_t id_offset,
                                         int64_t seg, int s, int n, unsigned long long key, int k, float* out_d,
                                         int64_t* out_i) {
    if (s < n) {
        const int64_t pos = (int64_t)(key & 0xFFFFFFFFull);
        out_d[seg * k + s] = D[seg * ld + pos];
        out_i[seg * k + s] = idmap ? idmap[seg * len + pos] : pos + id_offset;
    } else {
        out_d[seg * k + s] = INFINITY;
        out_i[seg * k + s] = INT64_MAX;
    }
}

// One block per query: bitonic sort of its selected keys in LDS (P = power of two >= ks, the
// key stride min(k, len); k output slots, those past the selected count padded).
__global__ __launch_bounds__(1024) void k_sel_sort(const float* __restrict__ D, int64_t len, int64_t ld,
                                                   const int* __restrict__ cnt, const unsigned long long* __restrict__ sel,
                                                   int k, int ks, int P, const int64_t* __restrict__ idmap,
                                                   int64_t id_offset, float* __restrict__ out_d,
                                                   int64_t* __restrict__ out_i, int32_t* __restrict__ out_n) {
    extern __shared__ unsigned long long sk[];
    const int64_t seg = blockIdx.x;
    const int tid = threadIdx.x;
    const int n = min(cnt[seg], ks);
    for (int i = tid; i < P; i += 1024) sk[i] = i < n ? sel[seg * (int64_t)ks + i] : ~0ull;
    __syncthreads();
    for (int size = 2; size <= P; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = tid; t < P / 2; t += 1024) {
                const int i = 2 * t - (t & (stride - 1));
                const int j = i + stride;
                const unsigned long long a = sk[i], b = sk[j];
                if ((a > b) == ((i & size) == 0)) { sk[i] = b; sk[j] = a; }
            }
            __syncthreads();
        }
    for (int s = tid; s < k; s += 1024) sel_emit(D, len, ld, idmap, id_offset, seg, s, n, s < n ? sk[s] : 0ull, k, out_d, out_i);
    if (tid == 0 && out_n) out_n[seg] = n;
}

// Large k: keys sorted by rocPRIM (stride ks = min(k, len)); unused slots were filled with ~0
// (sorted last); k output slots per query.
__global__ void k_sel_emit(const float* __restrict__ D, int64_t len, int64_t ld, const int* __restrict__ cnt,
                           const unsigned long long* __restrict__ sorted, int64_t nseg, int k, int ks,
                           const int64_t* __restrict__ idmap, int64_t id_offset, float* __restrict__ out_d,
                           int64_t* __restrict__ out_i, int32_t* __restrict__ out_n) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nseg * k) return;
    const int64_t seg = t / k;
    const int s = (int)(t - seg * k);
    const int n = min(cnt[seg], ks);
    sel_emit(D, len, ld, idmap, id_offset, seg, s, n, s < n ? sorted[seg * (int64_t)ks + s] : 0ull, k, out_d, out_i);
    if (s == 0 && out_n) out_n[seg] = n;
}

__global__ void k_fill_tail(unsigned long long* sel, const int* cnt, int64_t nseg, int k) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nseg * k) return;
    const int64_t seg = t / k;
    if ((int)(t - seg * k) >= cnt[seg]) sel[t] = ~0ull;
}

__global__ void k_seg_offsets(unsigned* off, int64_t nseg, int k) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= nseg) off[i] = (unsigned)(i * k);
}

}  // namespace

void select_topk(const float* D, int64_t nseg, int64_t len, int64_t ld, int k, const int64_t* idmap, int64_t id_offset,
                 float* out_d, int64_t* out_i, int32_t* out_n) {
    if (nseg <= 0 || k <= 0) return;
    RVX_REQUIRE(len >= 0 && len < ((int64_t)1 << 32) && ld >= len, RVX_ERR_INVALID_PARAMETER,
                "select_topk: rows of up to 2^32 entries");
    // keys per query: at most min(k, len) rows can be selected (k > len sized the key
    // buffers by k); the outputs keep k slots per query, padded
    const int ks = (int)std::max<int64_t>(1, std::min<int64_t>(k, len));
    RVX_REQUIRE(nseg * (int64_t)ks < ((int64_t)1 << 31), RVX_ERR_INVALID_PARAMETER, "select_topk: batch too large");
    auto* st = (SelState*)scratch_bytes("sel_state", nseg * (int64_t)sizeof(SelState));
    auto* hist = (unsigned*)scratch_bytes("sel_hist", nseg * SEL_BINS * 4);
    auto* cnt = (int*)scratch_bytes("sel_cnt", nseg * 4);
    auto* sel = (unsigned long long*)scratch_bytes("sel_keys", nseg * (int64_t)ks * 8);
    RVX_HIP(hipMemsetAsync(hist, 0, (size_t)nseg * SEL_BINS * 4, stream()));
    RVX_HIP(hipMemsetAsync(cnt, 0, (size_t)nseg * 4, stream()));
    RVX_LAUNCH("select_topk", k_sel_init, dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0, st, nseg, k);
    // blocks per query: >= 16 rows per thread, ~4096 blocks over the batch
    const int64_t per_block = std::max<int64_t>(256 * 16, (len * nseg + 4095) / 4096);
    const int64_t bx = std::max<int64_t>(1, (len + per_block - 1) / per_block);
    const int64_t chunk = (len + bx - 1) / bx;
    for (int64_t s0 = 0; s0 < nseg; s0 += 65535) {  // grid.y limit
        const int64_t ns = std::min<int64_t>(65535, nseg - s0);
        for (int p = 0; p < SEL_PASSES; ++p) {
            RVX_LAUNCH("select_topk", k_sel_hist, dim3((unsigned)bx, (unsigned)ns), dim3(256), 0, D + s0 * ld, len, ld,
                       st + s0, hist + s0 * SEL_BINS, SEL_WIDTH[p], chunk);
            RVX_LAUNCH("select_topk", k_sel_choose, dim3((unsigned)ns), dim3(256), 0, hist + s0 * SEL_BINS, st + s0,
                       SEL_WIDTH[p], p == 0 ? 1 : 0);
        }
        RVX_LAUNCH("select_topk", k_sel_compact, dim3((unsigned)bx, (unsigned)ns), dim3(256), 0, D + s0 * ld, len, ld,
                   st + s0, cnt + s0, sel + s0 * ks, ks, chunk);
    }
    if (ks <= SEL_LDS_SORT_MAX) {
        int P = 2;
        while (P < ks) P <<= 1;
        static bool attr = false;
        if (!attr) {
            RVX_HIP(hipFuncSetAttribute((const void*)k_sel_sort, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        SEL_LDS_SORT_MAX * 8));
            attr = true;
        }
        for (int64_t s0 = 0; s0 < nseg; s0 += 65535) {
            const int64_t ns = std::min<int64_t>(65535, nseg - s0);
            RVX_LAUNCH("select_topk", k_sel_sort, dim3((unsigned)ns), dim3(1024), (size_t)P * 8, D + s0 * ld, len, ld,
                       cnt + s0, sel + s0 * ks, k, ks, P, idmap ? idmap + s0 * len : nullptr, id_offset,
                       out_d + s0 * k, out_i + s0 * k, out_n ? out_n + s0 : nullptr);
        }
        return;
    }
    // k > 8192: slots past each query's count to ~0 (sorted last), rocPRIM's segmented
    // radix sort, then decode
    const int64_t tot = nseg * (int64_t)ks;
    auto* sorted = (unsigned long long*)scratch_bytes("sel_sorted", tot * 8);
    auto* off = (unsigned*)scratch_bytes("sel_offsets", (nseg + 1) * 4);
    RVX_LAUNCH("select_topk", k_seg_offsets, dim3((unsigned)((nseg + 1 + 255) / 256)), dim3(256), 0, off, nseg, ks);
    RVX_LAUNCH("select_topk", k_fill_tail, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, sel, cnt, nseg, ks);
    size_t tmp_bytes = 0;
    RVX_HIP(rocprim::segmented_radix_sort_keys(nullptr, tmp_bytes, sel, sorted, (unsigned)tot, (unsigned)nseg, off,
                                               off + 1, 0, 64, stream()));
    void* tmp = scratch_bytes("sel_rocprim_tmp", (int64_t)std::max<size_t>(tmp_bytes, 16));
    {
        ProfScope ps("select_topk_sort");
        RVX_HIP(rocprim::segmented_radix_sort_keys(tmp, tmp_bytes, sel, sorted, (unsigned)tot, (unsigned)nseg, off,
                                                   off + 1, 0, 64, stream()));
    }
    const int64_t outs = nseg * (int64_t)k;
    RVX_LAUNCH("select_topk", k_sel_emit, dim3((unsigned)((outs + 255) / 256)), dim3(256), 0, D, len, ld, cnt, sorted,
               nseg, k, ks, idmap, id_offset, out_d, out_i, out_n);
}

}  // namespace rvx
