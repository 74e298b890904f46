// k_hnsw.hip — batched HNSW search on a fixed graph (one wave per query).
//
// Semantics are those of hnsw_rs 0.3.3 as vendored in the reference:
//   Hnsw::search -> search_filter  (patches/hnsw_rs/src/hnsw.rs:1475-1589)
//     upper layers: ONE pass over the pivot's neighbour list per layer, the
//     pivot moves to the first neighbour with the smallest distance below the
//     running best (:1499-1517) — no iterated hill climb;
//     layer 0: search_layer(ef = max(ef_arg, k)) (:1519-1523)
//   search_layer (:913-1055): pop the nearest candidate c; stop when
//     d(c) > d(farthest result); for each neighbour e of c in stored order that
//     is not yet visited: mark visited, admit iff d(e) < d(farthest) or
//     |R| < ef, push to candidates and results, pop the farthest when |R| > ef.
//   into_sorted_vec + first min(k, ef, |R|) (:1532-1568).
// Distances use the reference's scalar accumulation order (see k_scan.hip), so
// on the same graph the returned ids and distances are bit-exact. The
// reference orders heap ties by distance only (:272-296); here ties are
// broken by node id, and the stop test compares (d, id) pairs (a measure-zero
// difference on real data; the oracle's search uses the same rule).
//
// Per query: the result set R as an ascending sorted array (farthest last) in
// LDS, each id's bit 31 marking an expanded entry; there is no candidate
// array — the nearest candidate is the nearest unexpanded entry of R
// (hnsw_dev.hpp merge_into_r). One expansion's fresh neighbours are admitted
// by exact sequential decisions in registers (decide_batch) and ONE merge
// into R whose cost grows with the entries behind the first insertion only.
// The visited set is an open-addressing hash in a per-wave global scratch slot
// (CAS-claimed by all lanes at once); neighbour distances are one row per lane.
#include <cstring>
#include <map>

#include "common.hpp"
#include "graph.hpp"
#include "hnsw.hpp"
#include "hnsw_dev.hpp"

namespace rvx {
namespace {
using namespace hnswdev;

struct SearchArgs {
    HnswDev g;
    const float* x; const float* xnorm; int d;
    const float* q; const float* qnorm; int64_t nq;
    int k, ef;
    unsigned long long* visited;  // [nslots][vcap] {query tag, node+1}, zeroed per launch
    unsigned* vbits;   // small tables: [nslots][vwords] visited bitmap, zeroed per query (else nullptr)
    int64_t vwords;    // words per slot, a multiple of 4
    int nslots;
    unsigned vcap;
    float* out_d; int64_t* out_i; int32_t* out_n;  // [nq][k]
    int* status;       // unused (the R-only search cannot overflow)
    unsigned long long* stats;  // [2]: distance evaluations, layer-0 expansions (per launch)
    float curv;        // Poincaré curvature
    int hyper;         // HyperbolicHnsw::search semantics (see below)
    int coop;          // wave-cooperative LDS-staged distances (hnsw_dev.hpp wave_dist)
    float* rg_d;       // RG kernels: R in HBM, [nslots][ef + 1] distances ...
    int* rg_i;         // ... and flagged ids (ef past one wave's LDS)
    int par_decide;    // hnsw_dev.hpp decide_par where R is in LDS
    int rg_buf;        // RG: R's admissions buffered in LDS (hnsw_dev.hpp RB_CAP); 0 = merge into HBM per batch
    int collect;       // layer-0 lists of <= FRESH_CAP claimed whole, fresh neighbours batched (collect_fresh)
};

// Diagnostic build only (-DRVX_HNSW_PHASES, scripts/exp/build_variant.sh): shader-clock cycles
// of each layer-0 phase summed over waves into stats[2..7] — 0 find the next unexpanded entry,
// 1 claim neighbours, 2 distances, 3 admission decisions + batch sort, 4 merge into R.
#ifdef RVX_HNSW_PHASES
#define PH_MARK(k)                                              \
    do {                                                        \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        ph[k] += t_ - ph_t;                                     \
        ph_t = t_;                                              \
    } while (0)
#else
#define PH_MARK(k) do {} while (0)
#endif

// RB: float4s per streamed row batch of the per-lane distances (hnsw_dev.hpp
// stream_acc); NST: LDS stages of the wave-cooperative distances. RG: the result list R
// lives in a per-slot HBM scratch row instead of LDS (ef beyond what one wave's 160 KB
// hold: 19,007 entries at d 768): the same code over global memory, with a workgroup
// fence after each write phase so the other lanes' reads see it.
// QG (LDS-staged distances only): the query is read from global memory through the constant
// address space (hnsw_dev.hpp wd_chunk QC) instead of being staged in LDS.
template <int METRIC, int RB, int NST = 2, bool RG = false, bool QG = false>
__device__ __forceinline__ void search_body(const SearchArgs& a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    const int lane = threadIdx.x;
    const int ef = a.ef;
    constexpr bool COOP_OK = METRIC != RVX_METRIC_POINCARE && METRIC != RVX_METRIC_HYP_L2;
    const bool coop = COOP_OK && (QG || a.coop);
    unsigned char* wst = lds_raw;                                // [NST * WD_STAGE] distance stages (coop)
    float* qs_l = reinterpret_cast<float*>(lds_raw + (coop ? wd_lds(NST) : 0));  // [d rounded to 4]
    const int dq = QG ? 0 : (a.d + 3) & ~3;
    float* qs = qs_l;
    float* rd;                                                  // R dist [ef+1]
    int* ri;                                                    // R id | expanded flag (bit 31)
    float* sdb;                                                 // admitted batch [64]
    if constexpr (RG) {
        rd = a.rg_d + (int64_t)blockIdx.x * (ef + 1);
        ri = a.rg_i + (int64_t)blockIdx.x * (ef + 1);
        sdb = qs_l + dq;
    } else {
        rd = qs_l + dq;
        ri = reinterpret_cast<int*>(rd + ef + 1);
        sdb = reinterpret_cast<float*>(ri + ef + 1);
    }
    int* sib = reinterpret_cast<int*>(sdb + 64);
    int* srk = sib + 64;  // the admitted batch's ranks in R (decide_par; R in LDS); RG: window origins
    float* bfd = reinterpret_cast<float*>(srk + 64);  // RG: R's LDS buffer (hnsw_dev.hpp RB_CAP) ...
    int* bfi = reinterpret_cast<int*>(bfd + RB_CAP);   // ... and its flagged ids
    int* frs = RG ? bfi + RB_CAP : srk + 64;           // an expansion's fresh neighbours [FRESH_CAP]

    unsigned long long* vis = a.vbits ? nullptr : a.visited + (int64_t)blockIdx.x * a.vcap;
    const unsigned vmask = a.vcap - 1;
    unsigned* vb = a.vbits ? a.vbits + (int64_t)blockIdx.x * a.vwords : nullptr;

    unsigned long long n_dist = 0, n_expand = 0;  // lane 0's tallies for this wave
#ifdef RVX_HNSW_PHASES
    unsigned long long ph[5] = {0, 0, 0, 0, 0}, ph_t = __builtin_amdgcn_s_memtime();
#endif
    for (int64_t qi = blockIdx.x; qi < a.nq; qi += a.nslots) {
        const unsigned long long qtag = (unsigned long long)(qi + 1) << 32;
        if constexpr (QG) qs = const_cast<float*>(a.q) + qi * a.d;  // (read only)
        for (int i = lane; i < dq; i += 64) qs[i] = (i < a.d) ? a.q[qi * a.d + i] : 0.0f;
        if (vb)  // this query's bitmap starts empty
            for (int64_t w = 4 * lane; w < a.vwords; w += 256) *reinterpret_cast<uint4*>(vb + w) = make_uint4(0, 0, 0, 0);
        __threadfence_block();  // (also orders the clears before this wave's claims)
        __builtin_amdgcn_wave_barrier();
        const float qn = (METRIC == RVX_METRIC_COSINE) ? a.qnorm[qi] : 0.0f;
        // claim node in this query's visited set: true if it was not visited yet
        auto claim = [&](int node) -> bool {
            if (vb) {
                const unsigned bit = 1u << (node & 31);
                return !(atomicOr(vb + (node >> 5), bit) & bit);
            }
            return visit_claim(vis, vmask, qtag, node, reinterpret_cast<int*>(a.stats + 7));
        };
        auto dist_of = [&](int node) {
            return row_dist<METRIC, false, RB>(qs, a.x + (int64_t)node * a.d, a.d,
                                    qn, METRIC == RVX_METRIC_COSINE ? a.xnorm[node] : 0.0f, a.curv);
        };
        // every lane calls; node < 0: no row (INFINITY)
        auto dist_lane = [&](int node) {
            float dv;
            if constexpr (COOP_OK) {
                if (coop) {
                    dv = wave_dist<METRIC, NST, QG>(qs, a.x, a.d, node, qn,
                                           (METRIC == RVX_METRIC_COSINE && node >= 0) ? a.xnorm[node] : 0.0f, wst, lane);
                    return node >= 0 ? dv : INFINITY;
                }
            }
            return node >= 0 ? dist_of(node) : INFINITY;
        };
        // Claim a whole layer-0 list (up to FRESH_CAP neighbours, the loads and claims of its
        // 64-entry slices issued back to back) and compact the fresh neighbours into frs in list
        // order: the admissions then take batches of up to 64 FRESH neighbours, one distance
        // pass each, instead of one pass per 64-entry slice of the list (M 128: 256-entry lists,
        // ~55 fresh per expansion at high ef — one pass instead of four). Claims do not depend on
        // admissions, so the admissions see the same neighbours in the same order.
        auto collect_fresh = [&](int64_t b, int64_t e) -> int {
            int nids[FRESH_CAP / 64];
            bool fr[FRESH_CAP / 64];
#pragma unroll
            for (int sl = 0; sl < FRESH_CAP / 64; ++sl) {
                const int64_t p = b + 64 * sl + lane;
                nids[sl] = p < e ? a.g.col0[p] : -1;
            }
#pragma unroll
            for (int sl = 0; sl < FRESH_CAP / 64; ++sl) fr[sl] = nids[sl] >= 0 && claim(nids[sl]);
            int nf = 0;
#pragma unroll
            for (int sl = 0; sl < FRESH_CAP / 64; ++sl) {
                const unsigned long long m = __ballot(fr[sl]);
                const int before = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                if (fr[sl]) frs[nf + before] = nids[sl];
                nf += __popcll(m);
            }
            __builtin_amdgcn_wave_barrier();
            return nf;
        };

        // ---- upper layers: single pass per layer (search_filter :1499-1517)
        int pivot = (int)a.g.entry;
        float best = dist_of(pivot);
        for (int l = a.g.max_level; l >= 1; --l) {
            // locate pivot in layer l's sorted id list
            const int* ids = a.g.up_ids + a.g.up_ids_off[l];
            const int64_t cnt = a.g.up_count[l];
            int64_t lo = 0, hi = cnt;
            while (lo < hi) { const int64_t mid = (lo + hi) >> 1; if (ids[mid] < pivot) lo = mid + 1; else hi = mid; }
            if (lo >= cnt || ids[lo] != pivot) continue;  // pivot not on this layer (cannot happen for a valid graph)
            const int64_t* rp = a.g.up_rp + a.g.up_rp_off[l];
            const int* col = a.g.up_col + a.g.up_col_off[l];
            bool moved;
            do {
                const int64_t b = rp[lo], e = rp[lo + 1];
                int new_pivot = pivot;
                float new_best = best;
                for (int64_t c0 = b; c0 < e; c0 += 64) {
                    const int64_t p = c0 + lane;
                    int pos = INT_MAX, nid = -1;
                    if (p < e) { nid = col[p]; pos = (int)(p - b); }
                    float dd = dist_lane(nid);
                    n_dist += (unsigned long long)min<int64_t>(64, e - c0);
                    // first position holding the minimum of this chunk
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) {
                        const float od = __shfl_xor(dd, o);
                        const int op = __shfl_xor(pos, o), on = __shfl_xor(nid, o);
                        if (od < dd || (od == dd && op < pos)) { dd = od; pos = op; nid = on; }
                    }
                    if (dd < new_best) { new_best = dd; new_pivot = nid; }
                }
                moved = new_pivot != pivot;
                pivot = new_pivot;
                best = new_best;
                // HyperbolicHnsw::search_layer_single (hnsw.rs:305-329) repeats the
                // pass from the new pivot until nothing improves
                if (moved && a.hyper) {
                    lo = 0; hi = cnt;
                    while (lo < hi) { const int64_t mid = (lo + hi) >> 1; if (ids[mid] < pivot) lo = mid + 1; else hi = mid; }
                    if (lo >= cnt || ids[lo] != pivot) break;
                }
            } while (moved && a.hyper);
        }

        // ---- layer 0, R in HBM: R = rd/ri (HBM, sorted) ∪ an LDS buffer (hnsw_dev.hpp RB_CAP):
        // the same set operations as the branch below, with admissions merged into the buffer and
        // the buffer moved into the HBM array when full (flush_into_r)
        if (RG && a.rg_buf) {
            int rs = 1, nb = 0;
            {
                const float d0 = dist_of(pivot);
                if (lane == 0) {
                    rd[0] = d0; ri[0] = pivot;
                    claim(pivot);
                }
                __threadfence_block();
                __builtin_amdgcn_wave_barrier();
            }
            int scan = 0;  // every entry of the HBM array before `scan` is expanded
            for (;;) {
                int at = -1, atb = -1;
                for (int b0 = scan; b0 < rs; b0 += 64) {
                    const unsigned long long m = __ballot(b0 + lane < rs && ri[b0 + lane] >= 0);
                    if (m) { at = b0 + __ffsll((long long)m) - 1; break; }
                }
                for (int b0 = 0; b0 < nb; b0 += 64) {
                    const unsigned long long m = __ballot(b0 + lane < nb && bfi[b0 + lane] >= 0);
                    if (m) { atb = b0 + __ffsll((long long)m) - 1; break; }
                }
                if (at < 0 && atb < 0) break;
                if (at >= 0 && atb >= 0 && lt_de(bfd[atb], bfi[atb], rd[at], ri[at])) at = -1;  // the buffer's is nearer
                int c_id;
                if (at >= 0) {
                    c_id = ri[at];
                    scan = at + 1;
                    __builtin_amdgcn_wave_barrier();
                    if (lane == 0) ri[at] = c_id | INT_MIN;
                    __threadfence_block();
                } else {
                    c_id = bfi[atb];
                    __builtin_amdgcn_wave_barrier();
                    if (lane == 0) bfi[atb] = c_id | INT_MIN;
                }
                __builtin_amdgcn_wave_barrier();
                const int64_t b = a.g.rp0[c_id], e = a.g.rp0[c_id + 1];
                n_expand += 1;
                PH_MARK(0);
                const bool whole = a.collect && e - b <= FRESH_CAP;  // (wave-uniform) else slice by slice
                const int nf = whole ? collect_fresh(b, e) : 0;
                for (int64_t c0 = whole ? 0 : b, c1 = whole ? nf : e; c0 < c1; c0 += 64) {
                    int nid = -1;
                    bool fresh = false;
                    if (whole) {
                        nid = c0 + lane < nf ? frs[c0 + lane] : -1;
                        fresh = nid >= 0;
                    } else if (c0 + lane < e) {
                        nid = a.g.col0[c0 + lane];
                        fresh = claim(nid);
                    }
                    const unsigned long long fmask = __ballot(fresh);
                    PH_MARK(1);
                    if (!fmask) continue;
                    const float dd = dist_lane(fresh ? nid : -1);
                    PH_MARK(2);
                    n_dist += (unsigned long long)__popcll(fmask);
                    float wd;
                    int wi, wsrc, wn, below;
                    union_window(rd, ri, rs, bfd, bfi, nb, sdb, sib, srk, wd, wi, wsrc, wn, below, lane);
                    int r = rs + nb;
                    const unsigned long long adm = decide_window(fmask, dd, nid, ef, wd, wi, wn, below, rs + nb, r, lane);
                    const int na = sort_batch(adm, dd, nid, sdb, sib, lane);
                    PH_MARK(3);
                    if (na == 0) continue;
                    int pop_r, pop_b, pop_a;
                    split_pops(wd, wi, wsrc, wn, sdb, sib, na, rs + nb + na - r, pop_r, pop_b, pop_a, lane);
                    rs -= pop_r;  // each array loses its own largest entries
                    nb -= pop_b;
                    const int keep = na - pop_a;
                    if (keep > 0) {
                        if (nb + keep > RB_CAP) {  // the buffer into the HBM array first
                            scan = min(scan, flush_into_r<RVX_MERGE_RG_G>(rd, ri, rs, bfd, bfi, nb, lane));
                            __threadfence_block();
                            rs += nb;
                            nb = 0;
                        }
                        merge_into_r<RVX_MERGE_LDS_G>(bfd, bfi, nb, sdb, sib, keep, nb + keep, lane);
                        nb += keep;
                    }
                    PH_MARK(4);
                }
            }
            if (nb > 0) {
                flush_into_r<RVX_MERGE_RG_G>(rd, ri, rs, bfd, bfi, nb, lane);
                __threadfence_block();
                __builtin_amdgcn_wave_barrier();
                rs += nb;
            }
            const int take = min(a.k, rs);
            for (int s = lane; s < a.k; s += 64) {
                a.out_d[qi * a.k + s] = s < take ? rd[s] : INFINITY;
                a.out_i[qi * a.k + s] = s < take ? (int64_t)(ri[s] & ID_MASK) : (int64_t)-1;
            }
            if (lane == 0 && a.out_n) a.out_n[qi] = take;
            __builtin_amdgcn_wave_barrier();
            continue;
        }

        // ---- layer 0: search_layer (:913-1055) over R alone (hnsw_dev.hpp
        // merge_into_r): expand the nearest unexpanded entry of R until none is left
        int rs = 1;
        {
            const float d0 = dist_of(pivot);
            if (lane == 0) {
                rd[0] = d0; ri[0] = pivot;
                claim(pivot);
            }
            __threadfence_block();
            __builtin_amdgcn_wave_barrier();
        }
        int scan = 0;  // every entry of R before `scan` is expanded
#ifdef RVX_HNSW_PHASES
        ph_t = __builtin_amdgcn_s_memtime();
#endif
        for (;;) {
            int at = -1;
            for (int b0 = scan; b0 < rs; b0 += 64) {
                const unsigned long long m = __ballot(b0 + lane < rs && ri[b0 + lane] >= 0);
                if (m) { at = b0 + __ffsll((long long)m) - 1; break; }
            }
            if (at < 0) break;
            const int c_id = ri[at];
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) ri[at] = c_id | INT_MIN;
            if constexpr (RG) __threadfence_block();
            __builtin_amdgcn_wave_barrier();
            scan = at + 1;
            const int64_t b = a.g.rp0[c_id], e = a.g.rp0[c_id + 1];
            n_expand += 1;
            PH_MARK(0);
            // (wave-uniform; with R in LDS only for the LDS-staged distances: per-lane distances over
            // R in LDS ran 16% slower batched, 1M x 768 M 128 ef 1,600; profiles/r06_hnsw_collect_ab_1m.log)
            const bool whole = a.collect && coop && e - b <= FRESH_CAP;
            const int nf = whole ? collect_fresh(b, e) : 0;
            for (int64_t c0 = whole ? 0 : b, c1 = whole ? nf : e; c0 < c1; c0 += 64) {
                int nid = -1;
                bool fresh = false;
                if (whole) {
                    nid = c0 + lane < nf ? frs[c0 + lane] : -1;
                    fresh = nid >= 0;
                } else if (c0 + lane < e) {
                    nid = a.g.col0[c0 + lane];
                    fresh = claim(nid);
                }
                const unsigned long long fmask = __ballot(fresh);
                PH_MARK(1);
                if (!fmask) continue;
                const float dd = dist_lane(fresh ? nid : -1);
                PH_MARK(2);
                n_dist += (unsigned long long)__popcll(fmask);
                // admission in neighbour order (hnsw.rs:1004-1046), batched exactly
                int r = rs, rk = 0;
                // R in LDS: admissions decided in parallel (decide_par), the ranks reused by the
                // merge; R in HBM (binary searches there cost round trips) or a NaN distance: the
                // sequential window (RVX_HNSW_PAR_DECIDE=0 keeps it everywhere)
                const bool par = !RG && a.par_decide && !__ballot(((fmask >> lane) & 1ull) && dd != dd);
                const unsigned long long adm = par ? decide_par(fmask, dd, nid, ef, rd, ri, rs, r, rk, lane)
                                                   : decide_batch(fmask, dd, nid, ef, rd, ri, rs, r, lane);
                const int na = sort_batch(adm, dd, nid, sdb, sib, lane, par ? srk : nullptr, rk);
                PH_MARK(3);
                if (na == 0) continue;
                scan = min(scan, merge_into_r<RG ? RVX_MERGE_RG_G : RVX_MERGE_LDS_G>(rd, ri, rs, sdb, sib, na, r, lane,
                                                                                  par ? srk : nullptr));
                if constexpr (RG) __threadfence_block();
                rs = r;
                PH_MARK(4);
            }
        }

        // ---- output: ascending, first min(k, ef, |R|)
        const int take = min(a.k, rs);
        for (int s = lane; s < a.k; s += 64) {
            a.out_d[qi * a.k + s] = s < take ? rd[s] : INFINITY;
            a.out_i[qi * a.k + s] = s < take ? (int64_t)(ri[s] & ID_MASK) : (int64_t)-1;
        }
        if (lane == 0 && a.out_n) a.out_n[qi] = take;  // counts are optional (device entry points)
        __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0 && a.stats) {
        atomicAdd(&a.stats[0], n_dist + 2);  // + the entry point's distance and layer 0's start
        atomicAdd(&a.stats[1], n_expand);
#ifdef RVX_HNSW_PHASES
        for (int k = 0; k < 5; ++k) atomicAdd(&a.stats[2 + k], ph[k]);
#endif
    }
}

#ifndef RVX_HNSW_WPE
#define RVX_HNSW_WPE
#endif
template <int METRIC>
__global__ __launch_bounds__(64) RVX_HNSW_WPE void k_hnsw_search(SearchArgs a) {
    search_body<METRIC, ROW_BATCH>(a);
}
// Short rows (d <= 256, per-lane distances): 4-float4 row batches and at least
// 4 waves per SIMD (117 VGPRs instead of 167 -> 3 waves). C1 100k x 128, ef 600:
// 334k vs 302k QPS; at d = 768 the deeper batches win (1M x 768 ef 800: 52.9k
// vs 47.3k), so they keep the default kernel (scripts/exp_hnsw_occupancy.sh).
template <int METRIC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void k_hnsw_search_short(SearchArgs a) {
    search_body<METRIC, 4>(a);
}
// LDS-staged rows (coop) with NST distance stages other than the default two:
// 1 past ef 1024 (R costs most of the LDS, more waves fit a CU), a deeper ring
// where one wave is alone on its CU (hnsw_nst). Capping it at 3 waves per SIMD
// (151 VGPRs instead of 171) made it slower although LDS sets the waves per CU
// there (4M x 768: ef 1600 22.8k -> 19.5k QPS, ef 3200 8.8k -> 7.4k;
// scripts/exp/exp_hnsw_variants.sh, profiles/r05_hnsw_variants_ab.txt).
#ifndef RVX_ST_WPE
#define RVX_ST_WPE
#endif
template <int METRIC, int NST>
__global__ __launch_bounds__(64) RVX_ST_WPE void k_hnsw_search_st(SearchArgs a) {
    search_body<METRIC, ROW_BATCH, NST>(a);
}
// LDS-staged distances with the query read from global memory (QG): NST 1 / 2, R in LDS or HBM
template <int METRIC, int NST, bool RG>
__global__ __launch_bounds__(64) void k_hnsw_search_qg(SearchArgs a) {
    search_body<METRIC, ROW_BATCH, NST, RG, true>(a);
}
// ef past one wave's LDS: R in HBM (one distance stage when coop). RVX_RG_WPE: occupancy
// attribute for A/B builds (scripts/exp/build_variant.sh).
#ifndef RVX_RG_WPE
#define RVX_RG_WPE
#endif
template <int METRIC, int NST = 1>
__global__ __launch_bounds__(64) RVX_RG_WPE void k_hnsw_search_rg(SearchArgs a) {
    search_body<METRIC, ROW_BATCH, NST, true>(a);
}

}  // namespace

SearchStats g_search_stats;

namespace {
struct SearchTally {
    unsigned long long* host = nullptr;  // [8]: distance evaluations, expansions, (phase cycles), visited overflow
    bool pending = false;
};
SearchTally& search_tally() {  // per device (callers hold its ComputeLock)
    static std::mutex mu;
    static std::map<int, SearchTally> t;
    std::lock_guard<std::mutex> lk(mu);
    SearchTally& s = t[device().id];
    if (!s.host) RVX_HIP(hipHostMalloc((void**)&s.host, 8 * 8, 0));
    return s;
}
}  // namespace

namespace {
template <int NST>
void set_st_attr() {
    RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_st<RVX_METRIC_L2, NST>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_st<RVX_METRIC_COSINE, NST>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_st<RVX_METRIC_DOT, NST>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_st<RVX_METRIC_L1, NST>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
}
template <int NST, bool RG>
void set_qg_attr() {
    RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_qg<RVX_METRIC_L2, NST, RG>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_qg<RVX_METRIC_COSINE, NST, RG>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_qg<RVX_METRIC_DOT, NST, RG>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_qg<RVX_METRIC_L1, NST, RG>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
}
template <int NST, bool RG>
void launch_qg(const char* t, int metric, int nslots, size_t lds, const SearchArgs& a) {
    switch (metric) {
        case RVX_METRIC_L2: RVX_LAUNCH(t, (k_hnsw_search_qg<RVX_METRIC_L2, NST, RG>), dim3(nslots), dim3(64), lds, a); break;
        case RVX_METRIC_COSINE: RVX_LAUNCH(t, (k_hnsw_search_qg<RVX_METRIC_COSINE, NST, RG>), dim3(nslots), dim3(64), lds, a); break;
        case RVX_METRIC_DOT: RVX_LAUNCH(t, (k_hnsw_search_qg<RVX_METRIC_DOT, NST, RG>), dim3(nslots), dim3(64), lds, a); break;
        default: RVX_LAUNCH(t, (k_hnsw_search_qg<RVX_METRIC_L1, NST, RG>), dim3(nslots), dim3(64), lds, a); break;
    }
}
template <int NST>
void launch_st(const char* t, int metric, int nslots, size_t lds, const SearchArgs& a) {
    switch (metric) {
        case RVX_METRIC_L2: RVX_LAUNCH(t, (k_hnsw_search_st<RVX_METRIC_L2, NST>), dim3(nslots), dim3(64), lds, a); break;
        case RVX_METRIC_COSINE: RVX_LAUNCH(t, (k_hnsw_search_st<RVX_METRIC_COSINE, NST>), dim3(nslots), dim3(64), lds, a); break;
        case RVX_METRIC_DOT: RVX_LAUNCH(t, (k_hnsw_search_st<RVX_METRIC_DOT, NST>), dim3(nslots), dim3(64), lds, a); break;
        default: RVX_LAUNCH(t, (k_hnsw_search_st<RVX_METRIC_L1, NST>), dim3(nslots), dim3(64), lds, a); break;
    }
}
}  // namespace

bool hnsw_coop(int metric, int d, int64_t rows) {
    // 0 off, 1 auto (tables past the per-CU translation reach), 2 always
    const int mode = env_int("RVX_HNSW_COOP", 1);  // read per launch: tests force both paths
    const int64_t min_bytes = (int64_t)env_int("RVX_HNSW_COOP_MIN_MB", 4096) << 20;
    if (!mode || metric == RVX_METRIC_POINCARE || metric == RVX_METRIC_HYP_L2 || !wave_dist_ok(d)) return false;
    return mode == 2 || rows * (int64_t)d * 4 >= min_bytes;
}

namespace {
size_t search_lds_nst(int d, int ef, int nst) {
    const int dq = (d + 3) & ~3;
    return (size_t)wd_lds(nst) + (size_t)dq * 4 + (size_t)(ef + 1) * 8 + 64 * 12 + (size_t)FRESH_CAP * 4;
}
}  // namespace

// Distance stages per wave of the LDS-staged (coop) search. RVX_HNSW_NST forces
// 1, 2, 3, 4 or 6 (read per call: tests and A/Bs); by default (RVX_HNSW_WIDE=0: always 2)
// 1 for rows of at most 8 chunks (d <= 256), where a second stage overlaps little within a
// row and costs waves, 1 at ef 1024-1151 up to d 768, else 2 (10k queries, NST 1 vs 2: d 128
// ef 400-3200 +2-21% for 1, ef 100 equal; d 384 ef 1024 +9% for 1, ef 1600 +10% for 2; d 768
// ef 1024 +2% for 1, 1280 / 1408 +5% / +15% for 2; d 1024 ef 1024-2400 +5-38% for 2;
// profiles/r05_hnsw_nst_by_d.txt, r05_hnsw_nst_d128_small_d1024.txt).
int hnsw_nst(bool coop, int d, int ef) {
    if (!coop) return 0;
    const int f = env_int("RVX_HNSW_NST", 0);
    if ((f == 1 || f == 2 || f == 3 || f == 4 || f == 6) && search_lds_nst(d, ef, f) <= 160 * 1024) return f;
    if (!env_int("RVX_HNSW_WIDE", 1)) return 2;
    if (d <= 256) return 1;
    return d <= 768 && ef >= 1024 && ef < 1152 ? 1 : 2;
}

size_t hnsw_search_lds(int d, int ef, bool coop) {
    const int dq = (d + 3) & ~3;
    return (coop ? (size_t)wd_lds(hnsw_nst(coop, d, ef)) : 0) + (size_t)dq * 4 + (size_t)(ef + 1) * 8 + 64 * 12 +
           (size_t)FRESH_CAP * 4;
}
// LDS of the RG kernel: distance stage + query + admitted batch (R is in HBM)
// distance stages of the RG kernel: 1 unless RVX_HNSW_RG_NST=2 (read per call). Round 5 (R merged
// into HBM per batch) preferred 2 (ef 12288: 1134 -> 1266 QPS); with R's LDS admission buffer
// (2.3 KB more LDS per wave) one stage fits 11 waves per CU instead of 7: 1M x 768 M 128 (LDS-staged
// forced) ef 8,192 1,405 -> 1,931 QPS, 12,288 995 -> 1,381; 10M x 768 M 128 (10k queries) within 1%
// either way (1,104 vs 1,097 at ef 12,288; profiles/r06_hnsw_coop_ab_1m.log,
// r06_c3_10m_m128_efc500_forms.log)
int hnsw_rg_nst() { return env_int("RVX_HNSW_RG_NST", 1) == 2 ? 2 : 1; }
size_t hnsw_search_lds_rg(int d, bool coop) {
    const int dq = (d + 3) & ~3;
    // + the union window's scratch (sdb / sib / origins) and R's LDS buffer (RB_CAP entries)
    return (coop ? (size_t)wd_lds(hnsw_rg_nst()) : 0) + (size_t)dq * 4 + 64 * 12 + (size_t)RB_CAP * 8 +
           (size_t)FRESH_CAP * 4;
}

void hnsw_search(const HnswDev& g, int metric, const float* x, const float* xnorm, int d, const float* q,
                 const float* qnorm, int64_t nq, int k, int ef, float* out_d, int64_t* out_i, int32_t* out_n,
                 const char* tag, float curv, int hyper) {
    if (nq <= 0) return;
    RVX_REQUIRE(ef >= 1 && ef <= HNSW_MAX_EF, RVX_ERR_INVALID_PARAMETER,
                "ef must be in [1, " + std::to_string(HNSW_MAX_EF) + "]");
    // R in LDS when one wave's 160 KB hold it, else in HBM. The LDS-staged (coop) search also
    // takes the HBM R once an LDS R would leave fewer than 4 waves per CU: each expansion is a
    // chain of dependent memory round trips, so waves in flight, not bytes, bound it (10M x 768
    // M 32, 1024 queries: ef 8192 1573 -> 2232 QPS, 12288 495 -> 1266, 16384 339 -> 827; 10k
    // queries: ef 3200 8.7k -> 11.0k, 4096 5.0k -> 8.2k; 20M x 128 ef 4096 11.5k -> 14.2k;
    // scripts/exp/exp_hnsw_nst.py, profiles/r05_hnsw_rg_rule_*.txt).
    // RVX_HNSW_RG: 1 always, 0 only past the LDS, unset auto (read per call: tests force both)
    // LDS-staged distances also for long rows on smaller tables when the layer-0 lists span several
    // 64-entry slices (round 6: with whole lists batched they fill the DMA stages; 1M x 768 M 128,
    // 2,048 queries: ef 1,600 8.71k -> 9.72k QPS, 4,096 4.20k -> 5.02k, 8,192 2.86k -> 3.22k,
    // 12,288 2.27k -> 2.46k against per-lane distances, profiles/r06_hnsw_collect_ab_1m.log)
    const bool coop0 = hnsw_coop(metric, d, g.n) ||
                       (env_int("RVX_HNSW_COOP", 1) == 1 && d >= 512 && g.max_deg > 64 &&
                        env_int("RVX_HNSW_COLLECT", 1) != 0 && hnsw_coop(metric, d, INT64_MAX / (4 * (int64_t)d)));
    const int rg_mode = env_int("RVX_HNSW_RG", -1);
    const size_t lds_r = hnsw_search_lds(d, ef, coop0);
    // waves per CU below which R moves to HBM: 4 (RVX_HNSW_RG_WAVES=W, read per call, for A/Bs),
    // on the footprint of the stage count hnsw_nst picks
    const int rg_waves = std::max(1, env_int("RVX_HNSW_RG_WAVES", 4));
    const bool rg_auto = lds_r * (size_t)rg_waves > 160 * 1024;
    // per-lane distances (tables below the translation reach, the Poincaré metrics): HBM R once
    // an LDS R would leave fewer than 6 waves per CU (RVX_HNSW_RG_WAVES_LANE). Round 6, with R's
    // admissions buffered in LDS (1M x 768 M 128, 2,048 queries, profiles/r06_hnsw_coop_ab_1m.log):
    // ef 4,096 (LDS R: 4.4 waves) 3.05k -> 3.99k QPS, 8,192 846 -> 2.29k, 12,288 300 -> 1.66k;
    // ef 1,600 (9 waves) stays in LDS (8.67k vs 8.18k)
    const int rg_waves_lane = std::max(1, env_int("RVX_HNSW_RG_WAVES_LANE", 6));
    const bool rg_auto_lane = lds_r * (size_t)rg_waves_lane > 160 * 1024;
    const bool rg = lds_r > 160 * 1024 || rg_mode == 1 ||
                    (rg_mode < 0 && (coop0 ? rg_auto : rg_auto_lane));
    const unsigned vcap = visited_capacity(ef, g.max_deg, g.n);
    // visited set: a per-slot bitmap over all n nodes (cleared per query by its
    // wave: no launch-wide memset, no probing, n/8 bytes touched) when at least
    // min(nq, 1024) slots' bitmaps fit the budget — what the scratch slot already
    // holds, else min(16 GiB, 1/4 of the free HBM), as the exact scan sizes its f16
    // image (10M nodes x 8192 slots = 10 GB) — else the tagged hash (zeroed per
    // launch; it stays for 100M-node tables). C1 ef 600: 336k -> 438k QPS; 4M x 768
    // ef 1600: 16.6k -> 22.2k
    const int64_t vwords = (g.n + 127) / 128 * 4;
    const int bm_mode = env_int("RVX_HNSW_BITMAP", 1);  // 0 off, 1 auto, 2 force (tests); read per call
    const int64_t bm_slots = std::min<int64_t>(nq, 8192);
    const int64_t held = scratch_held("hnsw_vbits");
    int64_t budget = held;
    {
        size_t fr = 0, tot = 0;
        RVX_HIP(hipMemGetInfo(&fr, &tot));
        budget = std::max<int64_t>(held, std::min<int64_t>((int64_t)16 << 30, ((int64_t)fr + held) / 4));
        const int64_t cap_mb = env_int("RVX_HNSW_BITMAP_BUDGET_MB", 0);  // tests force a small budget
        if (cap_mb > 0) budget = std::min<int64_t>(budget, cap_mb << 20);
    }
    const int64_t fit_slots = budget / (vwords * 4);
    const bool bitmap = bm_mode == 2 || (bm_mode == 1 && fit_slots >= std::min<int64_t>(bm_slots, 1024));
    // hash slots by bytes: 8 GiB of tables (one slot at the 2^30-entry maximum)
    const int64_t mem_slots = std::max<int64_t>(1, ((int64_t)8 << 30) / ((int64_t)vcap * 8));
    int nslots = (int)(bitmap ? (bm_mode == 2 ? bm_slots : std::min(bm_slots, fit_slots))
                              : std::min<int64_t>(bm_slots, mem_slots));
    // RG: each slot also holds an HBM row of ef + 1 R entries (8 B each), within 4 GiB
    if (rg) nslots = (int)std::max<int64_t>(1, std::min<int64_t>(nslots, ((int64_t)4 << 30) / ((int64_t)(ef + 1) * 8)));
    unsigned long long* vis = nullptr;
    unsigned* vbits = nullptr;
    if (bitmap) {
        vbits = (unsigned*)scratch_bytes("hnsw_vbits", (int64_t)nslots * vwords * 4);
    } else {
        vis = (unsigned long long*)scratch_bytes("hnsw_visited", (int64_t)nslots * vcap * 8);
        RVX_HIP(hipMemsetAsync(vis, 0, (size_t)nslots * vcap * 8, stream()));
    }
    int* status = (int*)scratch_bytes("hnsw_status", 256);
    auto* stats = reinterpret_cast<unsigned long long*>(status + 16);
    RVX_HIP(hipMemsetAsync(status, 0, 256, stream()));
    const bool coop = coop0;
    float* rg_d = nullptr;
    int* rg_i = nullptr;
    if (rg) {
        rg_d = scratch_f32("hnsw_rg_d", (int64_t)nslots * (ef + 1));
        rg_i = (int*)scratch_bytes("hnsw_rg_i", (int64_t)nslots * (ef + 1) * 4);
    }
    SearchArgs a{g, x, xnorm, d, q, qnorm, nq, k, ef, vis, vbits, vwords, nslots, vcap, out_d, out_i, out_n, status, stats,
                 curv, hyper, coop ? 1 : 0, rg_d, rg_i, env_int("RVX_HNSW_PAR_DECIDE", 1) != 0 ? 1 : 0,
                 env_int("RVX_HNSW_RG_BUF", 1) != 0 ? 1 : 0,  // (read per call: tests and A/Bs run both)
                 env_int("RVX_HNSW_COLLECT", 1) != 0 ? 1 : 0};
    // RVX_HNSW_QG=1 (read per call): LDS-staged distances read the query from global memory (no LDS copy)
    const int nst_sel = rg ? hnsw_rg_nst() : hnsw_nst(coop, d, ef);
    const bool qg = coop && (rg ? nst_sel == 2 : (nst_sel == 1 || nst_sel == 2)) && env_int("RVX_HNSW_QG", 0) != 0 &&
                    ((uintptr_t)q & 15) == 0;
    const size_t lds = (rg ? hnsw_search_lds_rg(d, coop) : hnsw_search_lds(d, ef, coop)) -
                       (qg ? (size_t)((d + 3) & ~3) * 4 : 0);
    RVX_REQUIRE(lds <= 160 * 1024, RVX_ERR_INVALID_PARAMETER, "dimension too large for one wave's LDS");
    static bool attr_qg = false;
    if (!attr_qg) {
        set_qg_attr<1, false>();
        set_qg_attr<2, false>();
        set_qg_attr<2, true>();
        attr_qg = true;
    }
    static bool attr = false;
    if (!attr) {
        RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search<RVX_METRIC_L2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search<RVX_METRIC_COSINE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search<RVX_METRIC_DOT>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search<RVX_METRIC_L1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search<RVX_METRIC_POINCARE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search<RVX_METRIC_HYP_L2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_short<RVX_METRIC_L2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_short<RVX_METRIC_COSINE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_short<RVX_METRIC_DOT>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_short<RVX_METRIC_L1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        set_st_attr<1>();
        set_st_attr<3>();
        set_st_attr<4>();
        set_st_attr<6>();
        RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_rg<RVX_METRIC_L2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_rg<RVX_METRIC_COSINE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_rg<RVX_METRIC_DOT>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_rg<RVX_METRIC_L1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_rg<RVX_METRIC_POINCARE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_hnsw_search_rg<RVX_METRIC_HYP_L2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr = true;
    }
    const char* t = tag ? tag : "hnsw_search";
    const bool short_rows = !coop && d <= 256 && env_int("RVX_HNSW_SHORT", 1);  // read per call: tests cover both
    if (qg) {
        if (rg) launch_qg<2, true>(t, metric, nslots, lds, a);
        else if (nst_sel == 1) launch_qg<1, false>(t, metric, nslots, lds, a);
        else launch_qg<2, false>(t, metric, nslots, lds, a);
    } else if (rg && coop && hnsw_rg_nst() == 2) {
        switch (metric) {
            case RVX_METRIC_L2: RVX_LAUNCH(t, (k_hnsw_search_rg<RVX_METRIC_L2, 2>), dim3(nslots), dim3(64), lds, a); break;
            case RVX_METRIC_COSINE: RVX_LAUNCH(t, (k_hnsw_search_rg<RVX_METRIC_COSINE, 2>), dim3(nslots), dim3(64), lds, a); break;
            case RVX_METRIC_DOT: RVX_LAUNCH(t, (k_hnsw_search_rg<RVX_METRIC_DOT, 2>), dim3(nslots), dim3(64), lds, a); break;
            default: RVX_LAUNCH(t, (k_hnsw_search_rg<RVX_METRIC_L1, 2>), dim3(nslots), dim3(64), lds, a); break;
        }
    } else if (rg) {
        switch (metric) {
            case RVX_METRIC_L2: RVX_LAUNCH(t, k_hnsw_search_rg<RVX_METRIC_L2>, dim3(nslots), dim3(64), lds, a); break;
            case RVX_METRIC_COSINE: RVX_LAUNCH(t, k_hnsw_search_rg<RVX_METRIC_COSINE>, dim3(nslots), dim3(64), lds, a); break;
            case RVX_METRIC_DOT: RVX_LAUNCH(t, k_hnsw_search_rg<RVX_METRIC_DOT>, dim3(nslots), dim3(64), lds, a); break;
            case RVX_METRIC_L1: RVX_LAUNCH(t, k_hnsw_search_rg<RVX_METRIC_L1>, dim3(nslots), dim3(64), lds, a); break;
            case RVX_METRIC_POINCARE: RVX_LAUNCH(t, k_hnsw_search_rg<RVX_METRIC_POINCARE>, dim3(nslots), dim3(64), lds, a); break;
            case RVX_METRIC_HYP_L2: RVX_LAUNCH(t, k_hnsw_search_rg<RVX_METRIC_HYP_L2>, dim3(nslots), dim3(64), lds, a); break;
            default: fail(RVX_ERR_UNSUPPORTED, "metric not supported by HNSW search");
        }
    } else if (short_rows && metric != RVX_METRIC_POINCARE && metric != RVX_METRIC_HYP_L2) {
        switch (metric) {
            case RVX_METRIC_L2: RVX_LAUNCH(t, k_hnsw_search_short<RVX_METRIC_L2>, dim3(nslots), dim3(64), lds, a); break;
            case RVX_METRIC_COSINE: RVX_LAUNCH(t, k_hnsw_search_short<RVX_METRIC_COSINE>, dim3(nslots), dim3(64), lds, a); break;
            case RVX_METRIC_DOT: RVX_LAUNCH(t, k_hnsw_search_short<RVX_METRIC_DOT>, dim3(nslots), dim3(64), lds, a); break;
            default: RVX_LAUNCH(t, k_hnsw_search_short<RVX_METRIC_L1>, dim3(nslots), dim3(64), lds, a); break;
        }
    } else if (coop && hnsw_nst(coop, d, ef) != 2) {  // coop is never set for the Poincaré metrics
        switch (hnsw_nst(coop, d, ef)) {
            case 1: launch_st<1>(t, metric, nslots, lds, a); break;
            case 3: launch_st<3>(t, metric, nslots, lds, a); break;
            case 4: launch_st<4>(t, metric, nslots, lds, a); break;
            default: launch_st<6>(t, metric, nslots, lds, a); break;
        }
    } else
    switch (metric) {
        case RVX_METRIC_L2: RVX_LAUNCH(t, k_hnsw_search<RVX_METRIC_L2>, dim3(nslots), dim3(64), lds, a); break;
        case RVX_METRIC_COSINE: RVX_LAUNCH(t, k_hnsw_search<RVX_METRIC_COSINE>, dim3(nslots), dim3(64), lds, a); break;
        case RVX_METRIC_DOT: RVX_LAUNCH(t, k_hnsw_search<RVX_METRIC_DOT>, dim3(nslots), dim3(64), lds, a); break;
        case RVX_METRIC_L1: RVX_LAUNCH(t, k_hnsw_search<RVX_METRIC_L1>, dim3(nslots), dim3(64), lds, a); break;
        case RVX_METRIC_POINCARE: RVX_LAUNCH(t, k_hnsw_search<RVX_METRIC_POINCARE>, dim3(nslots), dim3(64), lds, a); break;
        case RVX_METRIC_HYP_L2: RVX_LAUNCH(t, k_hnsw_search<RVX_METRIC_HYP_L2>, dim3(nslots), dim3(64), lds, a); break;
        default: fail(RVX_ERR_UNSUPPORTED, "metric not supported by HNSW search");
    }
    // the work tallies reach page-locked host memory behind the search; the search itself returns
    // with its work queued (no host wait) and rvx_hnsw_last_search_stats settles them on demand
    SearchTally& tl = search_tally();
    RVX_HIP(hipMemcpyAsync(tl.host, stats, 8 * 8, hipMemcpyDeviceToHost, stream()));
    tl.pending = true;
    g_search_stats.visited_overflow = 0;
    g_search_stats.r_in_hbm = rg ? 1 : 0;
    g_search_stats.stages = coop ? nst_sel : 0;
    g_search_stats.nq = nq;
    g_search_stats.visited_bitmap = bitmap ? 1 : 0;
    g_search_stats.slots = nslots;
#ifdef RVX_HNSW_PHASES
    {
        sync();
        const unsigned long long* tally = tl.host;
        const double tot = (double)(tally[2] + tally[3] + tally[4] + tally[5] + tally[6]);
        std::fprintf(stderr, "[hnsw phases] ef %d rg %d: next %.3f claim %.3f dist %.3f decide %.3f merge %.3f "
                     "(cycles per expansion %.0f)\n", ef, rg ? 1 : 0, tally[2] / tot, tally[3] / tot, tally[4] / tot,
                     tally[5] / tot, tally[6] / tot, tot / (double)std::max<unsigned long long>(tally[1], 1));
    }
#endif
}

void hnsw_search_stats_settle() {
    SearchTally& tl = search_tally();
    if (!tl.pending) return;
    sync();
    g_search_stats.n_dist = (int64_t)tl.host[0];
    g_search_stats.n_expand = (int64_t)tl.host[1];
    g_search_stats.visited_overflow = (int32_t)(tl.host[7] != 0);
    tl.pending = false;
}

void hnsw_search_check() {
    hnsw_search_stats_settle();
    RVX_REQUIRE(!g_search_stats.visited_overflow, RVX_ERR_INDEX,
                "HNSW search: a query's visited set filled its table (more than 8 ef expansions of full lists); "
                "results would skip nodes");
}

}  // namespace rvx
