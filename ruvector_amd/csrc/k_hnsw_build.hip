// k_hnsw_build.hip — batched HNSW construction on the GPU (K3).
//
// Follows hnsw_rs 0.3.3 insert_slice (patches/hnsw_rs/src/hnsw.rs:1068-1206) per
// point, run for a batch of points at once against the graph as it stood
// before the batch (what Hnsw::parallel_insert does with concurrent inserters,
// :1212-1218, made deterministic):
//   1. greedy descent with search_layer(ef = 1) on layers above the point's
//      level (:1105-1146), from the current entry point;
//   2. for l = level .. 0: search_layer(ef_construction) -> select_neighbours
//      (:1287-1409: keep e unless some already selected s has d(e,s) <= d(e,q);
//      2M at layer 0, M above) -> the point's list at l, sorted ascending;
//   3. reverse_update_neighborhood_simple (:1229-1277): the new point is added
//      to every selected neighbour's list AT THE NEW POINT'S OWN LEVEL (l_n),
//      kept sorted and truncated to the capacity (M, 2M at layer 0). With all
//      reverse edges of a batch known, the list becomes the best `cap` of
//      (old list ∪ new entries) — the same set the reference's push/sort/pop
//      sequence leaves. Reverse edges into a list that only exists above the
//      neighbour's own level (never traversed by search) are dropped.
// Batches grow geometrically (size ~ inserted/16) so batch-mates that cannot
// see each other stay a small fraction. Build parity is recall vs the
// oracle's CPU build.
//
// Storage (fixed capacity): layer 0 lists [n][2M] ids + distances + count;
// upper lists compacted per point (up_base[p] + l - 1) of capacity M.
// Distances are the reference scalar order (hnsw_dev.hpp), so a list's order
// matches hnsw_rs's sort_unstable by distance (ties by id here).
#include "common.hpp"
#include "graph.hpp"
#include "hnsw.hpp"
#include "hnsw_build.hpp"
#include "hnsw_dev.hpp"

namespace rvx {
namespace {
using namespace hnswdev;

constexpr int MAX_C0 = 256;  // layer-0 list capacity (2M for hnsw_rs: M <= 128)

struct BuildArgs {
    BuildGraph G;
    const float* x; const float* xnorm; int d;
    int64_t batch_begin; int batch_n;
    int entry; int entry_level;
    unsigned nonempty_mask;  // bit l: some inserted point has level exactly l (points_by_layer[l])
    int ef_c;
    unsigned long long* visited; int nslots; unsigned vcap;
    int* rev_head; int* rev_next; int* rev_key; float* rev_d; int* rev_src;  // reverse-edge chains
    int rev_cap;  // records per batch point
    float curv;  // Poincaré curvature
    int hyper;   // HyperbolicHnsw::insert rules
    int coop;    // wave-cooperative LDS-staged distances in the layer searches
    float* rg_d; int* rg_i;  // RG: R in HBM, [nslots][ef_c + 1] (ef_c past one wave's LDS)
    int* vis_full;           // set when a visited table fills (hnsw_dev.hpp visit_claim): the batch fails
    int collect;             // whole lists claimed first, fresh neighbours batched (RVX_HNSW_COLLECT, default 1)
};

__device__ __forceinline__ int list_get(const BuildGraph& G, int p, int l, const int** ids, const float** ds) {
    if (l == 0) {
        *ids = G.nb0 + (int64_t)p * G.C0;
        *ds = G.nbd0 + (int64_t)p * G.C0;
        return G.cnt0[p];
    }
    if ((int)G.level[p] < l) return 0;
    const int64_t li = G.up_base[p] + (l - 1);
    *ids = G.nbu + li * G.M;
    *ds = G.nbud + li * G.M;
    return G.cntu[li];
}
__device__ __forceinline__ int list_key(const BuildGraph& G, int p, int l) {  // -1: no live list
    if (l == 0) return p;
    if ((int)G.level[p] < l) return -1;
    return (int)(G.n_cap + G.up_base[p] + (l - 1));
}

// search_layer (hnsw.rs:913-1055) at layer l from ep; R left ascending in (rd, ri), returns |R|.
// R-only form (hnsw_dev.hpp merge_into_r, as the query kernel k_hnsw.hip): the
// nearest candidate is the nearest unexpanded entry of R (id bit 31 = expanded);
// the flags are cleared before returning.
template <int METRIC, bool RG = false, int NST = 2>
__device__ int build_search_layer(const BuildArgs& a, const float* qs, float qn, int ep, float d_ep, int ef, int l,
                                  unsigned long long* vis, unsigned vmask, unsigned long long tag, float* rd, int* ri,
                                  float* sdb, int* sib, unsigned char* wst, int lane) {
    if (!((a.nonempty_mask >> l) & 1u)) return 0;  // points_by_layer[layer].is_empty()
    int rs = 1;
    if (lane == 0) {
        rd[0] = d_ep; ri[0] = ep;
        visit_claim(vis, vmask, tag, ep, a.vis_full);
    }
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    int scan = 0;
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
        const int* nbi;
        const float* nbd;
        const int cnt = list_get(a.G, c_id, l, &nbi, &nbd);
        // The whole list claimed first and its fresh neighbours compacted in list order, then
        // admitted in batches of up to 64 (one distance pass each instead of one per 64-entry
        // slice; as the query kernel's collect_fresh, k_hnsw.hip). The fresh ids sit in the parts
        // of the selection arrays the search does not use: sd[64..MAX_C0) then si[64..MAX_C0).
        int* const fsd = reinterpret_cast<int*>(sdb) + 64;
        int* const fsi = sib + 64;
        auto fslot = [&](int f) -> int* { return f < MAX_C0 - 64 ? fsd + f : fsi + (f - (MAX_C0 - 64)); };
        const bool whole = a.collect && cnt <= MAX_C0 && cnt > 64;  // (wave-uniform; one slice needs no compaction)
        int nf = 0;
        if (whole) {
            int nids[MAX_C0 / 64];
            bool fr[MAX_C0 / 64];
#pragma unroll
            for (int sl = 0; sl < MAX_C0 / 64; ++sl) nids[sl] = 64 * sl + lane < cnt ? nbi[64 * sl + lane] : -1;
#pragma unroll
            for (int sl = 0; sl < MAX_C0 / 64; ++sl) fr[sl] = nids[sl] >= 0 && visit_claim(vis, vmask, tag, nids[sl], a.vis_full);
#pragma unroll
            for (int sl = 0; sl < MAX_C0 / 64; ++sl) {
                const unsigned long long m = __ballot(fr[sl]);
                const int before = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                if (fr[sl]) *fslot(nf + before) = nids[sl];
                nf += __popcll(m);
            }
            __builtin_amdgcn_wave_barrier();
        }
        for (int c0 = 0, c1 = whole ? nf : cnt; c0 < c1; c0 += 64) {
            const int p = c0 + lane;
            int nid = -1;
            bool fresh = false;
            if (whole) {
                nid = p < nf ? *fslot(p) : -1;
                fresh = nid >= 0;
            } else if (p < cnt) {
                nid = nbi[p];
                fresh = visit_claim(vis, vmask, tag, nid, a.vis_full);
            }
            const unsigned long long fmask = __ballot(fresh);
            if (!fmask) continue;
            float dd = INFINITY;
            bool coop = false;
            if constexpr (METRIC != RVX_METRIC_POINCARE && METRIC != RVX_METRIC_HYP_L2) coop = a.coop != 0;
            if (coop) {
                if constexpr (METRIC != RVX_METRIC_POINCARE && METRIC != RVX_METRIC_HYP_L2) {
                    const int row = fresh ? nid : -1;
                    const float dv = wave_dist<METRIC, NST>(qs, a.x, a.d, row, qn,
                                                       (METRIC == RVX_METRIC_COSINE && fresh) ? a.xnorm[nid] : 0.0f,
                                                       wst, lane);
                    if (fresh) dd = dv;
                }
            } else if (fresh) {
                dd = row_dist<METRIC>(qs, a.x + (int64_t)nid * a.d, a.d, qn,
                                      METRIC == RVX_METRIC_COSINE ? a.xnorm[nid] : 0.0f, a.curv);
            }
            int r = rs, rk = 0;
            // parallel admissions where R is in LDS (hnsw_dev.hpp decide_par, as the search)
            int* srk = sib + MAX_C0;
            const bool par = !RG && !__ballot(((fmask >> lane) & 1ull) && dd != dd);
            const unsigned long long adm = par ? decide_par(fmask, dd, nid, ef, rd, ri, rs, r, rk, lane)
                                               : decide_batch(fmask, dd, nid, ef, rd, ri, rs, r, lane);
            const int na = sort_batch(adm, dd, nid, sdb, sib, lane, par ? srk : nullptr, rk);
            if (na == 0) continue;
            scan = min(scan, merge_into_r<RG ? RVX_MERGE_RG_G : RVX_MERGE_LDS_G>(rd, ri, rs, sdb, sib, na, r, lane,
                                                                              par ? srk : nullptr));
            if constexpr (RG) __threadfence_block();
            rs = r;
        }
    }
    for (int i = lane; i < rs; i += 64) ri[i] &= ID_MASK;
    if constexpr (RG) __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    return rs;
}

#ifndef RVX_BUILD_WPE
#define RVX_BUILD_WPE
#endif
template <int METRIC, bool RG, int NST>
__device__ __forceinline__ void build_insert_body(const BuildArgs& a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    const int lane = threadIdx.x;
    const int ef = a.ef_c;
    const int dq = (a.d + 3) & ~3;
    unsigned char* wst = lds_raw;  // [NST * WD_STAGE] distance stages (coop)
    float* qs = reinterpret_cast<float*>(lds_raw + (a.coop ? wd_lds(NST) : 0));
    float* rd;
    int* ri;
    float* sd;  // selected [MAX_C0] (search: admitted batch [64])
    if constexpr (RG) {
        rd = a.rg_d + (int64_t)blockIdx.x * (ef + 1);
        ri = a.rg_i + (int64_t)blockIdx.x * (ef + 1);
        sd = qs + dq;
    } else {
        rd = qs + dq;
        ri = reinterpret_cast<int*>(rd + ef + 1);
        sd = reinterpret_cast<float*>(ri + ef + 1);
    }
    int* si = reinterpret_cast<int*>(sd + MAX_C0);
    unsigned long long* vis = a.visited + (int64_t)blockIdx.x * a.vcap;
    const unsigned vmask = a.vcap - 1;
    unsigned epoch = 0;

    for (int b = blockIdx.x; b < a.batch_n; b += a.nslots) {
        const int p = (int)(a.batch_begin + b);
        for (int i = lane; i < dq; i += 64) qs[i] = (i < a.d) ? a.x[(int64_t)p * a.d + i] : 0.0f;
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
        const float qn = (METRIC == RVX_METRIC_COSINE) ? a.xnorm[p] : 0.0f;
        const int lev = a.G.level[p];
        int rec = 0;  // reverse-edge records emitted for this point
        const int rbase = b * a.rev_cap;

        int ep = a.entry;
        float d_ep = row_dist<METRIC>(qs, a.x + (int64_t)ep * a.d, a.d, qn,
                                      METRIC == RVX_METRIC_COSINE ? a.xnorm[ep] : 0.0f, a.curv);
        // 1. greedy descent, ef = 1 (hnsw.rs:1105-1146)
        for (int l = a.entry_level; l >= lev + 1; --l) {
            const unsigned long long tag = (unsigned long long)(++epoch) << 32;
            const int rs = build_search_layer<METRIC, RG, NST>(a, qs, qn, ep, d_ep, 1, l, vis, vmask, tag, rd, ri, sd,
                                                               si, wst, lane);
            if (rs > 0 && rd[0] < d_ep) { ep = ri[0]; d_ep = rd[0]; }
        }
        // 2. layers lev .. 0 (hnsw.rs:1149-1196); HyperbolicHnsw inserts at
        //    min(level, max_level) .. 0 (hyperbolic hnsw.rs:213)
        const int ltop = a.hyper ? min(lev, a.entry_level) : lev;
        for (int l = ltop; l >= 0; --l) {
            const unsigned long long tag = (unsigned long long)(++epoch) << 32;
            const int rs = build_search_layer<METRIC, RG, NST>(a, qs, qn, ep, d_ep, ef, l, vis, vmask, tag, rd, ri, sd,
                                                               si, wst, lane);
            if (rs == 0) continue;
            const int nb_conn = l == 0 ? a.G.C0 : a.G.M;
            int ss = 0;
            if (rs <= nb_conn || a.hyper) {
                // all of R, or (HyperbolicHnsw, hnsw.rs:225) its closest nb_conn
                ss = min(rs, nb_conn);
                for (int i = lane; i < ss; i += 64) { sd[i] = rd[i]; si[i] = ri[i]; }
            } else {
                // select_neighbours heuristic (hnsw.rs:1350-1380), one lane per selected point
                for (int t = 0; t < rs && ss < nb_conn; ++t) {
                    const int e = ri[t];
                    const float de = rd[t];
                    bool bad = false;
                    for (int j = lane; j < ss && !bad; j += 64) {
                        const int s = si[j];
                        const float dse = row_dist<METRIC>(a.x + (int64_t)e * a.d, a.x + (int64_t)s * a.d, a.d,
                                                           METRIC == RVX_METRIC_COSINE ? a.xnorm[e] : 0.0f,
                                                           METRIC == RVX_METRIC_COSINE ? a.xnorm[s] : 0.0f, a.curv);
                        bad = dse <= de;
                    }
                    if (__ballot(bad) == 0ull) {
                        if (lane == 0) { sd[ss] = de; si[ss] = e; }
                        ss += 1;
                        __threadfence_block();
                        __builtin_amdgcn_wave_barrier();
                    }
                }
            }
            __threadfence_block();
            __builtin_amdgcn_wave_barrier();
            // the point's own list at layer l (sorted: R ascending, S is a subsequence)
            int* oid;
            float* od;
            int* ocnt;
            if (l == 0) {
                oid = a.G.nb0 + (int64_t)p * a.G.C0;
                od = a.G.nbd0 + (int64_t)p * a.G.C0;
                ocnt = a.G.cnt0 + p;
            } else {
                const int64_t li = a.G.up_base[p] + (l - 1);
                oid = a.G.nbu + li * a.G.M;
                od = a.G.nbud + li * a.G.M;
                ocnt = a.G.cntu + li;
            }
            for (int i = lane; i < ss; i += 64) { oid[i] = si[i]; od[i] = sd[i]; }
            if (lane == 0) *ocnt = ss;
            // reverse-edge records: p into s's list at p's own level (hnsw_rs quirk),
            // or at the current level l (HyperbolicHnsw, hnsw.rs:232-239)
            for (int i = lane; i < ss; i += 64) {
                const int s = si[i];
                const int key = (s == p) ? -1 : list_key(a.G, s, a.hyper ? l : lev);
                const int r = rbase + rec + i;
                a.rev_key[r] = key;
                a.rev_d[r] = sd[i];
                a.rev_src[r] = p;
                if (key >= 0) a.rev_next[r] = atomicExch(&a.rev_head[key], r);
            }
            rec += ss;
            ep = si[0];
            d_ep = sd[0];
            __builtin_amdgcn_wave_barrier();
        }
        for (int i = rec + lane; i < a.rev_cap; i += 64) a.rev_key[rbase + i] = -1;
    }
}

template <int METRIC, bool RG = false>
__global__ __launch_bounds__(64) RVX_BUILD_WPE void k_build_insert(BuildArgs a) {
    build_insert_body<METRIC, RG, 2>(a);
}

// One wave per list that received reverse edges (the record that found the
// chain head empty owns it): merge old list ∪ new entries, keep the best cap.
// Lane j holds elements j, 64 + j, ... of the sorted list (NE per lane, cap <= 64 NE).
template <int NE>
__global__ __launch_bounds__(256) void k_build_merge(BuildArgs a, int nrec) {
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * 4) + (threadIdx.x >> 6);
    const int r0 = wave * 64;
    if (r0 >= nrec) return;
    const int r = r0 + lane;
    // owner = the record at the END of its chain (rev_next == -1), i.e. the first pushed
    bool own = false;
    if (r < nrec && a.rev_key[r] >= 0) own = (a.rev_next[r] == -1);
    unsigned long long owners = __ballot(own);
    while (owners) {
        const int src = __ffsll((long long)owners) - 1;
        owners &= owners - 1;
        const int key = __shfl(a.rev_key[r < nrec ? r : r0], src);
        int* ids;
        float* ds;
        int* cntp;
        int cap;
        if (key < a.G.n_cap) {
            ids = a.G.nb0 + (int64_t)key * a.G.C0;
            ds = a.G.nbd0 + (int64_t)key * a.G.C0;
            cntp = a.G.cnt0 + key;
            cap = a.G.C0;
        } else {
            const int64_t li = key - a.G.n_cap;
            ids = a.G.nbu + li * a.G.M;
            ds = a.G.nbud + li * a.G.M;
            cntp = a.G.cntu + li;
            cap = a.G.M;
        }
        int cnt = *cntp;
        float md[NE];
        int mi[NE];
#pragma unroll
        for (int j = 0; j < NE; ++j) {
            const int e = 64 * j + lane;
            md[j] = e < cnt ? ds[e] : INFINITY;
            mi[j] = e < cnt ? ids[e] : INT_MAX;
        }
        int steps = 0;
        for (int h = a.rev_head[key]; h >= 0 && h < nrec && steps < nrec; h = a.rev_next[h], ++steps) {
            const float d = a.rev_d[h];
            const int id = a.rev_src[h];
            bool dup = false;
#pragma unroll
            for (int j = 0; j < NE; ++j) dup = dup || mi[j] == id;
            if (__ballot(dup) != 0ull) continue;  // already present
            if (cnt == cap) {
                const int jl = (cap - 1) >> 6, ll = (cap - 1) & 63;
                float ld = INFINITY;
                int li2 = INT_MAX;
#pragma unroll
                for (int j = 0; j < NE; ++j) {
                    const float tv = __shfl(md[j], ll);
                    const int ti = __shfl(mi[j], ll);
                    if (j == jl) { ld = tv; li2 = ti; }
                }
                if (!lt(d, id, ld, li2)) continue;
            }
            int pos = 0;
#pragma unroll
            for (int j = 0; j < NE; ++j) pos += __popcll(__ballot(64 * j + lane < cnt && lt(md[j], mi[j], d, id)));
            // shift elements >= pos up by one (element 64 j + 63 moves to 64 (j + 1))
            float cd[NE], upd[NE];
            int ci[NE], upi[NE];
#pragma unroll
            for (int j = 0; j < NE; ++j) {
                cd[j] = __shfl(md[j], 63);
                ci[j] = __shfl(mi[j], 63);
                upd[j] = __shfl_up(md[j], 1);
                upi[j] = __shfl_up(mi[j], 1);
            }
#pragma unroll
            for (int j = 0; j < NE; ++j) {
                const int e = 64 * j + lane;
                const int jp = j > 0 ? j - 1 : 0;  // lane 0 of chunk j takes chunk j-1's last (e > pos >= 0: j > 0)
                if (e > pos) {
                    md[j] = lane == 0 ? cd[jp] : upd[j];
                    mi[j] = lane == 0 ? ci[jp] : upi[j];
                }
                if (e == pos) { md[j] = d; mi[j] = id; }
            }
            cnt = min(cnt + 1, cap);
        }
#pragma unroll
        for (int j = 0; j < NE; ++j)
            if (64 * j + lane < cnt) { ds[64 * j + lane] = md[j]; ids[64 * j + lane] = mi[j]; }
        if (lane == 0) { *cntp = cnt; a.rev_head[key] = -1; }
    }
}

}  // namespace

size_t build_lds_bytes(int d, int ef, bool coop, bool rg = false, int nst = 2) {
    const int dq = (d + 3) & ~3;
    return (coop ? (size_t)wd_lds(nst) : 0) + (size_t)dq * 4 + (rg ? 0 : (size_t)(ef + 1) * 8) + (size_t)MAX_C0 * 8 +
           64 * 4;  // + the admitted batch's ranks in R
}

void build_insert_batch(const BuildGraph& G, int metric, const float* x, const float* xnorm, int d,
                        int64_t batch_begin, int batch_n, int entry, int entry_level, unsigned nonempty_mask, int ef_c,
                        BuildScratch& s, float curv, int hyper) {
    if (batch_n <= 0) return;
    RVX_REQUIRE(G.C0 <= MAX_C0 && G.M <= MAX_C0 / 2, RVX_ERR_UNSUPPORTED,
                "GPU HNSW build supports layer-0 lists of <= 256 and upper lists of <= 128 neighbours");
    RVX_REQUIRE(ef_c >= 1 && ef_c <= HNSW_MAX_EF, RVX_ERR_INVALID_PARAMETER, "ef_construction out of range");
    const unsigned vcap = visited_capacity(ef_c, G.C0, batch_begin + batch_n);
    const bool coop = hnsw_coop(metric, d, batch_begin + batch_n);
    // R in LDS when one wave's 160 KB hold it, else in HBM (RVX_HNSW_RG=1 forces, tests). Unlike
    // the high-ef search, more waves do not speed the build: R in HBM with one distance stage at
    // 3 waves per SIMD built the same graph slower (4M x 768 M 32: 41.7 vs 36.4 s; 2M M 128 ef_c
    // 500: > 180 vs 129 s; profiles/r05_build_wide_ab.txt, round 5).
    const bool rg = build_lds_bytes(d, ef_c, coop) > 160 * 1024 || env_int("RVX_HNSW_RG", 0) != 0;
    // visited tables within 4 GiB (memset per batch): 8,192 slots of 2^16 entries at ef_c 200 / M 32,
    // down to 4 slots of 2^27 at ef_c past 2^19 / 64 (no floor: a floor of 1,024 slots made
    // 128 GiB of tables at ef_c >= 32,768)
    int nslots = (int)std::min<int64_t>(std::min(batch_n, 8192),
                                        std::max<int64_t>(1, ((int64_t)4 << 30) / ((int64_t)vcap * 8)));
    if (rg) nslots = (int)std::max<int64_t>(1, std::min<int64_t>(nslots, ((int64_t)4 << 30) / ((int64_t)(ef_c + 1) * 8)));
    const int rev_cap = G.C0 + G.M * G.max_layer;
    BuildArgs a{};
    a.G = G; a.x = x; a.xnorm = xnorm; a.d = d;
    a.batch_begin = batch_begin; a.batch_n = batch_n; a.entry = entry; a.entry_level = entry_level;
    a.nonempty_mask = nonempty_mask; a.ef_c = ef_c;
    a.curv = curv; a.hyper = hyper;
    a.coop = coop ? 1 : 0;
    if (rg) {
        a.rg_d = scratch_f32("build_rg_d", (int64_t)nslots * (ef_c + 1));
        a.rg_i = (int*)scratch_bytes("build_rg_i", (int64_t)nslots * (ef_c + 1) * 4);
    }
    a.vcap = vcap;
    a.visited = (unsigned long long*)scratch_bytes("build_visited", (int64_t)nslots * vcap * 8);
    const int64_t nrec = (int64_t)batch_n * rev_cap;
    a.rev_next = (int*)scratch_bytes("build_rev_next", nrec * 4);
    a.rev_key = (int*)scratch_bytes("build_rev_key", nrec * 4);
    a.rev_d = (float*)scratch_bytes("build_rev_d", nrec * 4);
    a.rev_src = (int*)scratch_bytes("build_rev_src", nrec * 4);
    a.rev_head = s.rev_head;
    a.rev_cap = rev_cap;
    a.nslots = nslots;
    a.vis_full = (int*)scratch_bytes("build_vis_full", 64);
    a.collect = env_int("RVX_HNSW_COLLECT", 1) != 0 ? 1 : 0;  // (read per batch: tests build both ways)
    RVX_HIP(hipMemsetAsync(a.vis_full, 0, 4, stream()));
    RVX_HIP(hipMemsetAsync(a.visited, 0, (size_t)nslots * vcap * 8, stream()));
    const size_t lds = build_lds_bytes(d, ef_c, a.coop != 0, rg);
    RVX_REQUIRE(lds <= 160 * 1024, RVX_ERR_INVALID_PARAMETER, "dimension too large for one wave's LDS");
    static bool attr = false;
    if (!attr) {
        RVX_HIP(hipFuncSetAttribute((const void*)k_build_insert<RVX_METRIC_L2, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_build_insert<RVX_METRIC_COSINE, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_build_insert<RVX_METRIC_L1, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_build_insert<RVX_METRIC_POINCARE, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_build_insert<RVX_METRIC_HYP_L2, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_build_insert<RVX_METRIC_L2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_build_insert<RVX_METRIC_COSINE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_build_insert<RVX_METRIC_L1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_build_insert<RVX_METRIC_POINCARE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_build_insert<RVX_METRIC_HYP_L2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr = true;
    }
    if (rg) {
        switch (metric) {
            case RVX_METRIC_L2: RVX_LAUNCH("hnsw_build_insert", (k_build_insert<RVX_METRIC_L2, true>), dim3(nslots), dim3(64), lds, a); break;
            case RVX_METRIC_COSINE: RVX_LAUNCH("hnsw_build_insert", (k_build_insert<RVX_METRIC_COSINE, true>), dim3(nslots), dim3(64), lds, a); break;
            case RVX_METRIC_L1: RVX_LAUNCH("hnsw_build_insert", (k_build_insert<RVX_METRIC_L1, true>), dim3(nslots), dim3(64), lds, a); break;
            case RVX_METRIC_POINCARE: RVX_LAUNCH("hnsw_build_insert", (k_build_insert<RVX_METRIC_POINCARE, true>), dim3(nslots), dim3(64), lds, a); break;
            case RVX_METRIC_HYP_L2: RVX_LAUNCH("hnsw_build_insert", (k_build_insert<RVX_METRIC_HYP_L2, true>), dim3(nslots), dim3(64), lds, a); break;
            default: fail(RVX_ERR_UNSUPPORTED, "metric not supported by the GPU HNSW build");
        }
    } else
    switch (metric) {
        case RVX_METRIC_L2: RVX_LAUNCH("hnsw_build_insert", k_build_insert<RVX_METRIC_L2>, dim3(nslots), dim3(64), lds, a); break;
        case RVX_METRIC_COSINE: RVX_LAUNCH("hnsw_build_insert", k_build_insert<RVX_METRIC_COSINE>, dim3(nslots), dim3(64), lds, a); break;
        case RVX_METRIC_L1: RVX_LAUNCH("hnsw_build_insert", k_build_insert<RVX_METRIC_L1>, dim3(nslots), dim3(64), lds, a); break;
        case RVX_METRIC_POINCARE:
            RVX_LAUNCH("hnsw_build_insert", k_build_insert<RVX_METRIC_POINCARE>, dim3(nslots), dim3(64), lds, a);
            break;
        case RVX_METRIC_HYP_L2:
            RVX_LAUNCH("hnsw_build_insert", k_build_insert<RVX_METRIC_HYP_L2>, dim3(nslots), dim3(64), lds, a);
            break;
        default: fail(RVX_ERR_UNSUPPORTED, "metric not supported by the GPU HNSW build");
    }
    const int waves = (int)((nrec + 63) / 64);
    const dim3 mgrid((unsigned)((waves + 3) / 4));
    if (G.C0 <= 128) RVX_LAUNCH("hnsw_build_merge", k_build_merge<2>, mgrid, dim3(256), 0, a, (int)nrec);
    else RVX_LAUNCH("hnsw_build_merge", k_build_merge<4>, mgrid, dim3(256), 0, a, (int)nrec);
    int full = 0;
    RVX_HIP(hipMemcpyAsync(&full, a.vis_full, 4, hipMemcpyDeviceToHost, stream()));
    sync();
    RVX_REQUIRE(!full, RVX_ERR_INDEX,
                "HNSW build: an insert's visited set filled its table (more than 8 ef_c expansions of full lists)");
}

}  // namespace rvx
