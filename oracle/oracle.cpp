// oracle.cpp — CPU restatement of ruvector's GNN-learned-index hot path.
//
// TEST INFRASTRUCTURE ONLY. Nothing in ruvector_amd/ links, loads or calls this
// file; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg do,
// as the checker / CPU baseline. Each function restates the reference Rust
// literally (file:line under the Mu-L/ruvector checkout) in plain C++ compiled
// with -ffp-contract=off and no fast-math, so f32 arithmetic happens in the
// reference's order and libm (expf/logf/tanhf/sqrtf) is glibc's, as for Rust
// std on linux-gnu.
//
// Third-party arithmetic not vendored under /root/reference is restated from
// its published algorithm:
//   * ndarray 0.16.1 (Cargo.lock:5131): Array2·Array1 without BLAS is a per-row
//     numeric_util::unrolled_dot (8 partial sums, combined (p0+p4)+(p1+p5)+...),
//     Array1::mean = unrolled_fold sum / n.
//   * SimSIMD 5.9.11 (Cargo.lock:10262) is NOT restated: its ISA-dispatched f32
//     kernels are unpinned; distances follow the reference's own scalar
//     fallback (crates/ruvector-core/src/distance.rs:34-42, 52-63, 77-78, 85).
// hnsw_rs 0.3.3 is vendored (patches/hnsw_rs) and followed line by line,
// except that its entropy-seeded level generator is replaced by a seeded one
// and heap ties (unordered in the reference) are ordered by point id.
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <queue>
#include <thread>
#include <unordered_set>
#include <vector>

namespace {

inline uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

void pfor(int64_t n, int nthreads, const std::function<void(int64_t)>& f) {
    if (nthreads <= 1 || n < 2) {
        for (int64_t i = 0; i < n; ++i) f(i);
        return;
    }
    std::atomic<int64_t> next{0};
    std::vector<std::thread> th;
    const int nt = (int)std::min<int64_t>(nthreads, n);
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&] {
            for (;;) {
                const int64_t i = next.fetch_add(1);
                if (i >= n) break;
                f(i);
            }
        });
    for (auto& t : th) t.join();
}

struct Cand {
    float d;
    int64_t id;
};
inline bool cand_less(const Cand& a, const Cand& b) { return a.d < b.d || (a.d == b.d && a.id < b.id); }
struct CandMax {  // max-heap on (d, id)
    bool operator()(const Cand& a, const Cand& b) const { return cand_less(a, b); }
};
struct CandMin {  // min-heap on (d, id)
    bool operator()(const Cand& a, const Cand& b) const { return cand_less(b, a); }
};

enum { M_L2 = 0, M_COS = 1, M_DOT = 2, M_L1 = 3 };

// ---- CPU-baseline "fast mode" (SURVEY.md §8d): SIMD distances like the
// reference's default SimSIMD build / simd_intrinsics.rs:196-... (AVX-512 or
// AVX2 FMA, 16/8-lane partial sums, horizontal reduction). NOT the reference
// order: used only to time the CPU baseline (bench cpu_baseline legs,
// kind "simd"); parity always uses orc_distance.

__attribute__((target("avx512f"))) void simd3_512(const float* a, const float* b, int64_t d, int metric, float* o) {
    __m512 s0 = _mm512_setzero_ps(), s1 = _mm512_setzero_ps(), s2 = _mm512_setzero_ps();
    int64_t i = 0;
    for (; i + 16 <= d; i += 16) {
        const __m512 x = _mm512_loadu_ps(a + i), y = _mm512_loadu_ps(b + i);
        if (metric == M_L2) {
            const __m512 t = _mm512_sub_ps(x, y);
            s0 = _mm512_fmadd_ps(t, t, s0);
        } else if (metric == M_L1) {
            s0 = _mm512_add_ps(s0, _mm512_abs_ps(_mm512_sub_ps(x, y)));
        } else {
            s0 = _mm512_fmadd_ps(x, y, s0);
            if (metric == M_COS) { s1 = _mm512_fmadd_ps(x, x, s1); s2 = _mm512_fmadd_ps(y, y, s2); }
        }
    }
    if (i < d) {
        const __mmask16 m = (__mmask16)((1u << (d - i)) - 1);
        const __m512 x = _mm512_maskz_loadu_ps(m, a + i), y = _mm512_maskz_loadu_ps(m, b + i);
        if (metric == M_L2) { const __m512 t = _mm512_sub_ps(x, y); s0 = _mm512_fmadd_ps(t, t, s0); }
        else if (metric == M_L1) s0 = _mm512_add_ps(s0, _mm512_abs_ps(_mm512_sub_ps(x, y)));
        else {
            s0 = _mm512_fmadd_ps(x, y, s0);
            if (metric == M_COS) { s1 = _mm512_fmadd_ps(x, x, s1); s2 = _mm512_fmadd_ps(y, y, s2); }
        }
    }
    o[0] = _mm512_reduce_add_ps(s0);
    o[1] = _mm512_reduce_add_ps(s1);
    o[2] = _mm512_reduce_add_ps(s2);
}

__attribute__((target("avx2,fma"))) float hsum256(__m256 v) {
    const __m128 lo = _mm256_castps256_ps128(v), hi = _mm256_extractf128_ps(v, 1);
    __m128 s = _mm_add_ps(lo, hi);
    s = _mm_add_ps(s, _mm_movehl_ps(s, s));
    s = _mm_add_ss(s, _mm_shuffle_ps(s, s, 1));
    return _mm_cvtss_f32(s);
}

__attribute__((target("avx2,fma"))) void simd3_256(const float* a, const float* b, int64_t d, int metric, float* o) {
    __m256 s0 = _mm256_setzero_ps(), s1 = _mm256_setzero_ps(), s2 = _mm256_setzero_ps();
    const __m256 absm = _mm256_castsi256_ps(_mm256_set1_epi32(0x7fffffff));
    int64_t i = 0;
    for (; i + 8 <= d; i += 8) {
        const __m256 x = _mm256_loadu_ps(a + i), y = _mm256_loadu_ps(b + i);
        if (metric == M_L2) { const __m256 t = _mm256_sub_ps(x, y); s0 = _mm256_fmadd_ps(t, t, s0); }
        else if (metric == M_L1) s0 = _mm256_add_ps(s0, _mm256_and_ps(absm, _mm256_sub_ps(x, y)));
        else {
            s0 = _mm256_fmadd_ps(x, y, s0);
            if (metric == M_COS) { s1 = _mm256_fmadd_ps(x, x, s1); s2 = _mm256_fmadd_ps(y, y, s2); }
        }
    }
    float r0 = hsum256(s0), r1 = hsum256(s1), r2 = hsum256(s2);
    for (; i < d; ++i) {
        if (metric == M_L2) { const float t = a[i] - b[i]; r0 += t * t; }
        else if (metric == M_L1) r0 += std::fabs(a[i] - b[i]);
        else { r0 += a[i] * b[i]; if (metric == M_COS) { r1 += a[i] * a[i]; r2 += b[i] * b[i]; } }
    }
    o[0] = r0; o[1] = r1; o[2] = r2;
}

const bool g_avx512 = __builtin_cpu_supports("avx512f");

float fast_distance(const float* a, const float* b, int64_t d, int metric) {
    float s[3];
    if (g_avx512) simd3_512(a, b, d, metric, s);
    else simd3_256(a, b, d, metric, s);
    switch (metric) {
        case M_L2: return (float)std::sqrt((double)s[0]);  // distance.rs:30-32 (SimSIMD sqeuclidean)
        case M_COS: {
            const float den = std::sqrt(s[1]) * std::sqrt(s[2]);
            return den > 0.0f ? 1.0f - s[0] / den : 1.0f;
        }
        case M_DOT: return -s[0];
        default: return s[0];
    }
}

// ndarray numeric_util::unrolled_dot
float unrolled_dot(const float* x, const float* y, int64_t len) {
    float p0 = 0, p1 = 0, p2 = 0, p3 = 0, p4 = 0, p5 = 0, p6 = 0, p7 = 0;
    while (len >= 8) {
        p0 = p0 + x[0] * y[0]; p1 = p1 + x[1] * y[1]; p2 = p2 + x[2] * y[2]; p3 = p3 + x[3] * y[3];
        p4 = p4 + x[4] * y[4]; p5 = p5 + x[5] * y[5]; p6 = p6 + x[6] * y[6]; p7 = p7 + x[7] * y[7];
        x += 8; y += 8; len -= 8;
    }
    float sum = 0.0f;
    sum = sum + (p0 + p4);
    sum = sum + (p1 + p5);
    sum = sum + (p2 + p6);
    sum = sum + (p3 + p7);
    for (int64_t i = 0; i < len && i < 7; ++i) sum = sum + x[i] * y[i];
    return sum;
}
// ndarray numeric_util::unrolled_fold with add (Array1::sum)
float unrolled_sum(const float* x, int64_t len) {
    float p0 = 0, p1 = 0, p2 = 0, p3 = 0, p4 = 0, p5 = 0, p6 = 0, p7 = 0;
    while (len >= 8) {
        p0 = p0 + x[0]; p1 = p1 + x[1]; p2 = p2 + x[2]; p3 = p3 + x[3];
        p4 = p4 + x[4]; p5 = p5 + x[5]; p6 = p6 + x[6]; p7 = p7 + x[7];
        x += 8; len -= 8;
    }
    float acc = 0.0f;
    acc = acc + (p0 + p4);
    acc = acc + (p1 + p5);
    acc = acc + (p2 + p6);
    acc = acc + (p3 + p7);
    for (int64_t i = 0; i < len && i < 7; ++i) acc = acc + x[i];
    return acc;
}

}  // namespace

extern "C" {

// ============================================================ data generators
// Same integer stream as the device generator (ruvector_amd/csrc/k_data.hip).
void orc_fill_uniform(float* out, int64_t n, uint64_t seed, float lo, float hi) {
    const uint64_t s0 = sm64(seed);
    const float span = hi - lo;
    for (int64_t i = 0; i < n; ++i) {
        const float u = (float)(uint32_t)(sm64(s0 + (uint64_t)i) >> 40) * 5.9604644775390625e-08f;
        out[i] = u * span + lo;
    }
}

void orc_random_csr(int64_t n, int32_t deg, uint64_t seed, int64_t* row_ptr, int32_t* col) {
    const uint64_t s0 = sm64(seed);
    for (int64_t i = 0; i <= n; ++i) row_ptr[i] = i * deg;
    for (int64_t e = 0; e < n * deg; ++e) col[e] = (int32_t)(sm64(s0 + (uint64_t)e) % (uint64_t)n);
}

// ============================================================ distance.rs
float orc_distance(const float* a, const float* b, int64_t d, int32_t metric) {
    switch (metric) {
        case M_L2: {  // (x-y)*(x-y) summed in order, sqrt   (distance.rs:37-41)
            float s = 0.0f;
            for (int64_t i = 0; i < d; ++i) { const float t = a[i] - b[i]; s = s + t * t; }
            return std::sqrt(s);
        }
        case M_COS: {  // (distance.rs:55-62)
            float dot = 0.0f, na = 0.0f, nb = 0.0f;
            for (int64_t i = 0; i < d; ++i) dot = dot + a[i] * b[i];
            for (int64_t i = 0; i < d; ++i) na = na + a[i] * a[i];
            for (int64_t i = 0; i < d; ++i) nb = nb + b[i] * b[i];
            na = std::sqrt(na);
            nb = std::sqrt(nb);
            if (na > 1e-8f && nb > 1e-8f) return 1.0f - (dot / (na * nb));
            return 1.0f;
        }
        case M_DOT: {  // (distance.rs:77-78)
            float dot = 0.0f;
            for (int64_t i = 0; i < d; ++i) dot = dot + a[i] * b[i];
            return -dot;
        }
        case M_L1: {  // (distance.rs:85)
            float s = 0.0f;
            for (int64_t i = 0; i < d; ++i) s = s + std::fabs(a[i] - b[i]);
            return s;
        }
    }
    return std::numeric_limits<float>::quiet_NaN();
}

void orc_distance_matrix(const float* q, int64_t nq, const float* x, int64_t n, int64_t d, int32_t metric, float* out,
                         int32_t nthreads) {
    pfor(nq, nthreads, [&](int64_t i) {
        for (int64_t j = 0; j < n; ++j) out[i * n + j] = orc_distance(q + i * d, x + j * d, d, metric);
    });
}

// FlatIndex::search (index/flat.rs:36-76): distance to every live vector, sort
// ascending, truncate to k (ties by id).
void orc_flat_search(const float* base, int64_t n, int64_t d, int32_t metric, const uint8_t* deleted, const float* q,
                     int64_t nq, int32_t k, int64_t* out_ids, float* out_d, int32_t nthreads) {
    pfor(nq, nthreads, [&](int64_t qi) {
        std::vector<Cand> c;
        c.reserve(n);
        for (int64_t j = 0; j < n; ++j) {
            if (deleted && deleted[j]) continue;
            c.push_back({orc_distance(q + qi * d, base + j * d, d, metric), j});
        }
        const int64_t kk = std::min<int64_t>(k, (int64_t)c.size());
        std::partial_sort(c.begin(), c.begin() + kk, c.end(), cand_less);
        for (int64_t s = 0; s < k; ++s) {
            out_ids[qi * k + s] = s < kk ? c[s].id : -1;
            out_d[qi * k + s] = s < kk ? c[s].d : INFINITY;
        }
    });
}

// FlatIndex::search CPU baseline in fast mode (SIMD distances, all threads over
// row blocks like rayon's par_iter over the vectors, flat.rs:39-49; per-block
// top-k merged). Queries go in batches of 16 so each row is read once per batch.
void orc_flat_search_fast(const float* base, int64_t n, int64_t d, int32_t metric, const float* q, int64_t nq, int32_t k,
                          int64_t* out_ids, float* out_d, int32_t nthreads) {
    const int64_t QB = 16, RB = 8192;
    for (int64_t q0 = 0; q0 < nq; q0 += QB) {
        const int64_t nb = std::min(QB, nq - q0);
        const int64_t blocks = (n + RB - 1) / RB;
        std::vector<std::vector<Cand>> part((size_t)blocks * nb);
        pfor(blocks, nthreads, [&](int64_t bi) {
            const int64_t r0 = bi * RB, r1 = std::min(n, r0 + RB);
            std::vector<std::priority_queue<Cand, std::vector<Cand>, CandMax>> heap(nb);
            for (int64_t j = r0; j < r1; ++j)
                for (int64_t t = 0; t < nb; ++t) {
                    const Cand c{fast_distance(q + (q0 + t) * d, base + j * d, d, metric), j};
                    auto& h = heap[t];
                    if ((int)h.size() < k) h.push(c);
                    else if (cand_less(c, h.top())) { h.pop(); h.push(c); }
                }
            for (int64_t t = 0; t < nb; ++t) {
                auto& v = part[(size_t)(bi * nb + t)];
                while (!heap[t].empty()) { v.push_back(heap[t].top()); heap[t].pop(); }
            }
        });
        for (int64_t t = 0; t < nb; ++t) {
            std::vector<Cand> all;
            for (int64_t bi = 0; bi < blocks; ++bi) {
                const auto& v = part[(size_t)(bi * nb + t)];
                all.insert(all.end(), v.begin(), v.end());
            }
            const int64_t kk = std::min<int64_t>(k, (int64_t)all.size());
            std::partial_sort(all.begin(), all.begin() + kk, all.end(), cand_less);
            for (int64_t s2 = 0; s2 < k; ++s2) {
                out_ids[(q0 + t) * k + s2] = s2 < kk ? all[s2].id : -1;
                out_d[(q0 + t) * k + s2] = s2 < kk ? all[s2].d : INFINITY;
            }
        }
    }
}

}  // extern "C"

// ============================================================ hnsw_rs 0.3.3
namespace {

struct OHnsw {
    int64_t d = 0;
    int metric = 0, M = 0, ef_c = 0, max_layer = 0;
    uint64_t seed = 0;
    std::vector<float> data;
    std::vector<uint8_t> level;
    // nb[p][l]: neighbour list of point p at layer l, kept sorted by distance
    // to p (hnsw.rs:1186, 1268). Every point owns max_layer+1 lists, as
    // Point::neighbours does.
    std::vector<std::vector<std::vector<Cand>>> nb;
    std::unique_ptr<std::mutex[]> locks;
    std::vector<std::atomic<int64_t>> count_at_level;  // points_by_layer[l].len()
    std::mutex entry_mu;
    int64_t entry = -1;
    int entry_level = -1;

    OHnsw() : count_at_level(17) {}
    const float* v(int64_t i) const { return data.data() + i * d; }
    bool fast = false;  // CPU-baseline SIMD distances (not the reference order)
    // query-path stop rule: (d, id) as the GPU's R-only search (default), or the
    // reference's distance-only test (hnsw.rs:913-1055, ties in heap order)
    bool lex_stop = true;
    float dist(const float* a, int64_t j) const {
        return fast ? fast_distance(a, v(j), d, metric) : orc_distance(a, v(j), d, metric);
    }
};

// LayerGenerator::generate (hnsw.rs:358-369): floor(-ln(U) / ln(M)), redrawn
// uniformly in [0, maxlevel) when >= maxlevel. The reference seeds from
// entropy; here U comes from a seeded counter stream.
int gen_level(const OHnsw& h, int64_t i) {
    const double scale = 1.0 / std::log((double)h.M);
    const double u = (double)(sm64(sm64(h.seed) + (uint64_t)i) >> 11) * (1.0 / 9007199254740992.0);
    const double lev = -std::log(u) * scale;
    int64_t ul = std::isfinite(lev) ? (int64_t)std::floor(lev) : (int64_t)1 << 40;
    if (ul >= h.max_layer) ul = (int64_t)(sm64(sm64(h.seed ^ 0xABCDEFull) + (uint64_t)i) % (uint64_t)h.max_layer);
    return (int)ul;
}

std::vector<Cand> copy_list(const OHnsw& h, int64_t p, int l) {
    std::lock_guard<std::mutex> lk(h.locks[p]);
    return h.nb[p][l];
}

// search_layer (hnsw.rs:913-1055), no filter. Returns R sorted ascending.
// lex_stop (the query path, Hnsw::search): stop when the popped candidate is
// beyond R's farthest in the (d, id) order rather than by distance alone — the
// two differ only on an exact distance tie with the farthest, where the
// reference's heap order is unspecified; the GPU search uses this rule.
std::vector<Cand> search_layer(const OHnsw& h, const float* q, int64_t ep, int ef, int layer, bool lex_stop = false) {
    std::vector<Cand> out;
    if (h.count_at_level[layer].load() == 0) return out;  // points_by_layer[layer].is_empty()
    std::priority_queue<Cand, std::vector<Cand>, CandMax> R;
    std::priority_queue<Cand, std::vector<Cand>, CandMin> C;
    std::unordered_set<int64_t> visited;
    const float d0 = h.dist(q, ep);
    visited.insert(ep);
    C.push({d0, ep});
    R.push({d0, ep});
    while (!C.empty()) {
        const Cand c = C.top();
        C.pop();
        const Cand f = R.top();
        if (c.d > f.d || (lex_stop && c.d == f.d && c.id > f.id)) break;  // -(c.dist_to_ref) > f.dist_to_ref -> return
        const std::vector<Cand> lst = copy_list(h, c.id, layer);
        for (const Cand& e : lst) {
            if (!visited.insert(e.id).second) continue;
            const Cand ff = R.top();
            const float de = h.dist(q, e.id);
            if (de < ff.d || (int)R.size() < ef) {
                C.push({de, e.id});
                R.push({de, e.id});
                if ((int)R.size() > ef) R.pop();
            }
        }
    }
    out.resize(R.size());
    for (int64_t i = (int64_t)out.size() - 1; i >= 0; --i) { out[i] = R.top(); R.pop(); }
    return out;
}

// select_neighbours (hnsw.rs:1287-1409) with extend_candidates = keep_pruned = false.
std::vector<Cand> select_neighbours(const OHnsw& h, const std::vector<Cand>& cand_sorted, int nb_conn) {
    std::vector<Cand> nbv;
    if ((int)cand_sorted.size() <= nb_conn) return cand_sorted;  // transfer in pop order
    for (const Cand& e : cand_sorted) {
        if ((int)nbv.size() >= nb_conn) break;
        bool insert = true;
        if (!nbv.empty()) {
            const float* ev = h.v(e.id);
            for (const Cand& dd : nbv)
                if (h.dist(ev, dd.id) <= e.d) { insert = false; break; }
        }
        if (insert) nbv.push_back(e);
    }
    return nbv;
}

void insert_point(OHnsw& h, int64_t p) {
    const int level = h.level[p];
    h.count_at_level[level].fetch_add(1);  // generate_new_point pushes into points_by_layer
    int64_t ep;
    int max_obs;
    {
        std::lock_guard<std::mutex> lk(h.entry_mu);
        if (h.entry < 0) {  // first point: check_entry_point and return (hnsw.rs:1091-1095)
            h.entry = p;
            h.entry_level = level;
            return;
        }
        ep = h.entry;
        max_obs = h.entry_level;
    }
    const float* q = h.v(p);
    float dist_to_entry = h.dist(q, ep);
    for (int l = max_obs; l >= level + 1; --l) {  // greedy descent, ef = 1 (hnsw.rs:1105-1146)
        std::vector<Cand> sp = search_layer(h, q, ep, 1, l);
        if (!sp.empty()) {
            const Cand e = sp[0];
            {
                std::lock_guard<std::mutex> lk(h.locks[p]);
                if ((int)h.nb[p][l].size() < h.M) h.nb[p][l].push_back(e);
            }
            const float tmp = h.dist(q, e.id);
            if (tmp < dist_to_entry) { ep = e.id; dist_to_entry = tmp; }
        }
    }
    for (int l = level; l >= 0; --l) {  // (hnsw.rs:1149-1196)
        std::vector<Cand> sp = search_layer(h, q, ep, h.ef_c, l);
        if (sp.empty()) continue;
        const int nb_conn = l == 0 ? 2 * h.M : h.M;
        std::vector<Cand> nbv = select_neighbours(h, sp, nb_conn);
        std::sort(nbv.begin(), nbv.end(), cand_less);
        {
            std::lock_guard<std::mutex> lk(h.locks[p]);
            h.nb[p][l] = nbv;
        }
        if (!nbv.empty()) ep = nbv[0].id;
    }
    // reverse_update_neighborhood_simple (hnsw.rs:1229-1277): the new point is
    // added at ITS OWN level l_n in every neighbour's lists, for all l.
    for (int l = level; l >= 0; --l) {
        const std::vector<Cand> mine = copy_list(h, p, l);
        for (const Cand& qn : mine) {
            if (qn.id == p) continue;
            std::lock_guard<std::mutex> lk(h.locks[qn.id]);
            auto& lst = h.nb[qn.id][level];
            bool already = false;
            for (const Cand& o : lst)
                if (o.id == p) { already = true; break; }
            if (already) continue;
            lst.push_back({qn.d, p});
            const int threshold = level > 0 ? h.M : 2 * h.M;
            const bool shrink = (int)lst.size() > threshold;
            std::sort(lst.begin(), lst.end(), cand_less);
            if (shrink) lst.pop_back();
        }
    }
    std::lock_guard<std::mutex> lk(h.entry_mu);  // check_entry_point (hnsw.rs:529-552)
    if (level > h.entry_level) { h.entry = p; h.entry_level = level; }
}

}  // namespace

extern "C" {

// HnswIndex::new wiring (crates/ruvector-core/src/index/hnsw.rs:102-108): the
// caller passes max_layer = min(16, dimensions) (NB_LAYER_MAX, hnsw.rs:41,773).
void* orc_hnsw_new(int64_t d, int32_t metric, int32_t m, int32_t ef_c, int32_t max_layer, uint64_t seed) {
    auto* h = new OHnsw();
    h->d = d; h->metric = metric; h->M = m; h->ef_c = ef_c; h->seed = seed;
    h->max_layer = std::max(1, std::min(16, max_layer));
    return h;
}

void orc_hnsw_free(void* hp) { delete static_cast<OHnsw*>(hp); }

// CPU-baseline fast mode: SIMD distances for build and search (bench only).
void orc_hnsw_set_fast(void* hp, int32_t on) { static_cast<OHnsw*>(hp)->fast = on != 0; }
void orc_hnsw_set_lex_stop(void* hp, int32_t on) { static_cast<OHnsw*>(hp)->lex_stop = on != 0; }
int32_t orc_simd_width() { return g_avx512 ? 512 : 256; }

// Sequential add_batch (index/hnsw.rs:314-319) for nthreads <= 1, otherwise
// Hnsw::parallel_insert (hnsw.rs:1212-1218) semantics.
void orc_hnsw_insert(void* hp, const float* vecs, int64_t n, int32_t nthreads) {
    OHnsw& h = *static_cast<OHnsw*>(hp);
    const int64_t base = (int64_t)h.level.size();
    h.data.insert(h.data.end(), vecs, vecs + n * h.d);
    h.level.resize(base + n);
    h.nb.resize(base + n);
    std::unique_ptr<std::mutex[]> nl(new std::mutex[base + n]);
    h.locks = std::move(nl);
    for (int64_t i = base; i < base + n; ++i) {
        h.level[i] = (uint8_t)gen_level(h, i);
        h.nb[i].resize(h.max_layer + 1);
    }
    if (nthreads <= 1) {
        for (int64_t i = base; i < base + n; ++i) insert_point(h, i);
    } else {
        // first point alone so the entry exists
        int64_t start = base;
        if (h.entry < 0 && n > 0) { insert_point(h, base); start = base + 1; }
        pfor(base + n - start, nthreads, [&](int64_t t) { insert_point(h, start + t); });
    }
}

// search (hnsw.rs:1587) -> search_filter (hnsw.rs:1475-1570), no filter.
void orc_hnsw_search(void* hp, const float* q, int64_t nq, int32_t k, int32_t ef_arg, int64_t* out_ids, float* out_d,
                     int32_t* out_n, int32_t nthreads) {
    const OHnsw& h = *static_cast<OHnsw*>(hp);
    pfor(nq, nthreads, [&](int64_t qi) {
        const float* qv = q + qi * h.d;
        int64_t* oi = out_ids + qi * k;
        float* od = out_d + qi * k;
        for (int s = 0; s < k; ++s) { oi[s] = -1; od[s] = INFINITY; }
        if (h.entry < 0) { if (out_n) out_n[qi] = 0; return; }
        float dist_to_entry = h.dist(qv, h.entry);
        int64_t pivot = h.entry;
        for (int layer = h.entry_level; layer >= 1; --layer) {  // single pass (hnsw.rs:1499-1517)
            int64_t newp = -1;
            const std::vector<Cand> lst = copy_list(h, pivot, layer);
            for (const Cand& n : lst) {
                const float tmp = h.dist(qv, n.id);
                if (tmp < dist_to_entry) { newp = n.id; dist_to_entry = tmp; }
            }
            if (newp >= 0) pivot = newp;
        }
        const int ef = std::max(ef_arg, k);
        int layer_to_search = 0;
        while (layer_to_search < 16 && h.count_at_level[layer_to_search].load() == 0) ++layer_to_search;
        const std::vector<Cand> r = search_layer(h, qv, pivot, ef, layer_to_search, h.lex_stop);
        const int last = std::min<int64_t>(std::min(k, ef), (int64_t)r.size());
        for (int s = 0; s < last; ++s) { oi[s] = r[s].id; od[s] = r[s].d; }
        if (out_n) out_n[qi] = last;
    });
}

// Graph export in the rvx_hnsw_graph layout. Upper layer l lists every point
// whose layer-l list is non-empty (hnsw_rs keeps lists above a point's level
// that search can still reach), ids ascending.
void orc_hnsw_export_sizes(void* hp, int64_t* n, int32_t* max_level, int64_t* entry, int64_t* e0,
                           int64_t* upper_count /*[17]*/, int64_t* upper_edges /*[17]*/) {
    const OHnsw& h = *static_cast<OHnsw*>(hp);
    const int64_t N = (int64_t)h.level.size();
    *n = N;
    *max_level = std::max(0, h.entry_level);
    *entry = h.entry;
    int64_t e = 0;
    for (int64_t i = 0; i < N; ++i) e += (int64_t)h.nb[i][0].size();
    *e0 = e;
    for (int l = 0; l <= 16; ++l) { upper_count[l] = 0; upper_edges[l] = 0; }
    for (int l = 1; l <= *max_level; ++l)
        for (int64_t i = 0; i < N; ++i)
            if (l <= h.max_layer && !h.nb[i][l].empty()) { upper_count[l]++; upper_edges[l] += (int64_t)h.nb[i][l].size(); }
}

void orc_hnsw_export(void* hp, uint8_t* levels, int64_t* rp0, int32_t* col0, float* dist0, int32_t* up_ids,
                     int64_t* up_rp, int32_t* up_col) {
    const OHnsw& h = *static_cast<OHnsw*>(hp);
    const int64_t N = (int64_t)h.level.size();
    std::memcpy(levels, h.level.data(), N);
    int64_t e = 0;
    rp0[0] = 0;
    for (int64_t i = 0; i < N; ++i) {
        for (const Cand& c : h.nb[i][0]) { col0[e] = (int32_t)c.id; if (dist0) dist0[e] = c.d; ++e; }
        rp0[i + 1] = e;
    }
    int64_t oi = 0, orp = 0, oc = 0;
    for (int l = 1; l <= std::max(0, h.entry_level); ++l) {
        int64_t local = 0;
        up_rp[orp++] = 0;
        for (int64_t i = 0; i < N; ++i) {
            if (l > h.max_layer || h.nb[i][l].empty()) continue;
            up_ids[oi++] = (int32_t)i;
            for (const Cand& c : h.nb[i][l]) { up_col[oc++] = (int32_t)c.id; ++local; }
            up_rp[orp++] = local;
        }
    }
}

// Build a searchable handle from an exported graph (e.g. one built on the GPU).
void* orc_hnsw_from_graph(const float* vecs, int64_t n, int64_t d, int32_t metric, const uint8_t* levels, int64_t entry,
                          int32_t max_level, const int64_t* rp0, const int32_t* col0, const int64_t* upper_count,
                          const int32_t* up_ids, const int64_t* up_rp, const int32_t* up_col) {
    auto* h = new OHnsw();
    h->d = d; h->metric = metric; h->M = 16; h->ef_c = 0; h->max_layer = 16;
    h->data.resize((size_t)(n * d));
    h->level.assign(levels, levels + n);
    h->nb.resize(n);
    std::unique_ptr<std::mutex[]> nl(new std::mutex[std::max<int64_t>(n, 1)]);
    h->locks = std::move(nl);
    // rows and layer-0 lists in parallel (a 10M-node graph is the C3 CPU baseline's input)
    const int threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const int64_t blk = 65536;
    pfor((n + blk - 1) / blk, threads, [&](int64_t b) {
        const int64_t i0 = b * blk, i1 = std::min(n, i0 + blk);
        std::copy(vecs + i0 * d, vecs + i1 * d, h->data.begin() + i0 * d);
        for (int64_t i = i0; i < i1; ++i) {
            h->nb[i].resize(17);
            h->count_at_level[levels[i]].fetch_add(1);
            h->nb[i][0].reserve((size_t)(rp0[i + 1] - rp0[i]));
            for (int64_t p = rp0[i]; p < rp0[i + 1]; ++p) h->nb[i][0].push_back({0.0f, col0[p]});
        }
    });
    int64_t oi = 0, orp = 0, oc = 0;
    for (int l = 1; l <= max_level; ++l) {
        const int64_t cnt = upper_count[l];
        const int64_t* rp = up_rp + orp;
        for (int64_t t = 0; t < cnt; ++t) {
            const int64_t id = up_ids[oi + t];
            for (int64_t p = rp[t]; p < rp[t + 1]; ++p) h->nb[id][l].push_back({0.0f, up_col[oc + p]});
        }
        oi += cnt;
        oc += rp[cnt];
        orp += cnt + 1;
    }
    h->entry = entry;
    h->entry_level = max_level;
    return h;
}

// ============================================================ ruvector-postgres gnn
// GraphSAGELayer::with_aggregator deterministic init (graphsage.rs:56-78),
// GCNLayer::new_with_normalize (gcn.rs:32-41) is offset 0.
void orc_sage_init(int32_t in, int32_t out, int32_t offset, float* w /*[in][out]*/) {
    const float scale = std::sqrt(2.0f / (float)(in + out));
    for (int64_t i = 0; i < in; ++i)
        for (int64_t j = 0; j < out; ++j) {
            const float val = std::fmod((float)(uint64_t)(i * out + j + offset) * 0.01f, 1.0f);
            w[i * out + j] = (val - 0.5f) * scale;
        }
}

// build_adjacency_list (message_passing.rs:34-50) as a CSR: adj[dst].push(src)
// in edge order, edges with an out-of-range endpoint dropped. Returns E kept.
int64_t orc_build_csr(int64_t n, const int64_t* src, const int64_t* dst, int64_t ne, const float* w, int64_t* rp,
                      int32_t* col, float* wout) {
    std::vector<int64_t> cnt(n + 1, 0);
    for (int64_t e = 0; e < ne; ++e)
        if (src[e] >= 0 && src[e] < n && dst[e] >= 0 && dst[e] < n) cnt[dst[e] + 1]++;
    for (int64_t i = 0; i < n; ++i) cnt[i + 1] += cnt[i];
    for (int64_t i = 0; i <= n; ++i) rp[i] = cnt[i];
    std::vector<int64_t> fill(cnt.begin(), cnt.end() - 1);
    for (int64_t e = 0; e < ne; ++e) {
        if (!(src[e] >= 0 && src[e] < n && dst[e] >= 0 && dst[e] < n)) continue;
        const int64_t p = fill[dst[e]]++;
        col[p] = (int32_t)src[e];
        if (w && wout) wout[p] = w[e];
    }
    return cnt[n];
}

// sum_aggregate / mean_aggregate / max_aggregate (aggregators.rs:35-92) over
// each CSR row; weighted_aggregate (:104-128) scales each message first.
// Empty rows: zeros, or x_i when keep_isolated (propagate, message_passing.rs:75-78).
void orc_aggregate(const float* x, int64_t n, int32_t dim, const int64_t* rp, const int32_t* col, const float* w,
                   int32_t method /*0 sum 1 mean 2 max*/, int32_t keep_isolated, float* out) {
    for (int64_t i = 0; i < n; ++i) {
        float* o = out + i * dim;
        const int64_t beg = rp[i], end = rp[i + 1];
        if (beg == end) {
            for (int c = 0; c < dim; ++c) o[c] = keep_isolated ? x[i * dim + c] : 0.0f;
            continue;
        }
        for (int c = 0; c < dim; ++c) o[c] = method == 2 ? -INFINITY : 0.0f;
        for (int64_t e = beg; e < end; ++e) {
            const float* xv = x + (int64_t)col[e] * dim;
            for (int c = 0; c < dim; ++c) {
                const float v = w ? xv[c] * w[e] : xv[c];
                o[c] = method == 2 ? std::fmax(o[c], v) : o[c] + v;
            }
        }
        if (method == 1) {
            const float cnt = (float)(end - beg);
            for (int c = 0; c < dim; ++c) o[c] = o[c] / cnt;
        }
    }
}

// ---- rand 0.8.5 StdRng::seed_from_u64 + SliceRandom::partial_shuffle -----
// (third-party, not vendored under /root/reference: rand 0.8.5 / rand_core
// 0.6 / rand_chacha 0.3.1, Cargo.lock:6952,6993; called by
// GraphSAGELayer::sample_neighbors, graphsage.rs:92-102). Restated from the
// published algorithms:
//  * StdRng = ChaCha12Rng: ChaCha block function, 12 rounds, 256-bit key =
//    the 32-byte seed, 64-bit block counter (words 12-13) from 0, zero nonce;
//    next_u32 returns the keystream's little-endian words in order.
//  * SeedableRng::seed_from_u64 (rand_core 0.6): the seed is eight PCG32
//    outputs (state = state*6364136223846793005 + 11634580027462260723,
//    xorshifted = ((s>>18)^s)>>27, rotr by s>>59), each stored little-endian.
//  * gen_range(0..ub) for u32 (UniformInt::sample_single_inclusive): range
//    = ub, zone = (range << lzcnt(range)) - 1; draw v until lo32(v*range)
//    <= zone, return hi32(v*range).
//  * partial_shuffle(amount): for i in (len-amount..len).rev() swap(i,
//    gen_index(i+1)); the reference then keeps sampled[..k] (the prefix).
struct OrcChaCha {
    uint32_t key[8];
    uint64_t counter = 0;
    uint32_t buf[16];
    int idx = 16, rounds = 12;
    static uint32_t rotl(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }
    void refill() {
        uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
        for (int i = 0; i < 8; ++i) s[4 + i] = key[i];
        s[12] = (uint32_t)counter;
        s[13] = (uint32_t)(counter >> 32);
        s[14] = s[15] = 0;
        uint32_t w[16];
        std::memcpy(w, s, sizeof w);
        auto qr = [&](int a, int b, int c, int d) {
            w[a] += w[b]; w[d] = rotl(w[d] ^ w[a], 16);
            w[c] += w[d]; w[b] = rotl(w[b] ^ w[c], 12);
            w[a] += w[b]; w[d] = rotl(w[d] ^ w[a], 8);
            w[c] += w[d]; w[b] = rotl(w[b] ^ w[c], 7);
        };
        for (int r = 0; r < rounds; r += 2) {
            qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15);
            qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14);
        }
        for (int i = 0; i < 16; ++i) buf[i] = w[i] + s[i];
        ++counter;
        idx = 0;
    }
    uint32_t next_u32() {
        if (idx >= 16) refill();
        return buf[idx++];
    }
    void seed_from_u64(uint64_t state) {
        for (int i = 0; i < 8; ++i) {
            state = state * 6364136223846793005ull + 11634580027462260723ull;
            const uint32_t xs = (uint32_t)(((state >> 18) ^ state) >> 27);
            const uint32_t rot = (uint32_t)(state >> 59);
            key[i] = (xs >> rot) | (xs << ((32 - rot) & 31));
        }
        counter = 0;
        idx = 16;
    }
    uint32_t gen_index(uint32_t ub) {
        const uint32_t range = ub;
        const uint32_t zone = (range << __builtin_clz(range)) - 1u;
        for (;;) {
            const uint64_t m = (uint64_t)next_u32() * range;
            if ((uint32_t)m <= zone) return (uint32_t)(m >> 32);
        }
    }
};

// ChaCha keystream words (rounds 20 = the RFC 7539 / rand_chacha known-answer
// vectors, 12 = StdRng) for a given 8-word key, from block 0.
void orc_chacha_words(const uint32_t* key, int32_t rounds, int32_t nwords, uint32_t* out) {
    OrcChaCha r;
    std::memcpy(r.key, key, sizeof r.key);
    r.rounds = rounds;
    for (int i = 0; i < nwords; ++i) out[i] = r.next_u32();
}

// GraphSAGELayer::sample_neighbors (graphsage.rs:92-102) on positions
// 0..len-1: writes the k positions the reference keeps (len > k).
void orc_sage_sample_positions(int32_t len, int32_t k, int32_t* out) {
    std::vector<int32_t> a(len);
    for (int i = 0; i < len; ++i) a[i] = i;
    OrcChaCha r;
    r.seed_from_u64(42);
    for (int i = len - 1; i >= len - k; --i) std::swap(a[i], a[r.gen_index((uint32_t)i + 1)]);
    for (int t = 0; t < k; ++t) out[t] = a[t];
}

// GraphSAGELayer::forward_with_sampling (graphsage.rs:118-187) for rows
// [row0, row0+nrows); num_samples = k (rows with more than k neighbours
// aggregate the reference's sample_neighbors subset, in its order).
// aggregator 0 = Mean (and LSTM, :159), 1 = MaxPool.
void orc_sage_forward(const float* x, int64_t n, int32_t in, int32_t out, const int64_t* rp, const int32_t* col,
                      const float* wn, const float* ws, int32_t aggregator, int32_t normalize, int64_t row0,
                      int64_t nrows, float* y /*[nrows][out]*/, int32_t nthreads, int32_t num_samples) {
    std::mutex pm;
    std::map<int64_t, std::vector<int32_t>> pos_cache;
    pfor(nrows, nthreads, [&](int64_t t) {
        const int64_t i = row0 + t;
        std::vector<float> agg(in, 0.0f);
        // sampled neighbour list (sample_neighbors), then the id < n filter (:139-147)
        std::vector<int32_t> nb(col + rp[i], col + rp[i + 1]);
        if ((int64_t)nb.size() > num_samples) {
            std::vector<int32_t> pos;
            {
                std::lock_guard<std::mutex> lk(pm);
                auto& c = pos_cache[(int64_t)nb.size()];
                if (c.empty()) {
                    c.resize(num_samples);
                    orc_sage_sample_positions((int32_t)nb.size(), num_samples, c.data());
                }
                pos = c;
            }
            std::vector<int32_t> s(num_samples);
            for (int q = 0; q < num_samples; ++q) s[q] = nb[pos[q]];
            nb.swap(s);
        }
        const int64_t beg = 0, end = (int64_t)nb.size();
        const int32_t* colr = nb.data();
        int64_t cnt = 0;
        for (int64_t e = beg; e < end; ++e) if (colr[e] < n) ++cnt;
        if (cnt > 0) {
            if (aggregator == 1) {  // max_aggregate (aggregators.rs:77-92)
                std::fill(agg.begin(), agg.end(), -INFINITY);
                for (int64_t e = beg; e < end; ++e) {
                    if (colr[e] >= n) continue;
                    const float* xv = x + (int64_t)colr[e] * in;
                    for (int c = 0; c < in; ++c) agg[c] = std::fmax(agg[c], xv[c]);
                }
            } else {  // mean_aggregate: sum then / count (aggregators.rs:35-68)
                for (int64_t e = beg; e < end; ++e) {
                    if (colr[e] >= n) continue;
                    const float* xv = x + (int64_t)colr[e] * in;
                    for (int c = 0; c < in; ++c) agg[c] = agg[c] + xv[c];
                }
                const float cf = (float)cnt;
                for (int c = 0; c < in; ++c) agg[c] = agg[c] / cf;
            }
        }
        // linear_transform (graphsage.rs:105-115): result[j] += f_i * W[i][j], i outer
        std::vector<float> nh(out, 0.0f), sh(out, 0.0f);
        const float* xi = x + i * in;
        for (int64_t a = 0; a < in; ++a) {
            const float f = agg[a];
            const float* wr = wn + a * out;
            for (int64_t j = 0; j < out; ++j) nh[j] = nh[j] + f * wr[j];
        }
        for (int64_t a = 0; a < in; ++a) {
            const float f = xi[a];
            const float* wr = ws + a * out;
            for (int64_t j = 0; j < out; ++j) sh[j] = sh[j] + f * wr[j];
        }
        float* yo = y + t * out;
        for (int64_t j = 0; j < out; ++j) yo[j] = std::fmax(nh[j] + sh[j], 0.0f);
        if (normalize) {  // (graphsage.rs:177-182)
            float s = 0.0f;
            for (int64_t j = 0; j < out; ++j) s = s + yo[j] * yo[j];
            const float norm = std::sqrt(s);
            if (norm > 0.0f)
                for (int64_t j = 0; j < out; ++j) yo[j] = yo[j] / norm;
        }
    });
}

// GCNLayer::forward (gcn.rs:93-112) via propagate(_weighted) (message_passing.rs:61-162).
void orc_gcn_forward(const float* x, int64_t n, int32_t in, int32_t out, const int64_t* rp, const int32_t* col,
                     const float* ew /*nullable*/, const float* w /*[in][out]*/, const float* bias /*nullable*/,
                     int32_t normalize, float* y /*[n][out or in]*/, int32_t nthreads) {
    pfor(n, nthreads, [&](int64_t i) {
        const int64_t beg = rp[i], end = rp[i + 1];
        if (end == beg) {  // disconnected node: features unchanged, then ReLU
            for (int c = 0; c < in; ++c) y[i * out + c] = std::fmax(x[i * in + c], 0.0f);
            return;
        }
        std::vector<float> agg(in, 0.0f);
        for (int64_t e = beg; e < end; ++e) {
            const float wt = ew ? ew[e] : 1.0f;
            const float* xv = x + (int64_t)col[e] * in;
            for (int c = 0; c < in; ++c) agg[c] = agg[c] + xv[c] * wt;  // message x*w, sum_aggregate
        }
        if (normalize) {
            const float nrm = 1.0f / std::sqrt((float)(end - beg));
            for (int c = 0; c < in; ++c) agg[c] = agg[c] * nrm;
        }
        std::vector<float> r(out, 0.0f);
        for (int64_t a = 0; a < in; ++a)
            for (int64_t j = 0; j < out; ++j) r[j] = r[j] + agg[a] * w[a * out + j];
        if (bias)
            for (int64_t j = 0; j < out; ++j) r[j] = r[j] + bias[j];
        for (int64_t j = 0; j < out; ++j) y[i * out + j] = std::fmax(r[j], 0.0f);
    });
}

// ============================================================ ruvector-gnn layer.rs
struct orc_rvl {
    int32_t in, H, heads, hd;
    float dropout, eps;
    const float *w_msg, *b_msg, *w_agg, *b_agg;
    const float *w_z, *b_wz, *u_z, *b_uz, *w_r, *b_wr, *u_r, *b_ur, *w_h, *b_wh, *u_h, *b_uh;
    const float *q, *bq, *k, *bk, *v, *bv, *o, *bo;
    const float *gamma, *beta;
};

}  // extern "C"

namespace {

// Linear::forward (layer.rs:37-41): ndarray W.dot(x) + b
std::vector<float> linear(const float* W, const float* b, int out, int in, const float* x) {
    std::vector<float> y(out);
    for (int r = 0; r < out; ++r) y[r] = unrolled_dot(W + (int64_t)r * in, x, in) * 1.0f + b[r];
    return y;
}
// LayerNorm::forward (layer.rs:68-81)
std::vector<float> layer_norm(const orc_rvl& L, const std::vector<float>& x) {
    const int n = (int)x.size();
    const float mean = unrolled_sum(x.data(), n) / (float)n;
    float var = 0.0f;
    for (int i = 0; i < n; ++i) { const float dd = x[i] - mean; var = var + dd * dd; }
    var = var / (float)n;
    std::vector<float> y(n);
    for (int i = 0; i < n; ++i) {
        const float nz = (x[i] - mean) / std::sqrt(var + L.eps);
        y[i] = L.gamma[i] * nz + L.beta[i];
    }
    return y;
}
float sigmoid(float x) {  // GRUCell::sigmoid (layer.rs:278-285)
    if (x > 0.0f) return 1.0f / (1.0f + std::exp(-x));
    const float ex = std::exp(x);
    return ex / (1.0f + ex);
}

}  // namespace

extern "C" {

// RuvectorLayer::forward (layer.rs:379-418) for one node.
void orc_rvl_forward_one(const orc_rvl* Lp, const float* node, const float* nbrs, int32_t deg, const float* wts,
                         int32_t nw, float* out) {
    const orc_rvl& L = *Lp;
    const int H = L.H, in = L.in;
    std::vector<float> node_msg = linear(L.w_msg, L.b_msg, H, in, node);
    if (deg == 0) {
        std::vector<float> y = layer_norm(L, node_msg);
        std::memcpy(out, y.data(), H * 4);
        return;
    }
    std::vector<std::vector<float>> msgs(deg);
    for (int j = 0; j < deg; ++j) msgs[j] = linear(L.w_msg, L.b_msg, H, in, nbrs + (int64_t)j * in);
    // MultiHeadAttention::forward (layer.rs:129-160), keys = values = msgs
    std::vector<float> q = linear(L.q, L.bq, H, H, node_msg.data());
    std::vector<std::vector<float>> k(deg), v(deg);
    for (int j = 0; j < deg; ++j) k[j] = linear(L.k, L.bk, H, H, msgs[j].data());
    for (int j = 0; j < deg; ++j) v[j] = linear(L.v, L.bv, H, H, msgs[j].data());
    std::vector<float> concat(H, 0.0f);
    const float scale = std::sqrt((float)L.hd);
    for (int h = 0; h < L.heads; ++h) {  // scaled_dot_product_attention (layer.rs:174-210)
        std::vector<float> scores(deg);
        for (int j = 0; j < deg; ++j) {
            float dot = 0.0f;
            for (int c = 0; c < L.hd; ++c) dot = dot + q[h * L.hd + c] * k[j][h * L.hd + c];
            scores[j] = dot / scale;
        }
        float mx = -INFINITY;
        for (float s : scores) mx = std::fmax(mx, s);
        std::vector<float> ex(deg);
        for (int j = 0; j < deg; ++j) ex[j] = std::exp(scores[j] - mx);
        float sum = 0.0f;
        for (float e : ex) sum = sum + e;
        sum = std::fmax(sum, 1e-10f);
        for (int j = 0; j < deg; ++j) {
            const float a = ex[j] / sum;
            for (int c = 0; c < L.hd; ++c) concat[h * L.hd + c] = concat[h * L.hd + c] + a * v[j][h * L.hd + c];
        }
    }
    std::vector<float> att = linear(L.o, L.bo, H, H, concat.data());
    // aggregate_messages (layer.rs:421-445)
    std::vector<float> wagg(H, 0.0f);
    if (nw > 0) {
        float wsum = 0.0f;
        for (int j = 0; j < nw; ++j) wsum = wsum + wts[j];
        const int m = std::min(deg, nw);
        for (int j = 0; j < m; ++j) {
            const float wj = wsum > 0.0f ? wts[j] / wsum : 1.0f / (float)nw;
            for (int c = 0; c < H; ++c) wagg[c] = wagg[c] + wj * msgs[j][c];
        }
    }
    std::vector<float> combined(H);
    for (int c = 0; c < H; ++c) combined[c] = att[c] + wagg[c];
    std::vector<float> a = linear(L.w_agg, L.b_agg, H, H, combined.data());
    // GRUCell::forward (layer.rs:255-275), hidden = node_msg
    const std::vector<float>& hdn = node_msg;
    std::vector<float> t1 = linear(L.w_z, L.b_wz, H, H, a.data()), t2 = linear(L.u_z, L.b_uz, H, H, hdn.data());
    std::vector<float> z(H), r(H), rh(H), up(H);
    for (int c = 0; c < H; ++c) z[c] = sigmoid(t1[c] + t2[c]);
    t1 = linear(L.w_r, L.b_wr, H, H, a.data());
    t2 = linear(L.u_r, L.b_ur, H, H, hdn.data());
    for (int c = 0; c < H; ++c) r[c] = sigmoid(t1[c] + t2[c]);
    for (int c = 0; c < H; ++c) rh[c] = r[c] * hdn[c];
    t1 = linear(L.w_h, L.b_wh, H, H, a.data());
    t2 = linear(L.u_h, L.b_uh, H, H, rh.data());
    const float keep = 1.0f - L.dropout;
    for (int c = 0; c < H; ++c) {
        const float ht = std::tanh(t1[c] + t2[c]);
        const float omz = 1.0f - z[c];
        const float term1 = omz * hdn[c];
        const float term2 = z[c] * ht;
        up[c] = (term1 + term2) * keep;  // apply_dropout (layer.rs:448-451)
    }
    std::vector<float> y = layer_norm(L, up);
    std::memcpy(out, y.data(), H * 4);
}

// Batched driver over a CSR (edge weights nullable = empty weight slice).
void orc_rvl_forward_graph(const orc_rvl* L, const float* x, int64_t n, const int64_t* rp, const int32_t* col,
                           const float* ew, int64_t row0, int64_t nrows, float* y, int32_t nthreads) {
    pfor(nrows, nthreads, [&](int64_t t) {
        const int64_t i = row0 + t;
        const int64_t beg = rp[i], end = rp[i + 1];
        const int deg = (int)(end - beg);
        std::vector<float> nbrs((size_t)deg * L->in);
        for (int j = 0; j < deg; ++j) std::memcpy(&nbrs[(size_t)j * L->in], x + (int64_t)col[beg + j] * L->in, L->in * 4);
        orc_rvl_forward_one(L, x + i * L->in, nbrs.data(), deg, ew ? ew + beg : nullptr, ew ? deg : 0, y + t * L->H);
    });
}

// ============================================================ search.rs
// cosine_similarity (search.rs:4-26): f32 dot, f64 norms.
float orc_cosine_similarity(const float* a, const float* b, int64_t d) {
    float dot = 0.0f;
    for (int64_t i = 0; i < d; ++i) dot = dot + a[i] * b[i];
    double na2 = 0.0, nb2 = 0.0;
    for (int64_t i = 0; i < d; ++i) na2 = na2 + (double)a[i] * (double)a[i];
    for (int64_t i = 0; i < d; ++i) nb2 = nb2 + (double)b[i] * (double)b[i];
    const float na = (float)std::sqrt(na2), nb = (float)std::sqrt(nb2);
    if (na == 0.0f || nb == 0.0f) return 0.0f;
    return dot / (na * nb);
}

// differentiable_search (search.rs:56-94): idx/w have room for k entries;
// returns the number written.
int32_t orc_differentiable_search(const float* q, const float* cand, int32_t c, int64_t d, int32_t k, float temperature,
                                  int64_t* idx, float* w) {
    if (c == 0) return 0;
    const int kk = std::min(k, c);
    std::vector<float> sims(c);
    for (int j = 0; j < c; ++j) sims[j] = orc_cosine_similarity(q, cand + (int64_t)j * d, d);
    float mx = -INFINITY;
    for (float s : sims) mx = std::fmax(mx, s);
    std::vector<float> ex(c);
    for (int j = 0; j < c; ++j) ex[j] = std::exp((sims[j] - mx) / temperature);
    float sum = 0.0f;
    for (float e : ex) sum = sum + e;
    sum = std::fmax(sum, 1e-10f);
    std::vector<std::pair<int, float>> iw(c);
    for (int j = 0; j < c; ++j) iw[j] = {j, ex[j] / sum};
    std::stable_sort(iw.begin(), iw.end(), [](const std::pair<int, float>& a, const std::pair<int, float>& b) {
        return b.second < a.second;  // descending, stable
    });
    for (int t = 0; t < kk; ++t) { idx[t] = iw[t].first; w[t] = iw[t].second; }
    return kk;
}

// hierarchical_forward (search.rs:105-162) for one query: zip(levels, layers);
// an empty level is skipped; top-min(5, rows) at temperature 1; agg accumulated
// in top-k order (search.rs:133-140); combined = (cur + agg) / 2; then
// RuvectorLayer::forward(combined, top rows, top weights). out has room for the
// largest dim; returns the output dim.
int32_t orc_hierarchical_forward(const orc_rvl* const* layers, int32_t n_layers, const float* const* levels,
                                 const int64_t* level_rows, int32_t n_levels, const float* q, int32_t dim, float* out) {
    std::vector<float> cur(q, q + dim);
    const int steps = std::min(n_layers, n_levels);
    for (int s = 0; s < steps; ++s) {
        const int64_t rows = level_rows[s];
        if (rows == 0) continue;
        const int64_t d = (int64_t)cur.size();
        const float* emb = levels[s];
        const int k = (int)std::min<int64_t>(5, rows);
        std::vector<int64_t> idx(k);
        std::vector<float> w(k);
        const int kk = orc_differentiable_search(cur.data(), emb, (int32_t)rows, d, k, 1.0f, idx.data(), w.data());
        std::vector<float> agg(d, 0.0f);
        for (int t = 0; t < kk; ++t)
            for (int64_t i = 0; i < d; ++i) agg[i] += w[t] * emb[idx[t] * d + i];
        std::vector<float> combined(d);
        for (int64_t i = 0; i < d; ++i) combined[i] = (cur[i] + agg[i]) / 2.0f;
        std::vector<float> nbrs((size_t)kk * d);
        for (int t = 0; t < kk; ++t) std::memcpy(&nbrs[(size_t)t * d], emb + idx[t] * d, d * 4);
        std::vector<float> y(layers[s]->H);
        orc_rvl_forward_one(layers[s], combined.data(), nbrs.data(), kk, w.data(), kk, y.data());
        cur.swap(y);
    }
    std::memcpy(out, cur.data(), cur.size() * 4);
    return (int32_t)cur.size();
}

// ============================================================ edge_featured.rs
// EdgeFeaturedAttention::new init (edge_featured.rs:98-141): fills the four
// arrays in creation order.
void orc_efa_init(int32_t node_dim, int32_t edge_dim, int32_t heads, float* w_node, float* w_edge, float* a_src,
                  float* a_dst, float* a_edge) {
    const int hd = node_dim / heads;
    const float node_scale = std::sqrt(2.0f / (float)(node_dim + hd));
    const float edge_scale = std::sqrt(2.0f / (float)(edge_dim + hd));
    const float attn_scale = std::sqrt(1.0f / (float)hd);
    uint64_t seed = 42;
    auto rnd = [&]() {
        seed = seed * 6364136223846793005ull + 1ull;
        return (float)seed / (float)UINT64_MAX - 0.5f;
    };
    for (int64_t i = 0; i < (int64_t)heads * hd * node_dim; ++i) w_node[i] = rnd() * 2.0f * node_scale;
    for (int64_t i = 0; i < (int64_t)heads * hd * edge_dim; ++i) w_edge[i] = rnd() * 2.0f * edge_scale;
    for (int64_t i = 0; i < (int64_t)heads * hd; ++i) a_src[i] = rnd() * 2.0f * attn_scale;
    for (int64_t i = 0; i < (int64_t)heads * hd; ++i) a_dst[i] = rnd() * 2.0f * attn_scale;
    for (int64_t i = 0; i < (int64_t)heads * hd; ++i) a_edge[i] = rnd() * 2.0f * attn_scale;
}

// stable_softmax (crates/ruvector-attention/src/utils.rs:11-54)
static void stable_softmax(std::vector<float>& v) {
    const int n = (int)v.size();
    if (n == 0) return;
    float mx = -INFINITY;
    for (float x : v) if (std::isfinite(x)) mx = std::fmax(mx, x);
    if (!std::isfinite(mx)) { for (auto& x : v) x = 1.0f / (float)n; return; }
    float sum = 0.0f;
    for (auto& x : v) { x = std::isfinite(x) ? std::exp(x - mx) : 0.0f; }
    for (float x : v) sum = sum + x;
    if (sum <= 1e-10f || !std::isfinite(sum)) { for (auto& x : v) x = 1.0f / (float)n; return; }
    const float inv = 1.0f / sum;
    for (auto& x : v) x = x * inv;
}

// ============================================================ dual_space.rs
// DualSpaceAttention::new (crates/ruvector-attention/src/graph/dual_space.rs:107-131):
// three dim x dim matrices [out][in] from one LCG stream (seed 42), Xavier scale.
void orc_dsa_init(int32_t dim, float* w_euc, float* w_hyp, float* w_out) {
    const float w_scale = std::sqrt(2.0f / (float)(dim + dim));
    uint64_t seed = 42;
    auto rnd = [&]() {
        seed = seed * 6364136223846793005ull + 1ull;
        return ((float)seed / (float)UINT64_MAX - 0.5f) * 2.0f * w_scale;
    };
    const int64_t nn = (int64_t)dim * dim;
    for (int64_t i = 0; i < nn; ++i) w_euc[i] = rnd();
    for (int64_t i = 0; i < nn; ++i) w_hyp[i] = rnd();
    for (int64_t i = 0; i < nn; ++i) w_out[i] = rnd();
}

// y_i = sum_j x_j * W[i*dim + j], sequential in j (to_euclidean / to_hyperbolic /
// project_output, dual_space.rs:134-183)
static std::vector<float> dsa_project(const float* x, const float* W, int dim) {
    std::vector<float> y(dim);
    for (int i = 0; i < dim; ++i) {
        float s = 0.0f;
        for (int j = 0; j < dim; ++j) s = s + x[j] * W[(int64_t)i * dim + j];
        y[i] = s;
    }
    return y;
}

// project_to_ball (crates/ruvector-attention/src/hyperbolic/poincare.rs:121-132), EPS 1e-7
static void dsa_project_to_ball(std::vector<float>& x, float c, float eps) {
    c = std::fabs(c);
    float ns = 0.0f;
    for (float v : x) ns = ns + v * v;
    const float norm_x = std::sqrt(ns);
    const float max_norm = (1.0f / std::sqrt(c)) - eps;
    if (norm_x < max_norm) return;
    const float scale = max_norm / std::fmax(norm_x, 1e-7f);
    for (auto& v : x) v = scale * v;
}

// poincare_dist (dual_space.rs:14-27)
static float dsa_poincare_dist(const std::vector<float>& u, const std::vector<float>& v, float curvature) {
    const float c = std::fabs(curvature);
    const float sqrt_c = std::sqrt(c);
    float diff_sq = 0.0f, nu = 0.0f, nv = 0.0f;
    for (size_t i = 0; i < u.size(); ++i) { const float d = u[i] - v[i]; diff_sq = diff_sq + d * d; }
    for (float a : u) nu = nu + a * a;
    for (float b : v) nv = nv + b * b;
    const float denom = std::fmax(1.0f - c * nu, 1e-7f) * std::fmax(1.0f - c * nv, 1e-7f);
    const float arg = 1.0f + 2.0f * c * diff_sq / denom;
    return (1.0f / sqrt_c) * std::acosh(std::fmax(arg, 1.0f));
}

// Attention::compute (dual_space.rs:207-268): n >= 1 keys (the reference errors on
// empty keys), values of value_dim; output projection only when value_dim == dim.
int32_t orc_dsa_compute(int32_t dim, float curvature, float euclidean_weight, float hyperbolic_weight,
                        float temperature, const float* w_euc, const float* w_hyp, const float* w_out,
                        const float* query, const float* keys, const float* values, int32_t n, int32_t value_dim,
                        float* out) {
    if (n <= 0) return -1;
    const float scale = 1.0f / std::sqrt((float)dim);
    const std::vector<float> q_euc = dsa_project(query, w_euc, dim);
    std::vector<float> q_hyp = dsa_project(query, w_hyp, dim);
    dsa_project_to_ball(q_hyp, curvature, 1e-5f);
    std::vector<float> scores(n);
    for (int i = 0; i < n; ++i) {
        const std::vector<float> k_euc = dsa_project(keys + (int64_t)i * dim, w_euc, dim);
        std::vector<float> k_hyp = dsa_project(keys + (int64_t)i * dim, w_hyp, dim);
        dsa_project_to_ball(k_hyp, curvature, 1e-5f);
        float dot = 0.0f;
        for (int t = 0; t < dim; ++t) dot = dot + q_euc[t] * k_euc[t];
        const float euc = dot * scale;
        const float hyp = -dsa_poincare_dist(q_hyp, k_hyp, curvature);
        scores[i] = (euclidean_weight * euc + hyperbolic_weight * hyp) / temperature;
    }
    stable_softmax(scores);
    std::vector<float> o(value_dim, 0.0f);
    for (int i = 0; i < n; ++i)
        for (int t = 0; t < value_dim; ++t) o[t] = o[t] + scores[i] * values[(int64_t)i * value_dim + t];
    if (value_dim == dim) {
        const std::vector<float> p = dsa_project(o.data(), w_out, dim);
        std::copy(p.begin(), p.end(), out);
    } else {
        std::copy(o.begin(), o.end(), out);
    }
    return value_dim;
}

// compute_with_edges (edge_featured.rs:196-258); edges nullable = zero
// features (Attention::compute, :267-288). Returns output length.
int32_t orc_efa_compute(int32_t node_dim, int32_t edge_dim, int32_t heads, int32_t concat, float slope,
                        const float* w_node, const float* w_edge, const float* a_src, const float* a_dst,
                        const float* a_edge, const float* query, const float* keys, const float* values,
                        const float* edges, int32_t n, float* out) {
    const int hd = node_dim / heads;
    auto tnode = [&](const float* x, int h) {  // transform_node (:144-156)
        std::vector<float> t(hd);
        for (int i = 0; i < hd; ++i) {
            float s = 0.0f;
            for (int j = 0; j < node_dim; ++j) s = s + x[j] * w_node[(int64_t)h * hd * node_dim + (int64_t)i * node_dim + j];
            t[i] = s;
        }
        return t;
    };
    auto tedge = [&](const float* e, int h) {  // transform_edge (:159-171)
        std::vector<float> t(hd);
        for (int i = 0; i < hd; ++i) {
            float s = 0.0f;
            for (int j = 0; j < edge_dim; ++j) s = s + e[j] * w_edge[(int64_t)h * hd * edge_dim + (int64_t)i * edge_dim + j];
            t[i] = s;
        }
        return t;
    };
    std::vector<float> zero_edge(std::max(edge_dim, 1), 0.0f);
    std::vector<std::vector<float>> heads_out;
    for (int h = 0; h < heads; ++h) {
        const std::vector<float> qt = tnode(query, h);
        std::vector<float> coeffs(n);
        for (int i = 0; i < n; ++i) {
            const std::vector<float> kt = tnode(keys + (int64_t)i * node_dim, h);
            const std::vector<float> et = tedge(edges ? edges + (int64_t)i * edge_dim : zero_edge.data(), h);
            float score = 0.0f;  // attention_coeff (:174-191)
            for (int c = 0; c < hd; ++c) {
                const int off = h * hd + c;
                score = score + qt[c] * a_src[off];
                score = score + kt[c] * a_dst[off];
                score = score + et[c] * a_edge[off];
            }
            coeffs[i] = score < 0.0f ? slope * score : score;
        }
        stable_softmax(coeffs);
        std::vector<float> ho(hd, 0.0f);
        for (int i = 0; i < n; ++i) {
            const std::vector<float> vt = tnode(values + (int64_t)i * node_dim, h);
            for (int c = 0; c < hd; ++c) ho[c] = ho[c] + coeffs[i] * vt[c];
        }
        heads_out.push_back(ho);
    }
    if (concat) {
        int p = 0;
        for (auto& ho : heads_out) for (float v : ho) out[p++] = v;
        return p;
    }
    for (int c = 0; c < hd; ++c) out[c] = 0.0f;
    for (auto& ho : heads_out)
        for (int c = 0; c < hd; ++c) out[c] = out[c] + ho[c] / (float)heads;
    return hd;
}

// ============================================================ poincare.rs
// fused_norms (:135-168) + poincare_distance_from_norms (:238-255) + fast_acosh (:259-276)
float orc_poincare_distance(const float* u, const float* v, int64_t d, float c) {
    c = std::fmax(std::fabs(c), 1e-5f);
    float ds = 0.0f, nu = 0.0f, nv = 0.0f;
    int64_t i = 0;
    for (int64_t ch = 0; ch < d / 4; ++ch, i += 4) {
        const float d0 = u[i] - v[i], d1 = u[i + 1] - v[i + 1], d2 = u[i + 2] - v[i + 2], d3 = u[i + 3] - v[i + 3];
        ds = ds + (d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3);
        nu = nu + (u[i] * u[i] + u[i + 1] * u[i + 1] + u[i + 2] * u[i + 2] + u[i + 3] * u[i + 3]);
        nv = nv + (v[i] * v[i] + v[i + 1] * v[i + 1] + v[i + 2] * v[i + 2] + v[i + 3] * v[i + 3]);
    }
    for (; i < d; ++i) {
        const float di = u[i] - v[i];
        ds = ds + di * di;
        nu = nu + u[i] * u[i];
        nv = nv + v[i] * v[i];
    }
    const float sqrt_c = std::sqrt(c);
    const float lu = std::fmax(1.0f - c * nu, 1e-5f);
    const float lv = std::fmax(1.0f - c * nv, 1e-5f);
    const float num = 2.0f * c * ds;
    const float den = lu * lv;
    const float arg = 1.0f + num / den;
    if (arg <= 1.0f) return 0.0f;
    float ac;
    const float delta = arg - 1.0f;
    if (delta < 1e-4f) ac = std::sqrt(2.0f * delta);
    else if (arg < 1e6f) ac = std::log(arg + std::sqrt(arg * arg - 1.0f));
    else ac = std::log(2.0f * arg);
    return (1.0f / sqrt_c) * ac;
}

}  // extern "C"
