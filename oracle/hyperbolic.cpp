// hyperbolic.cpp — CPU restatement of ruvector-hyperbolic-hnsw's HyperbolicHnsw.
//
// TEST INFRASTRUCTURE ONLY (see oracle.cpp): the checker for the GPU
// hyperbolic path, never linked into ruvector_amd/.
//
// Follows crates/ruvector-hyperbolic-hnsw/src/ line by line:
//   poincare.rs   norm_squared :77-103, fused_norms :135-168, project_to_ball :173-203,
//                 poincare_distance_from_norms :238-255, fast_acosh :259-276,
//                 mobius_add :310-356, exp_map :407-428, log_map :431-451,
//                 frechet_mean :463-538 (PoincareConfig defaults :40-50)
//   hnsw.rs       distance :175-207, random_level :220-224, insert :226-293,
//                 search_layer_single :304-327, search_layer :329-402,
//                 prune_connections :404-425, search :427-448,
//                 search_with_pruning :450-489, build_tangent_cache :492-503
//   libm          f32::ln -> glibc logf, f32::tanh -> glibc tanhf, f32::atanh -> Rust
//                 std's 0.5 * ln_1p(2x / (1 - x)) over glibc log1pf (rust_atanh)
//   tangent.rs    TangentCache::new :47-73, tangent_distance_squared :109-119
// Deviations (documented, test-visible only through exact ties):
//   * rand::random levels -> a seeded counter stream (same formula as the GPU
//     index, so both build from identical levels);
//   * BinaryHeap ties (unordered in the reference) ordered by node id.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <queue>
#include <thread>
#include <unordered_set>
#include <vector>

namespace {

constexpr float EPS = 1e-5f;

uint64_t hsm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

float norm_squared(const float* x, int d) {
    float sum = 0.0f;
    int i = 0;
    for (int ch = 0; ch < d / 4; ++ch, i += 4) {
        const float a = x[i], b = x[i + 1], c = x[i + 2], e = x[i + 3];
        sum += a * a + b * b + c * c + e * e;
    }
    for (; i < d; ++i) sum += x[i] * x[i];
    return sum;
}

void fused_norms(const float* u, const float* v, int d, float& diff_sq, float& nu, float& nv) {
    diff_sq = 0.0f; nu = 0.0f; nv = 0.0f;
    int i = 0;
    for (int ch = 0; ch < d / 4; ++ch, i += 4) {
        const float u0 = u[i], u1 = u[i + 1], u2 = u[i + 2], u3 = u[i + 3];
        const float v0 = v[i], v1 = v[i + 1], v2 = v[i + 2], v3 = v[i + 3];
        const float d0 = u0 - v0, d1 = u1 - v1, d2 = u2 - v2, d3 = u3 - v3;
        diff_sq += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
        nu += u0 * u0 + u1 * u1 + u2 * u2 + u3 * u3;
        nv += v0 * v0 + v1 * v1 + v2 * v2 + v3 * v3;
    }
    for (; i < d; ++i) {
        const float di = u[i] - v[i];
        diff_sq += di * di;
        nu += u[i] * u[i];
        nv += v[i] * v[i];
    }
}

// Rust std's f32::atanh (library/std/src/f32.rs): 0.5 * ((2x) / (1 - x)).ln_1p(), with
// ln_1p = libm log1pf — not libm atanhf, which rounds differently.
float rust_atanh(float x) { return 0.5f * std::log1p((2.0f * x) / (1.0f - x)); }

float fast_acosh(float x) {
    if (x <= 1.0f) return 0.0f;
    const float delta = x - 1.0f;
    if (delta < 1e-4f) return std::sqrt(2.0f * delta);
    if (x < 1e6f) return std::log(x + std::sqrt(x * x - 1.0f));
    return std::log(2.0f * x);
}

float from_norms(float diff_sq, float nu, float nv, float c) {
    const float sqrt_c = std::sqrt(c);
    const float lu = std::max(1.0f - c * nu, EPS);
    const float lv = std::max(1.0f - c * nv, EPS);
    const float numerator = 2.0f * c * diff_sq;
    const float denominator = lu * lv;
    const float arg = 1.0f + numerator / denominator;
    if (arg <= 1.0f) return 0.0f;
    return (1.0f / sqrt_c) * fast_acosh(arg);
}

void project_inplace(std::vector<float>& x, float c, float eps) {
    c = std::max(std::fabs(c), EPS);
    const float ns = norm_squared(x.data(), (int)x.size());
    const float max_norm = (1.0f / std::sqrt(c)) - eps;
    if (ns >= max_norm * max_norm && ns >= eps * eps) {
        const float scale = max_norm / std::sqrt(ns);
        for (float& xi : x) xi *= scale;
    }
}

std::vector<float> mobius_add(const float* x, const float* y, int d, float c) {
    c = std::max(std::fabs(c), EPS);
    float nx = 0.0f, ny = 0.0f, dxy = 0.0f;
    int i = 0;
    for (int ch = 0; ch < d / 4; ++ch, i += 4) {
        nx += x[i] * x[i] + x[i + 1] * x[i + 1] + x[i + 2] * x[i + 2] + x[i + 3] * x[i + 3];
        ny += y[i] * y[i] + y[i + 1] * y[i + 1] + y[i + 2] * y[i + 2] + y[i + 3] * y[i + 3];
        dxy += x[i] * y[i] + x[i + 1] * y[i + 1] + x[i + 2] * y[i + 2] + x[i + 3] * y[i + 3];
    }
    for (; i < d; ++i) {
        nx += x[i] * x[i];
        ny += y[i] * y[i];
        dxy += x[i] * y[i];
    }
    const float coef_x = 1.0f + 2.0f * c * dxy + c * ny;
    const float coef_y = 1.0f - c * nx;
    const float denom = std::max(1.0f + 2.0f * c * dxy + c * c * nx * ny, EPS);
    const float inv_denom = 1.0f / denom;
    std::vector<float> r(d);
    for (int j = 0; j < d; ++j) r[j] = (coef_x * x[j] + coef_y * y[j]) * inv_denom;
    project_inplace(r, c, EPS);
    return r;
}

std::vector<float> log_map(const float* y, const float* p, int d, float c) {
    c = std::max(std::fabs(c), EPS);
    const float sqrt_c = std::sqrt(c);
    std::vector<float> neg_p(d);
    for (int i = 0; i < d; ++i) neg_p[i] = -p[i];
    std::vector<float> diff = mobius_add(neg_p.data(), y, d, c);
    const float norm_diff = std::sqrt(norm_squared(diff.data(), d));
    if (norm_diff < EPS) return std::vector<float>(d, 0.0f);
    const float lambda_p = 2.0f / std::max(1.0f - c * norm_squared(p, d), EPS);
    const float arg = std::min(sqrt_c * norm_diff, 1.0f - EPS);
    const float coef = (2.0f / (sqrt_c * lambda_p)) * rust_atanh(arg) / norm_diff;
    for (float& v : diff) v = coef * v;
    return diff;
}

std::vector<float> exp_map(const float* v, const float* p, int d, float c) {
    c = std::max(std::fabs(c), EPS);
    const float sqrt_c = std::sqrt(c);
    const float lambda_p = 2.0f / std::max(1.0f - c * norm_squared(p, d), EPS);
    const float norm_v = std::sqrt(norm_squared(v, d));
    if (norm_v < EPS) return std::vector<float>(p, p + d);
    const float scaled_norm = sqrt_c * lambda_p * norm_v / 2.0f;
    const float coef = std::tanh(scaled_norm) / (sqrt_c * norm_v);
    std::vector<float> t(d);
    for (int i = 0; i < d; ++i) t[i] = coef * v[i];
    return mobius_add(p, t.data(), d, c);
}

struct R {
    float d;
    int64_t id;
};
struct RMax {  // max-heap by (d, id)
    bool operator()(const R& a, const R& b) const { return a.d < b.d || (a.d == b.d && a.id < b.id); }
};
struct RMin {
    bool operator()(const R& a, const R& b) const { return a.d > b.d || (a.d == b.d && a.id > b.id); }
};
bool r_less(const R& a, const R& b) { return a.d < b.d || (a.d == b.d && a.id < b.id); }

struct OHyp {
    int d = 0, M = 16, M0 = 32, efc = 200, efs = 50, pf = 10;
    float lm = 0.0f, c = 1.0f;
    uint64_t seed = 0;
    std::vector<float> data;                    // projected vectors
    std::vector<int> level;
    std::vector<std::vector<std::vector<int64_t>>> conn;  // conn[p][l]
    int64_t entry = -1;
    int max_level = 0;
    bool has_cache = false;
    bool euclid = false;                        // DistanceMetric::Euclidean (hnsw.rs:182-185)
    std::vector<float> centroid, tangent;       // tangent [n][d]

    const float* v(int64_t i) const { return data.data() + i * d; }
    float dist(const float* a, const float* b) const {
        float ds, na, nb;
        fused_norms(a, b, d, ds, na, nb);
        return euclid ? std::sqrt(ds) : from_norms(ds, na, nb, c);
    }
};

int random_level(const OHyp& h, int64_t i) {
    const float r = (float)((hsm64(hsm64(h.seed) + (uint64_t)i) >> 40) + 1) * (1.0f / 16777216.0f);
    const float lev = -std::log(r) * h.lm;
    return (int)std::min<float>(std::floor(lev), 15.0f);
}

int64_t search_layer_single(const OHyp& h, const float* q, int64_t entry, int l) {
    int64_t current = entry;
    float current_dist = h.dist(q, h.v(current));
    for (;;) {
        bool changed = false;
        const std::vector<int64_t> lst = h.conn[current][l];
        for (int64_t nb : lst) {
            const float dd = h.dist(q, h.v(nb));
            if (dd < current_dist) {
                current_dist = dd;
                current = nb;
                changed = true;
            }
        }
        if (!changed) break;
    }
    return current;
}

// lex_stop (the query path): the stop test compares (d, id) pairs, as the GPU
// search does (oracle.cpp search_layer); differs only on exact distance ties.
std::vector<R> search_layer(const OHyp& h, const float* q, int64_t entry, int ef, int l, bool lex_stop = false) {
    const float ed = h.dist(q, h.v(entry));
    std::unordered_set<int64_t> visited{entry};
    std::priority_queue<R, std::vector<R>, RMin> cand;
    std::priority_queue<R, std::vector<R>, RMax> res;
    cand.push({ed, entry});
    res.push({ed, entry});
    while (!cand.empty()) {
        const R cur = cand.top();
        cand.pop();
        const R& f = res.top();
        if ((cur.d > f.d || (lex_stop && cur.d == f.d && cur.id > f.id)) && (int)res.size() >= ef) break;
        for (int64_t nb : h.conn[cur.id][l]) {
            if (!visited.insert(nb).second) continue;
            const float dd = h.dist(q, h.v(nb));
            if ((int)res.size() < ef || dd < res.top().d) {
                cand.push({dd, nb});
                res.push({dd, nb});
                if ((int)res.size() > ef) res.pop();
            }
        }
    }
    std::vector<R> out;
    while (!res.empty()) { out.push_back(res.top()); res.pop(); }
    std::sort(out.begin(), out.end(), r_less);
    return out;
}

void prune_connections(OHyp& h, int64_t node, int l, int max_conn) {
    std::vector<R> scored;
    for (int64_t id : h.conn[node][l]) scored.push_back({h.dist(h.v(node), h.v(id)), id});
    std::stable_sort(scored.begin(), scored.end(), [](const R& a, const R& b) { return a.d < b.d; });
    h.conn[node][l].clear();
    for (int i = 0; i < (int)scored.size() && i < max_conn; ++i) h.conn[node][l].push_back(scored[i].id);
}

void insert_one(OHyp& h, const float* vec) {
    std::vector<float> x(vec, vec + h.d);
    project_inplace(x, h.c, EPS);
    const int64_t id = (int64_t)h.level.size();
    const int level = random_level(h, id);
    h.data.insert(h.data.end(), x.begin(), x.end());
    h.level.push_back(level);
    h.conn.emplace_back(level + 1);
    if (h.entry < 0) {
        h.entry = id;
        h.max_level = level;
        return;
    }
    int64_t current = h.entry;
    for (int l = h.max_level; l >= level + 1; --l) current = search_layer_single(h, x.data(), current, l);
    const int insert_level = std::min(level, h.max_level);
    for (int l = insert_level; l >= 0; --l) {
        const std::vector<R> nbs = search_layer(h, x.data(), current, h.efc, l);
        const int max_conn = l == 0 ? h.M0 : h.M;
        std::vector<int64_t> selected;
        for (int i = 0; i < (int)nbs.size() && i < max_conn; ++i) selected.push_back(nbs[i].id);
        h.conn[id][l] = selected;
        for (int64_t nb : selected) {
            h.conn[nb][l].push_back(id);
            if ((int)h.conn[nb][l].size() > max_conn) prune_connections(h, nb, l, max_conn);
        }
        if (!nbs.empty()) current = nbs[0].id;
    }
    if (level > h.max_level) {
        h.entry = id;
        h.max_level = level;
    }
    h.has_cache = false;
}

void pfor(int64_t n, int threads, const std::function<void(int64_t)>& f) {
    if (threads <= 1 || n < 2) {
        for (int64_t i = 0; i < n; ++i) f(i);
        return;
    }
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t)
        ts.emplace_back([&, t] {
            for (int64_t i = t; i < n; i += threads) f(i);
        });
    for (auto& t : ts) t.join();
}

}  // namespace

extern "C" {

void* orc_hyp_new(int32_t d, int32_t M, int32_t M0, int32_t efc, int32_t efs, float level_mult, float c, int32_t pf,
                  uint64_t seed) {
    auto* h = new OHyp();
    h->d = d; h->M = M; h->M0 = M0; h->efc = efc; h->efs = efs; h->lm = level_mult; h->c = c; h->pf = pf;
    h->seed = seed;
    return h;
}
void orc_hyp_free(void* hp) { delete static_cast<OHyp*>(hp); }
// HyperbolicHnswConfig.metric: 0 Poincaré, 1 Euclidean (hnsw.rs:21-31, 175-185)
void orc_hyp_set_metric(void* hp, int32_t euclid) { static_cast<OHyp*>(hp)->euclid = euclid != 0; }
int64_t orc_hyp_len(void* hp) { return (int64_t)static_cast<OHyp*>(hp)->level.size(); }

void orc_hyp_insert(void* hp, const float* vecs, int64_t n) {
    OHyp& h = *static_cast<OHyp*>(hp);
    for (int64_t i = 0; i < n; ++i) insert_one(h, vecs + i * h.d);
}

void orc_hyp_get_vector(void* hp, int64_t id, float* out) {
    const OHyp& h = *static_cast<OHyp*>(hp);
    std::memcpy(out, h.v(id), sizeof(float) * h.d);
}

// search (hnsw.rs:427-448); ef_arg 0 -> ef_search. ids -1 past the end.
void orc_hyp_search(void* hp, const float* q, int64_t nq, int32_t k, int32_t ef_arg, int64_t* ids, float* dist,
                    int32_t* counts, int32_t threads) {
    const OHyp& h = *static_cast<OHyp*>(hp);
    pfor(nq, threads, [&](int64_t qi) {
        int64_t* oi = ids + qi * k;
        float* od = dist + qi * k;
        for (int s = 0; s < k; ++s) { oi[s] = -1; od[s] = INFINITY; }
        if (h.entry < 0) { if (counts) counts[qi] = 0; return; }
        std::vector<float> x(q + qi * h.d, q + (qi + 1) * h.d);
        project_inplace(x, h.c, EPS);
        int64_t current = h.entry;
        for (int l = h.max_level; l >= 1; --l) current = search_layer_single(h, x.data(), current, l);
        const int ef = std::max(ef_arg > 0 ? ef_arg : h.efs, k);
        std::vector<R> r = search_layer(h, x.data(), current, ef, 0, /*lex_stop=*/true);
        const int take = std::min<int>(k, (int)r.size());
        for (int s = 0; s < take; ++s) { oi[s] = r[s].id; od[s] = r[s].d; }
        if (counts) counts[qi] = take;
    });
}

// exact scan by distance (ground truth), ties by id
void orc_hyp_brute_force(void* hp, const float* q, int64_t nq, int32_t k, int64_t* ids, float* dist, int32_t threads) {
    const OHyp& h = *static_cast<OHyp*>(hp);
    const int64_t n = (int64_t)h.level.size();
    pfor(nq, threads, [&](int64_t qi) {
        std::vector<float> x(q + qi * h.d, q + (qi + 1) * h.d);
        project_inplace(x, h.c, EPS);
        std::vector<R> all((size_t)n);
        for (int64_t i = 0; i < n; ++i) all[(size_t)i] = {h.dist(x.data(), h.v(i)), i};
        const int take = (int)std::min<int64_t>(k, n);
        std::partial_sort(all.begin(), all.begin() + take, all.end(), r_less);
        for (int s = 0; s < k; ++s) {
            ids[qi * k + s] = s < take ? all[(size_t)s].id : -1;
            dist[qi * k + s] = s < take ? all[(size_t)s].d : INFINITY;
        }
    });
}

// Exact scan of raw rows for a bench's spot check at scale: merges the (distance, id)
// top-k of rows x[0..n) (ids id_base + i) into ids_io / dist_io, which hold k ascending
// entries per query (-1 / inf when empty). Called once per row chunk, so a caller can
// stream a large shard through host memory. Rows must already lie in the ball (the
// projection is the identity then); queries are projected as in orc_hyp_brute_force.
void orc_hyp_scan_rows(const float* x, int64_t n, int32_t d, float c, const float* q, int64_t nq, int32_t k,
                       int64_t id_base, int64_t* ids_io, float* dist_io, int32_t threads) {
    OHyp h;
    h.d = d;
    h.c = c;
    pfor(nq, threads, [&](int64_t qi) {
        std::vector<float> xq(q + qi * d, q + (qi + 1) * d);
        project_inplace(xq, c, EPS);
        std::vector<R> all;
        all.reserve((size_t)(n + k));
        for (int s = 0; s < k; ++s)
            if (ids_io[qi * k + s] >= 0) all.push_back({dist_io[qi * k + s], ids_io[qi * k + s]});
        for (int64_t i = 0; i < n; ++i) all.push_back({h.dist(xq.data(), x + i * d), id_base + i});
        const int take = (int)std::min<int64_t>(k, (int64_t)all.size());
        std::partial_sort(all.begin(), all.begin() + take, all.end(), r_less);
        for (int s = 0; s < k; ++s) {
            ids_io[qi * k + s] = s < take ? all[(size_t)s].id : -1;
            dist_io[qi * k + s] = s < take ? all[(size_t)s].d : INFINITY;
        }
    });
}

// build_tangent_cache (hnsw.rs:492-503) -> TangentCache::new (tangent.rs:47-73)
// -> frechet_mean (poincare.rs:463-538), PoincareConfig defaults.
void orc_hyp_build_tangent(void* hp) {
    OHyp& h = *static_cast<OHyp*>(hp);
    const int64_t n = (int64_t)h.level.size();
    if (n == 0) return;
    const int d = h.d;
    const float c = h.c;
    const float w = 1.0f / (float)n;
    std::vector<float> mean(d, 0.0f);
    for (int64_t p = 0; p < n; ++p)
        for (int i = 0; i < d; ++i) mean[i] += w * h.v(p)[i];
    project_inplace(mean, c, EPS);
    std::vector<float> grad(d);
    for (int it = 0; it < 100; ++it) {
        std::fill(grad.begin(), grad.end(), 0.0f);
        for (int64_t p = 0; p < n; ++p) {
            const std::vector<float> lr = log_map(h.v(p), mean.data(), d, c);
            for (int i = 0; i < d; ++i) grad[i] += w * lr[i];
        }
        if (std::sqrt(norm_squared(grad.data(), d)) < 1e-6f) break;
        std::vector<float> update(d);
        for (int i = 0; i < d; ++i) update[i] = 0.1f * grad[i];
        mean = exp_map(update.data(), mean.data(), d, c);
    }
    h.centroid = mean;
    h.tangent.assign((size_t)n * d, 0.0f);
    for (int64_t p = 0; p < n; ++p) {
        const std::vector<float> t = log_map(h.v(p), mean.data(), d, c);
        std::copy(t.begin(), t.end(), h.tangent.begin() + p * d);
    }
    h.has_cache = true;
}

void orc_hyp_centroid(void* hp, float* out) {
    const OHyp& h = *static_cast<OHyp*>(hp);
    std::copy(h.centroid.begin(), h.centroid.end(), out);
}

// search_with_pruning (hnsw.rs:450-489)
void orc_hyp_search_pruning(void* hp, const float* q, int64_t nq, int32_t k, int64_t* ids, float* dist, int32_t threads) {
    const OHyp& h = *static_cast<OHyp*>(hp);
    if (!h.has_cache) {
        orc_hyp_search(hp, q, nq, k, 0, ids, dist, nullptr, threads);
        return;
    }
    const int64_t n = (int64_t)h.level.size();
    const int d = h.d;
    pfor(nq, threads, [&](int64_t qi) {
        std::vector<float> x(q + qi * d, q + (qi + 1) * d);
        project_inplace(x, h.c, EPS);
        const std::vector<float> qt = log_map(x.data(), h.centroid.data(), d, h.c);
        std::vector<R> cands((size_t)n);
        for (int64_t i = 0; i < n; ++i) {
            const float* p = h.tangent.data() + i * d;
            float s = 0.0f;
            for (int j = 0; j < d; ++j) s += (qt[j] - p[j]) * (qt[j] - p[j]);
            cands[(size_t)i] = {s, i};
        }
        std::stable_sort(cands.begin(), cands.end(), [](const R& a, const R& b) { return a.d < b.d; });
        const int64_t nc = std::min<int64_t>((int64_t)k * h.pf, n);
        std::vector<R> res;
        for (int64_t i = 0; i < nc; ++i) res.push_back({h.dist(x.data(), h.v(cands[(size_t)i].id)), cands[(size_t)i].id});
        std::stable_sort(res.begin(), res.end(), [](const R& a, const R& b) { return a.d < b.d; });
        for (int s = 0; s < k; ++s) {
            ids[qi * k + s] = s < (int)res.size() ? res[(size_t)s].id : -1;
            dist[qi * k + s] = s < (int)res.size() ? res[(size_t)s].d : INFINITY;
        }
    });
}

// set_curvature (hnsw.rs:511-530)
void orc_hyp_set_curvature(void* hp, float c) {
    OHyp& h = *static_cast<OHyp*>(hp);
    h.c = c;
    const int64_t n = (int64_t)h.level.size();
    for (int64_t p = 0; p < n; ++p) {
        std::vector<float> x(h.v(p), h.v(p) + h.d);
        project_inplace(x, c, EPS);
        std::copy(x.begin(), x.end(), h.data.begin() + p * h.d);
    }
    if (h.has_cache) orc_hyp_build_tangent(hp);
}

// Graph in the rvx_hnsw_graph layout: layer l lists every node of level >= l.
void orc_hyp_export_sizes(void* hp, int64_t* n, int32_t* max_level, int64_t* entry, int64_t* e0,
                          int64_t* upper_count /*[17]*/, int64_t* upper_edges /*[17]*/) {
    const OHyp& h = *static_cast<OHyp*>(hp);
    const int64_t N = (int64_t)h.level.size();
    *n = N;
    *max_level = h.max_level;
    *entry = h.entry;
    int64_t e = 0;
    for (int64_t i = 0; i < N; ++i) e += (int64_t)h.conn[i][0].size();
    *e0 = e;
    for (int l = 0; l <= 16; ++l) { upper_count[l] = 0; upper_edges[l] = 0; }
    for (int l = 1; l <= h.max_level; ++l)
        for (int64_t i = 0; i < N; ++i)
            if (h.level[i] >= l) { upper_count[l]++; upper_edges[l] += (int64_t)h.conn[i][l].size(); }
}

void orc_hyp_export(void* hp, uint8_t* levels, int64_t* rp0, int32_t* col0, int32_t* up_ids, int64_t* up_rp,
                    int32_t* up_col) {
    const OHyp& h = *static_cast<OHyp*>(hp);
    const int64_t N = (int64_t)h.level.size();
    for (int64_t i = 0; i < N; ++i) levels[i] = (uint8_t)h.level[i];
    int64_t e = 0;
    rp0[0] = 0;
    for (int64_t i = 0; i < N; ++i) {
        for (int64_t c : h.conn[i][0]) col0[e++] = (int32_t)c;
        rp0[i + 1] = e;
    }
    int64_t oi = 0, orp = 0, oc = 0;
    for (int l = 1; l <= h.max_level; ++l) {
        int64_t local = 0;
        up_rp[orp++] = 0;
        for (int64_t i = 0; i < N; ++i) {
            if (h.level[i] < l) continue;
            up_ids[oi++] = (int32_t)i;
            for (int64_t c : h.conn[i][l]) { up_col[oc++] = (int32_t)c; ++local; }
            up_rp[orp++] = local;
        }
    }
}

// A searchable handle over given (already projected) vectors and graph.
void* orc_hyp_from_graph(const float* vecs, int64_t n, int32_t d, int32_t M, int32_t M0, int32_t efs, float c,
                         int32_t pf, const uint8_t* levels, int64_t entry, int32_t max_level, const int64_t* rp0,
                         const int32_t* col0, const int64_t* upper_count, const int32_t* up_ids, const int64_t* up_rp,
                         const int32_t* up_col) {
    auto* h = new OHyp();
    h->d = d; h->M = M; h->M0 = M0; h->efs = efs; h->c = c; h->pf = pf;
    h->data.assign(vecs, vecs + n * d);
    h->level.assign(levels, levels + n);
    h->conn.resize(n);
    for (int64_t i = 0; i < n; ++i) {
        h->conn[i].resize(levels[i] + 1);
        for (int64_t p = rp0[i]; p < rp0[i + 1]; ++p) h->conn[i][0].push_back(col0[p]);
    }
    int64_t oi = 0, orp = 0, oc = 0;
    for (int l = 1; l <= max_level; ++l) {
        const int64_t cnt = upper_count[l];
        for (int64_t j = 0; j < cnt; ++j) {
            const int64_t p = up_ids[oi + j];
            if ((int)h->conn[p].size() <= l) h->conn[p].resize(l + 1);
            for (int64_t t = up_rp[orp + j]; t < up_rp[orp + j + 1]; ++t) h->conn[p][l].push_back(up_col[oc + t]);
        }
        oc += up_rp[orp + cnt];
        oi += cnt;
        orp += cnt + 1;
    }
    h->entry = n > 0 ? entry : -1;
    h->max_level = max_level;
    return h;
}

}  // extern "C"
