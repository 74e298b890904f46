// api_hyper.cpp — HyperbolicHnsw over HBM (crates/ruvector-hyperbolic-hnsw/src/hnsw.rs:127-504,
// tangent.rs, poincare.rs). The graph lives in an rvx_index in hyperbolic mode:
// the GPU builder and search kernels with the Poincaré metric and the
// reference's insert/search rules (k_hnsw_build.hip / k_hnsw.hip, hyper = 1).
#include <cmath>
#include <shared_mutex>

#include "comm.hpp"
#include "graph.hpp"
#include "hnsw.hpp"
#include "hyper.hpp"
#include "index.hpp"
#include "kernels.hpp"
#include "poincare_dev.hpp"
#include "scan.hpp"

using namespace rvx;

struct rvx_hyperbolic {
    rvx_hyperbolic_config cfg{};
    rvx_index ix;
};

namespace {

void invalidate_tangent(rvx_hyperbolic* h) { h->ix.tan_valid = false; }

// HyperbolicHnsw::insert_batch (hnsw.rs:254-261): ids are insertion order
void insert_rows(rvx_hyperbolic* h, const float* rows, int64_t n, bool on_device, int64_t* first_id) {
    rvx_index* ix = &h->ix;
    const int64_t n0 = ix->n;
    if (first_id) *first_id = n0;
    if (n <= 0) return;
    std::vector<uint64_t> ids((size_t)n);
    for (int64_t i = 0; i < n; ++i) ids[(size_t)i] = (uint64_t)(n0 + i);
    index_append_rows(ix, rows, ids.data(), n, on_device);
    // project_to_ball(&vector, curvature, EPS) before storing (hnsw.rs:195)
    project_rows(ix->vecs.as<float>() + n0 * ix->cfg.dim, n, ix->cfg.dim, ix->curv);
    hnsw_insert_range(ix, n0, n);
    invalidate_tangent(h);
}

// queries projected into the ball (search / search_with_pruning, hnsw.rs:431, :458)
float* projected_queries(const rvx_hyperbolic* h, const float* q, int64_t nq, bool on_device) {
    const int d = h->ix.cfg.dim;
    float* dq = scratch_f32("hyp_q", nq * d);
    RVX_HIP(hipMemcpyAsync(dq, q, (size_t)(nq * d * 4), on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                           stream()));
    project_rows(dq, nq, d, h->ix.curv);
    return dq;
}

__global__ void k_rows_to_ids(const int64_t* rows, const float* dist, int64_t total, int64_t* ids, float* out_d) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int64_t r = rows[i];
    const bool ok = r >= 0 && r != INT64_MAX;
    ids[i] = ok ? r : -1;
    out_d[i] = ok ? dist[i] : INFINITY;
}

void finish_ids(const int64_t* rows, const float* dist, int64_t nq, int k, int64_t* ids, float* out_d) {
    const int64_t total = nq * k;
    if (total <= 0) return;
    hipLaunchKernelGGL(k_rows_to_ids, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream(), rows, dist, total,
                       ids, out_d);
    RVX_HIP(hipGetLastError());
}

__global__ void k_offset_ids(const int64_t* in, int64_t total, int64_t base, int64_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < total) out[i] = in[i] >= 0 ? in[i] + base : -1;
}

// local ids of a node-range shard -> global ids (shard.rs:360-363: local + the shard's first id)
void offset_ids(const int64_t* in, int64_t total, int64_t base, int64_t* out) {
    if (total <= 0) return;
    hipLaunchKernelGGL(k_offset_ids, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream(), in, total, base,
                       out);
    RVX_HIP(hipGetLastError());
}

// device search core; outputs on the device
void search_dev(const rvx_hyperbolic* h, const float* dq, int64_t nq, int k, int ef, int64_t* ids, float* dist,
                int32_t* counts, int mode /*0 graph, 1 exact, 2 pruned*/) {
    const rvx_index* ix = &h->ix;
    const int d = ix->cfg.dim;
    auto* rows = (int64_t*)scratch_bytes("hyp_rows", nq * k * 8);
    float* rd = scratch_f32("hyp_rd", nq * k);
    if (ix->n == 0) {
        RVX_HIP(hipMemsetAsync(rows, 0xFF, (size_t)(nq * k * 8), stream()));
        if (counts) RVX_HIP(hipMemsetAsync(counts, 0, (size_t)(nq * 4), stream()));
        finish_ids(rows, rd, nq, k, ids, dist);
        return;
    }
    if (mode == 1) {
        if (ix->cfg.metric == RVX_METRIC_POINCARE)
            poincare_topk(dq, nq, ix->vecs.as<float>(), ix->n, d, ix->curv, k, rd, rows);
        else  // DistanceMetric::Euclidean: the same tiled scan, sqrt of the chunked |q-x|^2
            scan_topk(RVX_METRIC_HYP_L2, dq, nullptr, nq, ix->vecs.as<float>(), nullptr, nullptr, ix->n, d, k, 0, rd,
                      rows, "hyp_brute_force");
        if (counts) {
            std::vector<int32_t> c((size_t)nq, (int32_t)std::min<int64_t>(k, ix->n));
            RVX_HIP(hipMemcpyAsync(counts, c.data(), (size_t)nq * 4, hipMemcpyHostToDevice, stream()));
            sync();
        }
    } else if (mode == 2) {
        // search_with_pruning (hnsw.rs:450-489): tangent-space L2 scan of every
        // point, keep k * prune_factor, exact Poincaré re-rank
        RVX_REQUIRE(ix->cfg.metric == RVX_METRIC_POINCARE, RVX_ERR_UNSUPPORTED,
                    "search_with_pruning is implemented for the Poincaré metric");
        const int64_t nc64 = std::min<int64_t>((int64_t)k * h->cfg.prune_factor, ix->n);
        RVX_REQUIRE(nc64 < ((int64_t)1 << 31), RVX_ERR_INVALID_PARAMETER, "k * prune_factor too large");
        const int nc = (int)nc64;
        float* qt = scratch_f32("hyp_qt", nq * d);
        std::vector<float> cen((size_t)d);
        ix->tan_centroid.download(cen.data(), (int64_t)d * 4);
        log_map_rows(dq, nq, d, ix->tan_norms.as<float>(), pdev::norm_sq(cen.data(), d), ix->curv, qt);
        float* cdist = scratch_f32("hyp_cand_d", nq * nc);
        auto* cand = (int64_t*)scratch_bytes("hyp_cand_i", nq * nc * 8);
        // tangent_distance_squared (tangent.rs:105-117): the sequential sum without a
        // square root, ranked (distance, id) as the reference's stable sort
        scan_topk(METRIC_L2SQ, qt, nullptr, nq, ix->tan_coords.as<float>(), nullptr, nullptr, ix->n, d, nc, 0, cdist,
                  cand, "hyp_tangent_scan");
        rerank(dq, nq, ix->vecs.as<float>(), d, ix->curv, cand, nc, k, rd, rows, counts);
    } else {
        index_search_rows(ix, dq, nq, k, ef, rd, rows, counts, false);
    }
    finish_ids(rows, rd, nq, k, ids, dist);
}

// TangentCache::new (tangent.rs:47-73): centroid = frechet_mean (poincare.rs:463-538,
// PoincareConfig defaults: max_iter 100, tol 1e-6, learning rate 0.1), then
// log_centroid of every point. The weighted sums run in the reference's point-major f32
// order (col_chain: one sequential chain per dimension, continued across row chunks) and
// the log / exp maps use the glibc transcendentals, so the centroid and every tangent
// coordinate equal the reference's bit for bit.
void build_tangent(rvx_hyperbolic* h) {
    rvx_index* ix = &h->ix;
    const int64_t n = ix->n;
    const int d = ix->cfg.dim;
    RVX_REQUIRE(n > 0, RVX_ERR_INVALID_PARAMETER, "empty collection");
    const float c = ix->curv;
    const float w = 1.0f / (float)n;
    const float* x = ix->vecs.as<float>();
    float* dacc = scratch_f32("hyp_fm_acc", d);
    std::vector<float> mean((size_t)d), grad((size_t)d), tmp((size_t)d), upd((size_t)d), negp((size_t)d);
    RVX_HIP(hipMemsetAsync(dacc, 0, (size_t)d * 4, stream()));
    col_chain(x, n, d, w, dacc);  // mean[i] += weight * val (poincare.rs:501-506)
    RVX_HIP(hipMemcpyAsync(mean.data(), dacc, (size_t)d * 4, hipMemcpyDeviceToHost, stream()));
    sync();
    pdev::project_inplace(mean.data(), d, c, pdev::EPS);
    const int64_t chunk = std::min<int64_t>(n, (int64_t)1 << 20);
    float* logs = scratch_f32("hyp_fm_logs", chunk * d);
    float* dnegp = scratch_f32("hyp_fm_negp", d);
    for (int it = 0; it < 100; ++it) {
        for (int i = 0; i < d; ++i) negp[(size_t)i] = -mean[(size_t)i];
        RVX_HIP(hipMemcpyAsync(dnegp, negp.data(), (size_t)d * 4, hipMemcpyHostToDevice, stream()));
        const float np_sq = pdev::norm_sq(mean.data(), d);
        RVX_HIP(hipMemsetAsync(dacc, 0, (size_t)d * 4, stream()));
        for (int64_t r0 = 0; r0 < n; r0 += chunk) {
            const int64_t rows = std::min(chunk, n - r0);
            log_map_rows(x + r0 * d, rows, d, dnegp, np_sq, c, logs);
            col_chain(logs, rows, d, w, dacc);  // grad[i] += weight * val (:519-525)
        }
        RVX_HIP(hipMemcpyAsync(grad.data(), dacc, (size_t)d * 4, hipMemcpyDeviceToHost, stream()));
        sync();
        if (std::sqrt(pdev::norm_sq(grad.data(), d)) < 1e-6f) break;
        for (int i = 0; i < d; ++i) upd[(size_t)i] = 0.1f * grad[(size_t)i];
        std::vector<float> next((size_t)d);
        pdev::exp_map(upd.data(), mean.data(), d, c, next.data(), tmp.data());
        mean.swap(next);
    }
    ix->tan_centroid.reset((int64_t)d * 4);
    ix->tan_centroid.upload(mean.data(), (int64_t)d * 4);
    for (int i = 0; i < d; ++i) negp[(size_t)i] = -mean[(size_t)i];
    ix->tan_norms.reset((int64_t)d * 4);  // holds -centroid for the query log maps
    ix->tan_norms.upload(negp.data(), (int64_t)d * 4);
    ix->tan_coords.reset(std::max<int64_t>(n * d, 1) * 4);
    log_map_rows(x, n, d, ix->tan_norms.as<float>(), pdev::norm_sq(mean.data(), d), c, ix->tan_coords.as<float>());
    sync();
    ix->tan_valid = true;
}

void check_cfg(const rvx_hyperbolic_config* c) {
    RVX_REQUIRE(c->dim > 0, RVX_ERR_INVALID_PARAMETER, "dimension must be positive");
    // the GPU builder's list capacities (k_hnsw_build.hip: MAX_C0 = 256 layer-0 slots)
    RVX_REQUIRE(c->max_connections >= 1 && c->max_connections <= 128 && c->max_connections_0 >= 1 &&
                    c->max_connections_0 <= 256,
                RVX_ERR_UNSUPPORTED, "max_connections must be in [1, 128] and max_connections_0 in [1, 256]");
    RVX_REQUIRE(c->ef_construction >= 1 && c->ef_construction <= HNSW_MAX_EF && c->ef_search >= 1,
                RVX_ERR_INVALID_PARAMETER, "ef out of range");
    RVX_REQUIRE(c->curvature > 0.0f, RVX_ERR_INVALID_PARAMETER, "invalid curvature (must be > 0)");
    RVX_REQUIRE(c->level_mult > 0.0f && c->prune_factor >= 1, RVX_ERR_INVALID_PARAMETER, "bad level_mult / prune_factor");
    RVX_REQUIRE(c->metric == RVX_METRIC_POINCARE || c->metric == RVX_METRIC_HYP_L2, RVX_ERR_UNSUPPORTED,
                "HyperbolicHnsw metric must be Poincare or Euclidean");
}

}  // namespace

extern "C" {

void rvx_hyperbolic_default_config(rvx_hyperbolic_config* c) {
    if (!c) return;
    c->dim = 0;
    c->max_connections = 16;
    c->max_connections_0 = 32;
    c->ef_construction = 200;
    c->ef_search = 50;
    c->level_mult = 1.0f / std::log(16.0f);
    c->curvature = 1.0f;
    c->prune_factor = 10;
    c->seed = 0;
    c->metric = RVX_METRIC_POINCARE;
}

rvx_status rvx_hyperbolic_create(const rvx_hyperbolic_config* cfg, rvx_hyperbolic** out) {
    return guard([&] {
        RVX_REQUIRE(cfg && out, RVX_ERR_INVALID_PARAMETER, "null argument");
        check_cfg(cfg);
        auto h = std::make_unique<rvx_hyperbolic>();
        h->cfg = *cfg;
        rvx_index& ix = h->ix;
        ix.cfg.kind = RVX_INDEX_HNSW;
        ix.cfg.dim = cfg->dim;
        ix.cfg.metric = cfg->metric;  // Poincaré or DistanceMetric::Euclidean (hnsw.rs:173-185)
        ix.cfg.m = cfg->max_connections;
        ix.cfg.ef_construction = cfg->ef_construction;
        ix.cfg.ef_search = cfg->ef_search;
        ix.cfg.seed = cfg->seed;
        ix.cfg.curvature = cfg->curvature;
        ix.hyper = true;
        ix.m0 = cfg->max_connections_0;
        ix.level_mult = cfg->level_mult;
        ix.curv = cfg->curvature;
        *out = h.release();
    });
}

rvx_status rvx_hyperbolic_destroy(rvx_hyperbolic* h) {
    return guard([&] { delete h; });
}

rvx_status rvx_hyperbolic_index(rvx_hyperbolic* h, rvx_index** out) {
    return guard([&] {
        RVX_REQUIRE(h && out, RVX_ERR_INVALID_PARAMETER, "null argument");
        *out = &h->ix;
    });
}

rvx_status rvx_hyperbolic_insert_batch(rvx_hyperbolic* h, const float* vecs, int64_t n, int64_t* first_id) {
    return guard([&] {
        RVX_REQUIRE(h && n >= 0 && (n == 0 || vecs), RVX_ERR_INVALID_PARAMETER, "bad arguments");
        std::unique_lock<std::shared_mutex> lk(h->ix.mu);
        ComputeLock cl;
        insert_rows(h, vecs, n, false, first_id);
    });
}

rvx_status rvx_hyperbolic_insert_batch_device(rvx_hyperbolic* h, const rvx_buffer* vecs, int64_t n, int64_t* first_id) {
    return guard([&] {
        RVX_REQUIRE(h && vecs && n >= 0, RVX_ERR_INVALID_PARAMETER, "bad arguments");
        RVX_REQUIRE(vecs->mem.bytes >= n * h->cfg.dim * 4, RVX_ERR_DIMENSION_MISMATCH, "buffer smaller than n*dim");
        std::unique_lock<std::shared_mutex> lk(h->ix.mu);
        ComputeLock cl;
        insert_rows(h, vecs->mem.as<float>(), n, true, first_id);
    });
}

rvx_status rvx_hyperbolic_len(const rvx_hyperbolic* h, int64_t* len) {
    return guard([&] {
        RVX_REQUIRE(h && len, RVX_ERR_INVALID_PARAMETER, "null argument");
        *len = h->ix.n;
    });
}

static rvx_status hyp_search_host(const rvx_hyperbolic* h, const float* q, int64_t nq, int32_t k, int32_t ef,
                                  int64_t* ids, float* dist, int32_t* counts, int mode) {
    return guard([&] {
        RVX_REQUIRE(h && nq >= 0 && k >= 1 && (nq == 0 || (q && ids && dist)), RVX_ERR_INVALID_PARAMETER,
                    "bad search arguments");
        if (nq == 0) return;
        std::shared_lock<std::shared_mutex> lk(h->ix.mu);
        ComputeLock cl;
        const int m = (mode == 2 && !h->ix.tan_valid) ? 0 : mode;  // no cache -> regular search (hnsw.rs:452-454)
        float* dq = projected_queries(h, q, nq, false);
        auto* di = (int64_t*)scratch_bytes("hyp_out_i", nq * k * 8);
        float* dd = scratch_f32("hyp_out_d", nq * k);
        int32_t* dn = counts ? (int32_t*)scratch_bytes("hyp_out_n", nq * 4) : nullptr;
        search_dev(h, dq, nq, k, ef, di, dd, dn, m);
        RVX_HIP(hipMemcpyAsync(ids, di, (size_t)(nq * k * 8), hipMemcpyDeviceToHost, stream()));
        RVX_HIP(hipMemcpyAsync(dist, dd, (size_t)(nq * k * 4), hipMemcpyDeviceToHost, stream()));
        if (counts) RVX_HIP(hipMemcpyAsync(counts, dn, (size_t)(nq * 4), hipMemcpyDeviceToHost, stream()));
        sync();
    });
}

rvx_status rvx_hyperbolic_search(const rvx_hyperbolic* h, const float* q, int64_t nq, int32_t k, int32_t ef,
                                 int64_t* ids, float* dist, int32_t* counts) {
    return hyp_search_host(h, q, nq, k, ef, ids, dist, counts, 0);
}

rvx_status rvx_hyperbolic_search_with_pruning(const rvx_hyperbolic* h, const float* q, int64_t nq, int32_t k,
                                              int64_t* ids, float* dist, int32_t* counts) {
    return hyp_search_host(h, q, nq, k, 0, ids, dist, counts, 2);
}

rvx_status rvx_hyperbolic_brute_force(const rvx_hyperbolic* h, const float* q, int64_t nq, int32_t k, int64_t* ids,
                                      float* dist) {
    return hyp_search_host(h, q, nq, k, 0, ids, dist, nullptr, 1);
}

rvx_status rvx_hyperbolic_search_device(const rvx_hyperbolic* h, const rvx_buffer* q, int64_t nq, int32_t k, int32_t ef,
                                        int32_t mode, rvx_buffer* ids, rvx_buffer* dist) {
    return guard([&] {
        RVX_REQUIRE(h && q && ids && dist && nq >= 0 && k >= 1 && mode >= 0 && mode <= 2, RVX_ERR_INVALID_PARAMETER,
                    "bad search arguments");
        RVX_REQUIRE(q->mem.bytes >= nq * h->cfg.dim * 4 && ids->mem.bytes >= nq * k * 8 && dist->mem.bytes >= nq * k * 4,
                    RVX_ERR_DIMENSION_MISMATCH, "buffer too small");
        if (nq == 0) return;
        std::shared_lock<std::shared_mutex> lk(h->ix.mu);
        ComputeLock cl;
        const int m = (mode == 2 && !h->ix.tan_valid) ? 0 : mode;
        float* dq = projected_queries(h, q->mem.as<float>(), nq, true);
        search_dev(h, dq, nq, k, ef, ids->mem.as<int64_t>(), dist->mem.as<float>(), nullptr, m);
    });
}

// The shard-dependent conditions search_dev enforces (pruned: the Poincaré metric;
// graph: a fresh graph), checked locally before the sharded entry points enter any
// collective. k, ef and k * prune_factor are unbounded as in the reference
// (hnsw.rs:427-489).
static void hyp_shard_precheck(const rvx_hyperbolic* h, int64_t nq, int k, int ef, int mode) {
    RVX_REQUIRE(h && nq >= 0 && k >= 1 && mode >= 0 && mode <= 2, RVX_ERR_INVALID_PARAMETER,
                "bad sharded search arguments");
    const rvx_index* ix = &h->ix;
    if (ix->n == 0 || nq == 0) return;
    const int m = (mode == 2 && !ix->tan_valid) ? 0 : mode;
    if (m == 2) {
        RVX_REQUIRE(ix->cfg.metric == RVX_METRIC_POINCARE, RVX_ERR_UNSUPPORTED,
                    "search_with_pruning is implemented for the Poincaré metric");
        RVX_REQUIRE((int64_t)k * h->cfg.prune_factor < ((int64_t)1 << 31), RVX_ERR_INVALID_PARAMETER,
                    "k * prune_factor too large");
    } else if (m == 0) {
        RVX_REQUIRE(ix->has_graph && ix->graph_n == ix->n, RVX_ERR_INDEX, "HNSW graph missing or stale");
    }
}

// ShardedHyperbolicHnsw::search across processes (shard.rs:354-373): rank 0's
// queries are broadcast, every rank searches its node-range shard (local ids +
// id_base = global ids), one all-gather moves every rank's top-k, and each rank
// merges them on the GPU. q_dev: the queries on rank 0 (device), ignored elsewhere.
static void sharded_search_dev(const rvx_hyperbolic* h, rvx_comm* comm, int64_t id_base, const float* q_dev,
                               int64_t nq, int k, int ef, int mode, int64_t* gid, int64_t* lid, float* dist,
                               int32_t* counts) {
    const int d = h->ix.cfg.dim;
    float* dq = scratch_f32("shard_q", nq * d);
    if (comm_rank(comm) == 0)
        RVX_HIP(hipMemcpyAsync(dq, q_dev, (size_t)(nq * d * 4), hipMemcpyDeviceToDevice, stream()));
    {
        ProfScope ps("shard_bcast");
        comm_broadcast_bytes(comm, dq, nq * d * 4, 0, stream());
    }
    project_rows(dq, nq, d, h->ix.curv);
    const int m = (mode == 2 && !h->ix.tan_valid) ? 0 : mode;  // no cache -> regular search (hnsw.rs:450-454)
    auto* li = (int64_t*)scratch_bytes("shard_local_i", nq * k * 8);
    float* ld = scratch_f32("shard_local_d", nq * k);
    search_dev(h, dq, nq, k, ef, li, ld, nullptr, m);
    auto* gi = (int64_t*)scratch_bytes("shard_local_g", nq * k * 8);
    offset_ids(li, nq * k, id_base, gi);
    sharded_merge(comm, gi, li, ld, nq, k, gid, lid, dist, counts);
}

rvx_status rvx_hyperbolic_sharded_search(const rvx_hyperbolic* h, rvx_comm* comm, int64_t id_base, const float* q,
                                         int64_t nq, int32_t k, int32_t ef, int32_t mode, int64_t* out_gid,
                                         int64_t* out_lid, float* out_dist, int32_t* out_count) {
    return guard([&] {
        rvx_status st = RVX_OK;
        std::string why;
        try {  // local verdict first; every rank learns every verdict before any data moves
            hyp_shard_precheck(h, nq, k, ef, mode);
            RVX_REQUIRE(id_base >= 0, RVX_ERR_INVALID_PARAMETER, "bad sharded search arguments");
            RVX_REQUIRE(nq == 0 || (out_gid && out_dist && (comm_rank(comm) != 0 || q)), RVX_ERR_INVALID_PARAMETER,
                        "null argument");
        } catch (const Error& e) {
            st = e.code;
            why = e.what();
        }
        shard_agree(comm, st, why, {nq, (int64_t)k, (int64_t)ef, (int64_t)mode, h ? (int64_t)h->cfg.dim : 0});
        if (nq == 0) return;
        std::shared_lock<std::shared_mutex> lk(h->ix.mu);
        ComputeLock cl;
        const int d = h->ix.cfg.dim;
        float* hq = scratch_f32("shard_hq", nq * d);
        if (comm_rank(comm) == 0)
            RVX_HIP(hipMemcpyAsync(hq, q, (size_t)(nq * d * 4), hipMemcpyHostToDevice, stream()));
        auto* gi = (int64_t*)scratch_bytes("shard_out_g", nq * k * 8);
        auto* li = (int64_t*)scratch_bytes("shard_out_l", nq * k * 8);
        float* dd = scratch_f32("shard_out_d", nq * k);
        auto* dn = (int32_t*)scratch_bytes("shard_out_n", nq * 4);
        sharded_search_dev(h, comm, id_base, hq, nq, k, ef, mode, gi, li, dd, dn);
        RVX_HIP(hipMemcpyAsync(out_gid, gi, (size_t)(nq * k * 8), hipMemcpyDeviceToHost, stream()));
        if (out_lid) RVX_HIP(hipMemcpyAsync(out_lid, li, (size_t)(nq * k * 8), hipMemcpyDeviceToHost, stream()));
        RVX_HIP(hipMemcpyAsync(out_dist, dd, (size_t)(nq * k * 4), hipMemcpyDeviceToHost, stream()));
        if (out_count) RVX_HIP(hipMemcpyAsync(out_count, dn, (size_t)(nq * 4), hipMemcpyDeviceToHost, stream()));
        sync();
    });
}

rvx_status rvx_hyperbolic_sharded_search_device(const rvx_hyperbolic* h, rvx_comm* comm, int64_t id_base,
                                                const rvx_buffer* q, int64_t nq, int32_t k, int32_t ef, int32_t mode,
                                                rvx_buffer* out_gid, rvx_buffer* out_lid, rvx_buffer* out_dist) {
    return guard([&] {
        rvx_status st = RVX_OK;
        std::string why;
        try {  // local verdict first; every rank learns every verdict before any data moves
            hyp_shard_precheck(h, nq, k, ef, mode);
            RVX_REQUIRE(id_base >= 0 && out_gid && out_dist, RVX_ERR_INVALID_PARAMETER, "bad sharded search arguments");
            RVX_REQUIRE(comm_rank(comm) != 0 || (q && q->mem.bytes >= nq * h->cfg.dim * 4), RVX_ERR_DIMENSION_MISMATCH,
                        "query buffer too small");
            RVX_REQUIRE(out_gid->mem.bytes >= nq * k * 8 && out_dist->mem.bytes >= nq * k * 4 &&
                            (!out_lid || out_lid->mem.bytes >= nq * k * 8),
                        RVX_ERR_DIMENSION_MISMATCH, "output buffer too small");
        } catch (const Error& e) {
            st = e.code;
            why = e.what();
        }
        shard_agree(comm, st, why, {nq, (int64_t)k, (int64_t)ef, (int64_t)mode, h ? (int64_t)h->cfg.dim : 0});
        if (nq == 0) return;
        std::shared_lock<std::shared_mutex> lk(h->ix.mu);
        ComputeLock cl;
        sharded_search_dev(h, comm, id_base, comm_rank(comm) == 0 ? q->mem.as<float>() : nullptr, nq, k, ef, mode,
                           out_gid->mem.as<int64_t>(), out_lid ? out_lid->mem.as<int64_t>() : nullptr,
                           out_dist->mem.as<float>(), nullptr);
    });
}

rvx_status rvx_hyperbolic_build_tangent_cache(rvx_hyperbolic* h) {
    return guard([&] {
        RVX_REQUIRE(h, RVX_ERR_INVALID_PARAMETER, "null argument");
        std::unique_lock<std::shared_mutex> lk(h->ix.mu);
        if (h->ix.n == 0) return;  // build_tangent_cache: Ok(()) on an empty index (hnsw.rs:493-495)
        ComputeLock cl;
        build_tangent(h);
    });
}

rvx_status rvx_hyperbolic_tangent_centroid(const rvx_hyperbolic* h, float* centroid) {
    return guard([&] {
        RVX_REQUIRE(h && centroid, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(h->ix.tan_valid, RVX_ERR_NOT_FOUND, "no tangent cache");
        h->ix.tan_centroid.download(centroid, (int64_t)h->cfg.dim * 4);
    });
}

rvx_status rvx_hyperbolic_get_vector(const rvx_hyperbolic* h, int64_t id, float* out) {
    return guard([&] {
        RVX_REQUIRE(h && out, RVX_ERR_INVALID_PARAMETER, "null argument");
        std::shared_lock<std::shared_mutex> lk(h->ix.mu);
        RVX_REQUIRE(id >= 0 && id < h->ix.n, RVX_ERR_NOT_FOUND, "no such id");
        h->ix.vecs.download(out, (int64_t)h->cfg.dim * 4, id * h->cfg.dim * 4);
    });
}

rvx_status rvx_hyperbolic_set_curvature(rvx_hyperbolic* h, float curvature) {
    return guard([&] {
        RVX_REQUIRE(h, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(curvature > 0.0f, RVX_ERR_INVALID_PARAMETER, "invalid curvature (must be > 0)");
        std::unique_lock<std::shared_mutex> lk(h->ix.mu);
        ComputeLock cl;
        // set_curvature (hnsw.rs:510-528): reproject every vector, rebuild an existing cache
        h->cfg.curvature = curvature;
        h->ix.curv = curvature;
        h->ix.cfg.curvature = curvature;
        project_rows(h->ix.vecs.as<float>(), h->ix.n, h->cfg.dim, curvature);
        sync();
        if (h->ix.tan_valid) build_tangent(h);
    });
}

}  // extern "C"
