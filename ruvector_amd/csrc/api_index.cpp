// api_index.cpp — VectorIndex over HBM (crates/ruvector-core/src/index.rs:11-36):
// FlatIndex (index/flat.rs) and HnswIndex (index/hnsw.rs) semantics, plus the
// distance-matrix entry point (distance.rs:9-107).
#include <algorithm>
#include <shared_mutex>
#include <unordered_map>

#include "comm.hpp"
#include "graph.hpp"
#include "hnsw.hpp"
#include "hyper.hpp"
#include "index.hpp"
#include "kernels.hpp"
#include "scan.hpp"

using namespace rvx;

namespace {

__global__ void k_map_ids(const int64_t* rows, const float* dist, int64_t nq, int k, const uint64_t* ids,
                          const uint8_t* deleted, int compact, uint64_t* out_ids, float* out_d, int32_t* out_n) {
    const int64_t qi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (qi >= nq) return;
    int w = 0;
    for (int s = 0; s < k; ++s) {
        const int64_t r = rows[qi * k + s];
        if (r < 0 || r == INT64_MAX) continue;
        if (compact && deleted[r]) continue;  // HnswIndex::search filter_map (index/hnsw.rs:250-258)
        out_ids[qi * k + w] = ids[r];
        out_d[qi * k + w] = dist[qi * k + s];
        ++w;
    }
    for (int s = w; s < k; ++s) { out_ids[qi * k + s] = UINT64_MAX; out_d[qi * k + s] = INFINITY; }
    if (out_n) out_n[qi] = w;
}

void ensure_capacity(rvx_index* ix, int64_t need) {
    if (need <= ix->cap) return;
    int64_t cap = std::max<int64_t>(need, std::max<int64_t>(1024, ix->cap * 2));
    if (ix->cfg.max_elements > 0) cap = std::max(need, std::min(cap, ix->cfg.max_elements));
    const int d = ix->cfg.dim;
    DevMem v(cap * d * 4), nr(cap * 4), idd(cap * 8), del(cap);
    if (ix->n) {
        RVX_HIP(hipMemcpyAsync(v.p, ix->vecs.p, (size_t)(ix->n * d * 4), hipMemcpyDeviceToDevice, stream()));
        RVX_HIP(hipMemcpyAsync(nr.p, ix->norms.p, (size_t)(ix->n * 4), hipMemcpyDeviceToDevice, stream()));
        RVX_HIP(hipMemcpyAsync(idd.p, ix->ids_dev.p, (size_t)(ix->n * 8), hipMemcpyDeviceToDevice, stream()));
        RVX_HIP(hipMemcpyAsync(del.p, ix->deleted.p, (size_t)ix->n, hipMemcpyDeviceToDevice, stream()));
    }
    sync();
    ix->vecs = std::move(v); ix->norms = std::move(nr); ix->ids_dev = std::move(idd); ix->deleted = std::move(del);
    ix->cap = cap;
}

void append_rows(rvx_index* ix, const float* dev_rows, const uint64_t* ids, int64_t cnt, bool rows_on_device) {
    const int d = ix->cfg.dim;
    for (int64_t i = 0; i < cnt; ++i)
        RVX_REQUIRE(ix->id_to_row.find(ids[i]) == ix->id_to_row.end(), RVX_ERR_INVALID_PARAMETER,
                    "duplicate vector id " + std::to_string(ids[i]));
    ensure_capacity(ix, ix->n + cnt);
    float* dst = ix->vecs.as<float>() + ix->n * d;
    RVX_HIP(hipMemcpyAsync(dst, dev_rows, (size_t)(cnt * d * 4),
                           rows_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, stream()));
    RVX_HIP(hipMemcpyAsync(ix->ids_dev.as<uint64_t>() + ix->n, ids, (size_t)(cnt * 8), hipMemcpyHostToDevice, stream()));
    RVX_HIP(hipMemsetAsync(ix->deleted.as<uint8_t>() + ix->n, 0, (size_t)cnt, stream()));
    row_norms(dst, cnt, d, ix->norms.as<float>() + ix->n);
    for (int64_t i = 0; i < cnt; ++i) {
        ix->id_to_row[ids[i]] = ix->n + i;
        ix->ids.push_back(ids[i]);
        ix->deleted_h.push_back(0);
    }
    ix->n += cnt;
    ix->live += cnt;
    sync();
}

// Device search core: rows/dist for nq queries (q on device).
void search_rows(const rvx_index* ix, const float* q, int64_t nq, int k, int ef, float* dd, int64_t* di, int32_t* dn,
                 bool exact) {
    const int d = ix->cfg.dim;
    if (ix->n == 0) {  // an empty index answers every query with no result (flat.rs:36-76 over no entries)
        RVX_HIP(hipMemsetD32Async((hipDeviceptr_t)dd, 0x7F800000u, (size_t)(nq * k), stream()));  // +inf
        RVX_HIP(hipMemsetAsync(di, 0xFF, (size_t)(nq * k * 8), stream()));                         // row -1
        if (dn) RVX_HIP(hipMemsetAsync(dn, 0, (size_t)(nq * 4), stream()));
        return;
    }
    float* qn = nullptr;
    if (ix->cfg.metric == RVX_METRIC_COSINE) {
        qn = scratch_f32("index_qnorm", nq);
        row_norms(q, nq, d, qn);
    }
    if (exact && ix->cfg.metric == RVX_METRIC_POINCARE) {
        poincare_topk(q, nq, ix->vecs.as<float>(), ix->n, d, ix->curv, k, dd, di);
        return;
    }
    if (exact || ix->cfg.kind == RVX_INDEX_FLAT) {
        scan_topk(ix->cfg.metric, q, qn, nq, ix->vecs.as<float>(), ix->norms.as<float>(),
                  ix->cfg.kind == RVX_INDEX_FLAT ? ix->deleted.as<uint8_t>() : nullptr, ix->n, d, k, 0, dd, di,
                  exact ? "brute_force" : "flat_search");
        return;
    }
    RVX_REQUIRE(ix->has_graph && ix->graph_n == ix->n, RVX_ERR_INDEX,
                "HNSW graph missing or stale");
    const int e = std::max(ef > 0 ? ef : ix->cfg.ef_search, k);  // ef = max(ef_arg, knbn) (hnsw.rs:1519)
    hnsw_search(ix->g, ix->cfg.metric, ix->vecs.as<float>(), ix->norms.as<float>(), d, q, qn, nq, k, e, dd, di, dn,
                "hnsw_search", ix->curv, ix->hyper ? 1 : 0);
}

void map_out(const rvx_index* ix, const int64_t* di, const float* dd, int64_t nq, int k, uint64_t* oi, float* od,
             int32_t* on, bool compact) {
    hipLaunchKernelGGL(k_map_ids, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, stream(), di, dd, nq, k,
                       ix->ids_dev.as<uint64_t>(), ix->deleted.as<uint8_t>(), compact ? 1 : 0, oi, od, on);
    RVX_HIP(hipGetLastError());
}

void check_query_args(const rvx_index* ix, int64_t nq, int k) {
    RVX_REQUIRE(ix, RVX_ERR_INVALID_PARAMETER, "null index");
    RVX_REQUIRE(nq >= 0 && k >= 1, RVX_ERR_INVALID_PARAMETER, "nq >= 0 and k >= 1 required");
}

// The shard-dependent conditions search_rows enforces, checked locally before the
// sharded entry points enter any collective (shard_agree).
void index_shard_precheck(const rvx_index* ix, int64_t nq, int k, int ef, bool exact) {
    check_query_args(ix, nq, k);
    if (ix->n == 0 || nq == 0) return;
    if (exact || ix->cfg.kind == RVX_INDEX_FLAT) return;  // any k (flat.rs:63-64)
    RVX_REQUIRE(ix->has_graph && ix->graph_n == ix->n, RVX_ERR_INDEX, "HNSW graph missing or stale");
}

}  // namespace

namespace rvx {

void index_append_rows(rvx_index* ix, const float* rows, const uint64_t* ids, int64_t cnt, bool rows_on_device) {
    append_rows(ix, rows, ids, cnt, rows_on_device);
}

void index_search_rows(const rvx_index* ix, const float* q, int64_t nq, int k, int ef, float* dd, int64_t* di,
                       int32_t* dn, bool exact) {
    search_rows(ix, q, nq, k, ef, dd, di, dn, exact);
}

// Validate a caller's graph and make it the searchable graph (caller holds ix->mu).
void index_load_graph(rvx_index* ix, const rvx_hnsw_graph* hg) {
    RVX_REQUIRE(hg->n == ix->n, RVX_ERR_DIMENSION_MISMATCH, "graph size != number of stored vectors");
    RVX_REQUIRE(hg->max_level >= 0 && hg->max_level <= HNSW_MAX_LEVEL, RVX_ERR_INVALID_PARAMETER, "bad max_level");
    RVX_REQUIRE(hg->n == 0 || (hg->entry_point >= 0 && hg->entry_point < hg->n), RVX_ERR_INDEX, "bad entry point");
    const int64_t n = hg->n;
    HostGraph h;
    h.n = n;
    h.max_level = hg->max_level;
    h.entry = hg->entry_point;
    h.levels.assign(hg->levels, hg->levels + n);
    h.rp0.assign(hg->row_ptr0, hg->row_ptr0 + n + 1);
    RVX_REQUIRE(h.rp0[0] == 0, RVX_ERR_INDEX, "row_ptr0[0] must be 0");
    // validate layer 0: ids in range, no duplicate inside a list
    std::vector<int64_t> mark(n, -1);
    for (int64_t i = 0; i < n; ++i) {
        RVX_REQUIRE(h.rp0[i + 1] >= h.rp0[i], RVX_ERR_INDEX, "row_ptr0 must be non-decreasing");
        for (int64_t p = h.rp0[i]; p < h.rp0[i + 1]; ++p) {
            const int32_t c = hg->col0[p];
            RVX_REQUIRE(c >= 0 && c < n, RVX_ERR_INDEX, "layer-0 neighbour out of range");
            RVX_REQUIRE(mark[c] != i, RVX_ERR_INDEX, "duplicate neighbour in a layer-0 list");
            mark[c] = i;
        }
    }
    h.col0.assign(hg->col0, hg->col0 + h.rp0[n]);
    h.up_ids.assign(h.max_level + 1, {});
    h.up_rp.assign(h.max_level + 1, {});
    h.up_col.assign(h.max_level + 1, {});
    for (int l = 1; l <= h.max_level; ++l) {
        const int64_t cnt = hg->upper_count[l];
        for (int64_t i = 0; i < cnt; ++i) {
            RVX_REQUIRE(i == 0 || hg->upper_ids[l][i] > hg->upper_ids[l][i - 1], RVX_ERR_INDEX,
                        "upper-layer ids must be strictly increasing");
            RVX_REQUIRE(hg->upper_ids[l][i] >= 0 && hg->upper_ids[l][i] < n, RVX_ERR_INDEX, "upper id out of range");
        }
        h.up_ids[l].assign(hg->upper_ids[l], hg->upper_ids[l] + cnt);
        h.up_rp[l].assign(hg->upper_row_ptr[l], hg->upper_row_ptr[l] + cnt + 1);
        const int64_t ec = h.up_rp[l][cnt];
        for (int64_t p = 0; p < ec; ++p)
            RVX_REQUIRE(hg->upper_col[l][p] >= 0 && hg->upper_col[l][p] < n, RVX_ERR_INDEX, "upper neighbour out of range");
        h.up_col[l].assign(hg->upper_col[l], hg->upper_col[l] + ec);
    }
    ComputeLock cl;
    ix->build_valid = false;
    hnsw_install(ix, std::move(h));
}

}  // namespace rvx

extern "C" {

rvx_status rvx_index_create(const rvx_index_config* cfg, rvx_index** out) {
    return guard([&] {
        RVX_REQUIRE(cfg && out, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(cfg->dim > 0, RVX_ERR_INVALID_PARAMETER, "dimension must be positive");
        RVX_REQUIRE(cfg->kind == RVX_INDEX_FLAT || cfg->kind == RVX_INDEX_HNSW, RVX_ERR_INVALID_PARAMETER,
                    "unknown index kind");
        RVX_REQUIRE(cfg->metric >= RVX_METRIC_L2 && cfg->metric <= RVX_METRIC_L1, RVX_ERR_UNSUPPORTED,
                    "metric not supported by VectorIndex");
        if (cfg->kind == RVX_INDEX_HNSW) {
            RVX_REQUIRE(cfg->m > 0 && cfg->m <= 256, RVX_ERR_INVALID_PARAMETER, "m must be in [1,256] (hnsw.rs:785)");
            RVX_REQUIRE(cfg->metric != RVX_METRIC_DOT, RVX_ERR_INVALID_PARAMETER,
                        "DotProduct distances are negative; hnsw_rs asserts dist >= 0 (hnsw.rs:965)");
        }
        auto ix = std::make_unique<rvx_index>();
        ix->cfg = *cfg;
        if (ix->cfg.ef_search <= 0) ix->cfg.ef_search = 100;
        if (ix->cfg.ef_construction <= 0) ix->cfg.ef_construction = 200;
        *out = ix.release();
    });
}

rvx_status rvx_index_destroy(rvx_index* ix) {
    return guard([&] { delete ix; });
}

rvx_status rvx_index_add_batch(rvx_index* ix, const float* vecs, const uint64_t* ids, int64_t n) {
    return guard([&] {
        RVX_REQUIRE(ix && (n == 0 || (vecs && ids)) && n >= 0, RVX_ERR_INVALID_PARAMETER, "null argument");
        std::unique_lock<std::shared_mutex> lk(ix->mu);
        ComputeLock cl;
        append_rows(ix, vecs, ids, n, false);
        if (ix->cfg.kind == RVX_INDEX_HNSW) hnsw_insert_range(ix, ix->n - n, n);  // Hnsw::insert per vector
    });
}

rvx_status rvx_index_add_batch_device(rvx_index* ix, const rvx_buffer* vecs, int64_t n, uint64_t first_id) {
    return guard([&] {
        RVX_REQUIRE(ix && vecs && n >= 0, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(vecs->mem.bytes >= n * ix->cfg.dim * 4, RVX_ERR_DIMENSION_MISMATCH, "buffer smaller than n*dim");
        std::unique_lock<std::shared_mutex> lk(ix->mu);
        ComputeLock cl;
        std::vector<uint64_t> ids(n);
        for (int64_t i = 0; i < n; ++i) ids[i] = first_id + (uint64_t)i;
        append_rows(ix, vecs->mem.as<float>(), ids.data(), n, true);
        if (ix->cfg.kind == RVX_INDEX_HNSW) hnsw_insert_range(ix, ix->n - n, n);
    });
}

rvx_status rvx_index_len(const rvx_index* ix, int64_t* len) {
    return guard([&] {
        RVX_REQUIRE(ix && len, RVX_ERR_INVALID_PARAMETER, "null argument");
        std::shared_lock<std::shared_mutex> lk(ix->mu);
        *len = ix->live;
    });
}

rvx_status rvx_index_remove(rvx_index* ix, uint64_t id, int32_t* removed) {
    return guard([&] {
        RVX_REQUIRE(ix, RVX_ERR_INVALID_PARAMETER, "null index");
        std::unique_lock<std::shared_mutex> lk(ix->mu);
        auto it = ix->id_to_row.find(id);
        int32_t r = 0;
        if (it != ix->id_to_row.end() && !ix->deleted_h[it->second]) {
            const int64_t row = it->second;
            ix->deleted_h[row] = 1;
            const uint8_t one = 1;
            ix->deleted.upload(&one, 1, row);
            ix->live -= 1;
            r = 1;
        }
        if (removed) *removed = r;
    });
}

rvx_status rvx_index_search_device(const rvx_index* ix, const rvx_buffer* q, int64_t nq, int32_t k, int32_t ef,
                                   rvx_buffer* out_ids, rvx_buffer* out_dist) {
    return guard([&] {
        check_query_args(ix, nq, k);
        RVX_REQUIRE(q && out_ids && out_dist, RVX_ERR_INVALID_PARAMETER, "null buffer");
        RVX_REQUIRE(q->mem.bytes >= nq * ix->cfg.dim * 4, RVX_ERR_DIMENSION_MISMATCH, "query buffer too small");
        RVX_REQUIRE(out_ids->mem.bytes >= nq * k * 8 && out_dist->mem.bytes >= nq * k * 4, RVX_ERR_INVALID_PARAMETER,
                    "output buffers too small");
        std::shared_lock<std::shared_mutex> lk(ix->mu);
        ComputeLock cl;
        float* dd = scratch_f32("index_dd", nq * k);
        int64_t* di = (int64_t*)scratch_bytes("index_di", nq * k * 8);
        int32_t* dn = (int32_t*)scratch_bytes("index_dn", nq * 4);
        search_rows(ix, q->mem.as<float>(), nq, k, ef, dd, di, dn, false);
        map_out(ix, di, dd, nq, k, out_ids->mem.as<uint64_t>(), out_dist->mem.as<float>(), nullptr,
                ix->cfg.kind == RVX_INDEX_HNSW);
    });
}

rvx_status rvx_index_search(const rvx_index* ix, const float* q, int64_t nq, int32_t k, int32_t ef, uint64_t* out_ids,
                            float* out_dist, int32_t* out_count) {
    return guard([&] {
        check_query_args(ix, nq, k);
        RVX_REQUIRE(nq == 0 || (q && out_ids && out_dist), RVX_ERR_INVALID_PARAMETER, "null argument");
        if (nq == 0) return;
        std::shared_lock<std::shared_mutex> lk(ix->mu);
        ComputeLock cl;
        const int d = ix->cfg.dim;
        float* dq = scratch_f32("index_q", nq * d);
        RVX_HIP(hipMemcpyAsync(dq, q, (size_t)(nq * d * 4), hipMemcpyHostToDevice, stream()));
        float* dd = scratch_f32("index_dd", nq * k);
        int64_t* di = (int64_t*)scratch_bytes("index_di", nq * k * 8);
        int32_t* dn = (int32_t*)scratch_bytes("index_dn", nq * 4);
        search_rows(ix, dq, nq, k, ef, dd, di, dn, false);
        uint64_t* oi = (uint64_t*)scratch_bytes("index_oi", nq * k * 8);
        float* od = scratch_f32("index_od", nq * k);
        int32_t* on = (int32_t*)scratch_bytes("index_on", nq * 4);
        map_out(ix, di, dd, nq, k, oi, od, on, ix->cfg.kind == RVX_INDEX_HNSW);
        RVX_HIP(hipMemcpyAsync(out_ids, oi, (size_t)(nq * k * 8), hipMemcpyDeviceToHost, stream()));
        RVX_HIP(hipMemcpyAsync(out_dist, od, (size_t)(nq * k * 4), hipMemcpyDeviceToHost, stream()));
        if (out_count) RVX_HIP(hipMemcpyAsync(out_count, on, (size_t)(nq * 4), hipMemcpyDeviceToHost, stream()));
        sync();
        if (ix->cfg.kind == RVX_INDEX_HNSW) hnsw_search_check();  // (after the wait above: no extra sync)
    });
}

rvx_status rvx_index_brute_force_device(const rvx_index* ix, const rvx_buffer* q, int64_t nq, int32_t k,
                                        rvx_buffer* out_ids, rvx_buffer* out_dist) {
    return guard([&] {
        check_query_args(ix, nq, k);
        RVX_REQUIRE(q && out_ids && out_dist, RVX_ERR_INVALID_PARAMETER, "null buffer");
        RVX_REQUIRE(q->mem.bytes >= nq * ix->cfg.dim * 4, RVX_ERR_DIMENSION_MISMATCH, "query buffer too small");
        std::shared_lock<std::shared_mutex> lk(ix->mu);
        ComputeLock cl;
        float* dd = scratch_f32("index_dd", nq * k);
        int64_t* di = (int64_t*)scratch_bytes("index_di", nq * k * 8);
        search_rows(ix, q->mem.as<float>(), nq, k, 0, dd, di, nullptr, true);
        map_out(ix, di, dd, nq, k, out_ids->mem.as<uint64_t>(), out_dist->mem.as<float>(), nullptr, false);
    });
}

rvx_status rvx_index_brute_force(const rvx_index* ix, const float* q, int64_t nq, int32_t k, uint64_t* out_ids,
                                 float* out_dist) {
    return guard([&] {
        check_query_args(ix, nq, k);
        if (nq == 0) return;
        RVX_REQUIRE(q && out_ids && out_dist, RVX_ERR_INVALID_PARAMETER, "null argument");
        std::shared_lock<std::shared_mutex> lk(ix->mu);
        ComputeLock cl;
        const int d = ix->cfg.dim;
        float* dq = scratch_f32("index_q", nq * d);
        RVX_HIP(hipMemcpyAsync(dq, q, (size_t)(nq * d * 4), hipMemcpyHostToDevice, stream()));
        float* dd = scratch_f32("index_dd", nq * k);
        int64_t* di = (int64_t*)scratch_bytes("index_di", nq * k * 8);
        search_rows(ix, dq, nq, k, 0, dd, di, nullptr, true);
        uint64_t* oi = (uint64_t*)scratch_bytes("index_oi", nq * k * 8);
        float* od = scratch_f32("index_od", nq * k);
        map_out(ix, di, dd, nq, k, oi, od, nullptr, false);
        RVX_HIP(hipMemcpyAsync(out_ids, oi, (size_t)(nq * k * 8), hipMemcpyDeviceToHost, stream()));
        RVX_HIP(hipMemcpyAsync(out_dist, od, (size_t)(nq * k * 4), hipMemcpyDeviceToHost, stream()));
        sync();
    });
}

// Node-range-sharded VectorIndex search across processes (SURVEY.md §8e option 2, the
// merge of shard.rs:354-373 applied to ruvector-core indices): rank 0's queries are
// broadcast, every rank searches its shard (exact = 1: FlatIndex scan), the per-rank
// (user id, distance) lists are all-gathered and merged on every rank by distance,
// ties in rank order. User ids are global by construction (the caller's keys).
static void index_sharded_dev(const rvx_index* ix, rvx_comm* comm, const float* q_dev, int64_t nq, int k, int ef,
                              bool exact, uint64_t* oi, float* od, int32_t* on) {
    const int d = ix->cfg.dim;
    float* dq = scratch_f32("shard_q", nq * d);
    if (comm_rank(comm) == 0)
        RVX_HIP(hipMemcpyAsync(dq, q_dev, (size_t)(nq * d * 4), hipMemcpyDeviceToDevice, stream()));
    {
        ProfScope ps("shard_bcast");
        comm_broadcast_bytes(comm, dq, nq * d * 4, 0, stream());
    }
    float* dd = scratch_f32("index_dd", nq * k);
    int64_t* di = (int64_t*)scratch_bytes("index_di", nq * k * 8);
    search_rows(ix, dq, nq, k, ef, dd, di, nullptr, exact);
    auto* li = (uint64_t*)scratch_bytes("shard_local_u", nq * k * 8);
    float* ld = scratch_f32("shard_local_d", nq * k);
    map_out(ix, di, dd, nq, k, li, ld, nullptr, !exact && ix->cfg.kind == RVX_INDEX_HNSW);
    sharded_merge(comm, (const int64_t*)li, nullptr, ld, nq, k, (int64_t*)oi, nullptr, od, on);
}

rvx_status rvx_index_sharded_search(const rvx_index* ix, rvx_comm* comm, const float* q, int64_t nq, int32_t k,
                                    int32_t ef, int32_t exact, uint64_t* out_ids, float* out_dist,
                                    int32_t* out_count) {
    return guard([&] {
        rvx_status st = RVX_OK;
        std::string why;
        try {  // local verdict first; every rank learns every verdict before any data moves
            index_shard_precheck(ix, nq, k, ef, exact != 0);
            RVX_REQUIRE(nq == 0 || (out_ids && out_dist && (comm_rank(comm) != 0 || q)), RVX_ERR_INVALID_PARAMETER,
                        "null argument");
        } catch (const Error& e) {
            st = e.code;
            why = e.what();
        }
        shard_agree(comm, st, why, {nq, (int64_t)k, (int64_t)ef, (int64_t)exact, ix ? (int64_t)ix->cfg.dim : 0});
        if (nq == 0) return;
        std::shared_lock<std::shared_mutex> lk(ix->mu);
        ComputeLock cl;
        const int d = ix->cfg.dim;
        float* hq = scratch_f32("shard_hq", nq * d);
        if (comm_rank(comm) == 0)
            RVX_HIP(hipMemcpyAsync(hq, q, (size_t)(nq * d * 4), hipMemcpyHostToDevice, stream()));
        uint64_t* oi = (uint64_t*)scratch_bytes("shard_out_u", nq * k * 8);
        float* od = scratch_f32("shard_out_d", nq * k);
        int32_t* on = (int32_t*)scratch_bytes("shard_out_n", nq * 4);
        index_sharded_dev(ix, comm, hq, nq, k, ef, exact != 0, oi, od, on);
        RVX_HIP(hipMemcpyAsync(out_ids, oi, (size_t)(nq * k * 8), hipMemcpyDeviceToHost, stream()));
        RVX_HIP(hipMemcpyAsync(out_dist, od, (size_t)(nq * k * 4), hipMemcpyDeviceToHost, stream()));
        if (out_count) RVX_HIP(hipMemcpyAsync(out_count, on, (size_t)(nq * 4), hipMemcpyDeviceToHost, stream()));
        sync();
    });
}

rvx_status rvx_index_sharded_search_device(const rvx_index* ix, rvx_comm* comm, const rvx_buffer* q, int64_t nq,
                                           int32_t k, int32_t ef, int32_t exact, rvx_buffer* out_ids,
                                           rvx_buffer* out_dist) {
    return guard([&] {
        rvx_status st = RVX_OK;
        std::string why;
        try {  // local verdict first; every rank learns every verdict before any data moves
            index_shard_precheck(ix, nq, k, ef, exact != 0);
            RVX_REQUIRE(out_ids && out_dist, RVX_ERR_INVALID_PARAMETER, "null buffer");
            RVX_REQUIRE(comm_rank(comm) != 0 || (q && q->mem.bytes >= nq * ix->cfg.dim * 4),
                        RVX_ERR_DIMENSION_MISMATCH, "query buffer too small");
            RVX_REQUIRE(out_ids->mem.bytes >= nq * k * 8 && out_dist->mem.bytes >= nq * k * 4,
                        RVX_ERR_DIMENSION_MISMATCH, "output buffers too small");
        } catch (const Error& e) {
            st = e.code;
            why = e.what();
        }
        shard_agree(comm, st, why, {nq, (int64_t)k, (int64_t)ef, (int64_t)exact, ix ? (int64_t)ix->cfg.dim : 0});
        if (nq == 0) return;
        std::shared_lock<std::shared_mutex> lk(ix->mu);
        ComputeLock cl;
        index_sharded_dev(ix, comm, comm_rank(comm) == 0 ? q->mem.as<float>() : nullptr, nq, k, ef, exact != 0,
                          out_ids->mem.as<uint64_t>(), out_dist->mem.as<float>(), nullptr);
    });
}

rvx_status rvx_index_load_graph(rvx_index* ix, const rvx_hnsw_graph* hg) {
    return guard([&] {
        RVX_REQUIRE(ix && hg, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(ix->cfg.kind == RVX_INDEX_HNSW, RVX_ERR_INVALID_PARAMETER, "not an HNSW index");
        std::unique_lock<std::shared_mutex> lk(ix->mu);
        index_load_graph(ix, hg);
    });
}

rvx_status rvx_index_graph_sizes(const rvx_index* ix, int64_t* n, int32_t* max_level, int64_t* entry, int64_t* e0,
                                 int64_t* upper_count, int64_t* upper_edges) {
    return guard([&] {
        RVX_REQUIRE(ix && ix->has_graph, RVX_ERR_INDEX, "no HNSW graph");
        std::shared_lock<std::shared_mutex> lk(ix->mu);
        const HostGraph& h = ix->hg;
        if (n) *n = h.n;
        if (max_level) *max_level = h.max_level;
        if (entry) *entry = h.entry;
        if (e0) *e0 = h.rp0.empty() ? 0 : h.rp0.back();
        for (int l = 0; l <= HNSW_MAX_LEVEL; ++l) {
            const bool has = l >= 1 && l <= h.max_level;
            if (upper_count) upper_count[l] = has ? (int64_t)h.up_ids[l].size() : 0;
            if (upper_edges) upper_edges[l] = has ? (int64_t)h.up_col[l].size() : 0;
        }
    });
}

rvx_status rvx_index_export_graph(const rvx_index* ix, uint8_t* levels, int64_t* row_ptr0, int32_t* col0,
                                  int32_t* up_ids, int64_t* up_row_ptr, int32_t* up_col) {
    return guard([&] {
        RVX_REQUIRE(ix && ix->has_graph, RVX_ERR_INDEX, "no HNSW graph");
        std::shared_lock<std::shared_mutex> lk(ix->mu);
        const HostGraph& h = ix->hg;
        if (levels) std::copy(h.levels.begin(), h.levels.end(), levels);
        if (row_ptr0) std::copy(h.rp0.begin(), h.rp0.end(), row_ptr0);
        if (col0) std::copy(h.col0.begin(), h.col0.end(), col0);
        int64_t oi = 0, orp = 0, oc = 0;
        for (int l = 1; l <= h.max_level; ++l) {
            if (up_ids) std::copy(h.up_ids[l].begin(), h.up_ids[l].end(), up_ids + oi);
            if (up_row_ptr) std::copy(h.up_rp[l].begin(), h.up_rp[l].end(), up_row_ptr + orp);
            if (up_col) std::copy(h.up_col[l].begin(), h.up_col[l].end(), up_col + oc);
            oi += (int64_t)h.up_ids[l].size();
            orp += (int64_t)h.up_rp[l].size();
            oc += (int64_t)h.up_col[l].size();
        }
    });
}

rvx_status rvx_index_layer0_size(const rvx_index* ix, int64_t* n, int64_t* e) {
    return guard([&] {
        RVX_REQUIRE(ix && ix->has_graph, RVX_ERR_INDEX, "no HNSW graph");
        std::shared_lock<std::shared_mutex> lk(ix->mu);
        if (n) *n = ix->graph_n;
        if (e) *e = ix->hg.rp0.empty() ? 0 : ix->hg.rp0.back();
    });
}

rvx_status rvx_index_export_layer0(const rvx_index* ix, int64_t* row_ptr, int32_t* col, float* dist) {
    return guard([&] {
        RVX_REQUIRE(ix && ix->has_graph, RVX_ERR_INDEX, "no HNSW graph");
        std::shared_lock<std::shared_mutex> lk(ix->mu);
        ComputeLock cl;
        const int64_t n = ix->graph_n, e = ix->hg.rp0.back();
        if (row_ptr) std::copy(ix->hg.rp0.begin(), ix->hg.rp0.end(), row_ptr);
        if (col) std::copy(ix->hg.col0.begin(), ix->hg.col0.end(), col);
        if (dist && e > 0) {
            // edge weight = distance(owner, neighbour) in the reference order
            float* dv = scratch_f32("export_dist", e);
            edge_distances(ix->cfg.metric, ix->vecs.as<float>(), ix->norms.as<float>(), ix->g.rp0, ix->g.col0, n,
                           ix->cfg.dim, dv);
            RVX_HIP(hipMemcpyAsync(dist, dv, (size_t)e * 4, hipMemcpyDeviceToHost, stream()));
            sync();
        }
    });
}

rvx_status rvx_distance_matrix(int32_t metric, const float* q, int64_t nq, const float* x, int64_t n, int32_t d,
                               float curvature, float* out) {
    return guard([&] {
        RVX_REQUIRE(d > 0 && nq >= 0 && n >= 0, RVX_ERR_INVALID_PARAMETER, "bad sizes");
        if (nq == 0 || n == 0) return;
        ComputeLock cl;
        float* dq = scratch_f32("dm_q", nq * d);
        float* dx = scratch_f32("dm_x", n * d);
        float* dout = scratch_f32("dm_out", nq * n);
        RVX_HIP(hipMemcpyAsync(dq, q, (size_t)(nq * d * 4), hipMemcpyHostToDevice, stream()));
        RVX_HIP(hipMemcpyAsync(dx, x, (size_t)(n * d * 4), hipMemcpyHostToDevice, stream()));
        if (metric == RVX_METRIC_POINCARE) {
            poincare_matrix(dq, nq, dx, n, d, curvature, dout);
        } else {
            float *qn = nullptr, *xn = nullptr;
            if (metric == RVX_METRIC_COSINE) {
                qn = scratch_f32("dm_qn", nq);
                xn = scratch_f32("dm_xn", n);
                row_norms(dq, nq, d, qn);
                row_norms(dx, n, d, xn);
            }
            distance_matrix(metric, dq, qn, nq, dx, xn, n, d, dout);
        }
        RVX_HIP(hipMemcpyAsync(out, dout, (size_t)(nq * n * 4), hipMemcpyDeviceToHost, stream()));
        sync();
    });
}

rvx_status rvx_selftest_libm(int32_t fn, uint64_t start, uint64_t stride, int64_t count, float* out) {
    return guard([&] {
        RVX_REQUIRE(fn >= 0 && fn <= 4 && count >= 0 && out, RVX_ERR_INVALID_PARAMETER, "bad selftest arguments");
        if (count == 0) return;
        ComputeLock cl;
        float* dout = scratch_f32("libm_out", count);
        libm_eval(fn, start, stride, count, dout);
        RVX_HIP(hipMemcpyAsync(out, dout, (size_t)count * 4, hipMemcpyDeviceToHost, stream()));
        sync();
    });
}

rvx_status rvx_scan_last_stats(int64_t* mfma_queries, int64_t* valu_queries, int64_t* fallback_queries) {
    return guard([&] {
        const ScanStats& s = last_scan_stats();
        if (mfma_queries) *mfma_queries = s.mfma_queries;
        if (valu_queries) *valu_queries = s.valu_queries;
        if (fallback_queries) *fallback_queries = s.fallback_queries;
    });
}

rvx_status rvx_scan_last_second_pass(int64_t* second_pass_queries) {
    return guard([&] {
        RVX_REQUIRE(second_pass_queries, RVX_ERR_INVALID_PARAMETER, "null argument");
        *second_pass_queries = last_scan_stats().second_pass_queries;
    });
}

rvx_status rvx_scan_last_band(int64_t* band_queries) {
    return guard([&] {
        RVX_REQUIRE(band_queries, RVX_ERR_INVALID_PARAMETER, "null argument");
        *band_queries = last_scan_stats().band_queries;
    });
}

rvx_status rvx_hnsw_last_search_stats(int64_t* n_dist, int64_t* n_expand, int64_t* nq) {
    return guard([&] {
        ComputeLock cl;
        hnsw_search_stats_settle();
        if (n_dist) *n_dist = g_search_stats.n_dist;
        if (n_expand) *n_expand = g_search_stats.n_expand;
        if (nq) *nq = g_search_stats.nq;
    });
}

rvx_status rvx_hnsw_last_search_visited(int32_t* bitmap, int32_t* slots) {
    return guard([&] {
        if (bitmap) *bitmap = g_search_stats.visited_bitmap;
        if (slots) *slots = g_search_stats.slots;
    });
}

rvx_status rvx_hnsw_last_search_form(int32_t* r_in_hbm, int32_t* stages, int32_t* visited_overflow) {
    return guard([&] {
        if (visited_overflow) {
            hnsw_search_stats_settle();
            *visited_overflow = g_search_stats.visited_overflow;
        }
        if (r_in_hbm) *r_in_hbm = g_search_stats.r_in_hbm;
        if (stages) *stages = g_search_stats.stages;
    });
}

}  // extern "C"
