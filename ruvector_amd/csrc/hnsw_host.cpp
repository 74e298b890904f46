// hnsw_host.cpp — host orchestration of the GPU HNSW build and graph install.
//
// HnswIndex::add_batch (crates/ruvector-core/src/index/hnsw.rs:287-329) inserts
// every new vector into the hnsw_rs graph; here the insertion runs in
// geometrically growing batches on the GPU (k_hnsw_build.hip), then the
// fixed-capacity lists are converted to the CSR the search kernel reads.
#include <cmath>

#include "graph.hpp"
#include "index.hpp"

namespace rvx {

namespace {
uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

template <class T>
void grow(DevMem& m, int64_t old_elems, int64_t new_elems, int fill_byte) {
    DevMem n((int64_t)std::max<int64_t>(new_elems, 1) * (int64_t)sizeof(T));
    if (old_elems > 0 && m.p)
        RVX_HIP(hipMemcpyAsync(n.p, m.p, (size_t)old_elems * sizeof(T), hipMemcpyDeviceToDevice, stream()));
    if (new_elems > old_elems)
        RVX_HIP(hipMemsetAsync((char*)n.p + old_elems * sizeof(T), fill_byte, (size_t)(new_elems - old_elems) * sizeof(T),
                               stream()));
    sync();
    m = std::move(n);
}

BuildGraph build_view(rvx_index* ix) {
    BuildGraph G;
    G.n_cap = ix->bn_cap;
    G.M = ix->cfg.m;
    G.C0 = ix->hyper ? ix->m0 : 2 * ix->cfg.m;
    G.max_layer = ix->hyper ? HNSW_MAX_LEVEL : std::min(16, ix->cfg.dim);
    G.level = ix->b_level.as<uint8_t>();
    G.nb0 = ix->b_nb0.as<int>();
    G.nbd0 = ix->b_nbd0.as<float>();
    G.cnt0 = ix->b_cnt0.as<int>();
    G.up_base = ix->b_up_base.as<int64_t>();
    G.nbu = ix->b_nbu.as<int>();
    G.nbud = ix->b_nbud.as<float>();
    G.cntu = ix->b_cntu.as<int>();
    return G;
}

HostGraph build_to_host(rvx_index* ix, int64_t n) {
    const int M = ix->cfg.m, C0 = ix->hyper ? ix->m0 : 2 * M;
    HostGraph hg;
    hg.n = n;
    hg.max_level = std::max(0, ix->entry_level);
    hg.entry = std::max(0, ix->entry);
    hg.levels.assign(ix->h_level.begin(), ix->h_level.begin() + n);
    std::vector<int> cnt0(n), nb0((size_t)n * C0);
    std::vector<float> nbd0((size_t)n * C0);
    ix->b_cnt0.download(cnt0.data(), n * 4);
    ix->b_nb0.download(nb0.data(), n * C0 * 4);
    ix->b_nbd0.download(nbd0.data(), n * C0 * 4);
    hg.rp0.resize(n + 1);
    hg.rp0[0] = 0;
    for (int64_t i = 0; i < n; ++i) hg.rp0[i + 1] = hg.rp0[i] + cnt0[i];
    hg.col0.resize(hg.rp0[n]);
    hg.dist0.resize(hg.rp0[n]);
    for (int64_t i = 0; i < n; ++i)
        for (int j = 0; j < cnt0[i]; ++j) {
            hg.col0[hg.rp0[i] + j] = nb0[(size_t)i * C0 + j];
            hg.dist0[hg.rp0[i] + j] = nbd0[(size_t)i * C0 + j];
        }
    const int64_t U = ix->n_upper;
    std::vector<int> cntu(std::max<int64_t>(U, 1)), nbu((size_t)std::max<int64_t>(U, 1) * M);
    if (U) {
        ix->b_cntu.download(cntu.data(), U * 4);
        ix->b_nbu.download(nbu.data(), U * M * 4);
    }
    hg.up_ids.assign(hg.max_level + 1, {});
    hg.up_rp.assign(hg.max_level + 1, {});
    hg.up_col.assign(hg.max_level + 1, {});
    for (int l = 1; l <= hg.max_level; ++l) {
        auto& ids = hg.up_ids[l];
        auto& rp = hg.up_rp[l];
        auto& col = hg.up_col[l];
        rp.push_back(0);
        for (int64_t p = 0; p < n; ++p) {
            if (hg.levels[p] < l) continue;
            const int64_t li = ix->h_up_base[p] + (l - 1);
            ids.push_back((int32_t)p);
            for (int j = 0; j < cntu[li]; ++j) col.push_back(nbu[(size_t)li * M + j]);
            rp.push_back((int64_t)col.size());
        }
    }
    return hg;
}

}  // namespace

int hnsw_level(uint64_t seed, int m, int max_layer, int64_t i) {
    const double scale = 1.0 / std::log((double)m);
    const double u = (double)(sm64(sm64(seed) + (uint64_t)i) >> 11) * (1.0 / 9007199254740992.0);
    const double lev = -std::log(u) * scale;
    int64_t ul = std::isfinite(lev) ? (int64_t)std::floor(lev) : (int64_t)1 << 40;
    if (ul >= max_layer) ul = (int64_t)(sm64(sm64(seed ^ 0xABCDEFull) + (uint64_t)i) % (uint64_t)max_layer);
    return (int)ul;
}

int hyper_level(uint64_t seed, float level_mult, int64_t i) {
    // r in (0, 1]: rand::random::<f32>() is [0, 1); r = 0 would give an
    // unbounded level, capped like every level at the storage limit
    const float r = (float)((sm64(sm64(seed) + (uint64_t)i) >> 40) + 1) * (1.0f / 16777216.0f);
    const float lev = -std::log(r) * level_mult;
    return (int)std::min<float>(std::floor(lev), (float)(HNSW_MAX_LEVEL - 1));
}

void hnsw_install(rvx_index* ix, HostGraph&& hg) {
    const int64_t n = hg.n;
    HnswDev g;
    g.n = n;
    g.max_level = hg.max_level;
    g.entry = hg.entry;
    for (int64_t i = 0; i < n; ++i) g.max_deg = std::max<int>(g.max_deg, (int)(hg.rp0[i + 1] - hg.rp0[i]));
    ix->rp0.reset((n + 1) * 8);
    ix->rp0.upload(hg.rp0.data(), (n + 1) * 8);
    ix->col0.reset(std::max<int64_t>((int64_t)hg.col0.size(), 1) * 4);
    ix->col0.upload(hg.col0.data(), (int64_t)hg.col0.size() * 4);
    g.rp0 = ix->rp0.as<int64_t>();
    g.col0 = ix->col0.as<int>();
    std::vector<int32_t> ids, cols;
    std::vector<int64_t> rps;
    for (int l = 1; l <= hg.max_level; ++l) {
        g.up_count[l] = (int64_t)hg.up_ids[l].size();
        g.up_ids_off[l] = (int64_t)ids.size();
        g.up_rp_off[l] = (int64_t)rps.size();
        g.up_col_off[l] = (int64_t)cols.size();
        ids.insert(ids.end(), hg.up_ids[l].begin(), hg.up_ids[l].end());
        rps.insert(rps.end(), hg.up_rp[l].begin(), hg.up_rp[l].end());
        cols.insert(cols.end(), hg.up_col[l].begin(), hg.up_col[l].end());
    }
    ix->up_ids.reset(std::max<size_t>(ids.size(), 1) * 4);
    ix->up_ids.upload(ids.data(), (int64_t)ids.size() * 4);
    ix->up_rp.reset(std::max<size_t>(rps.size(), 1) * 8);
    ix->up_rp.upload(rps.data(), (int64_t)rps.size() * 8);
    ix->up_col.reset(std::max<size_t>(cols.size(), 1) * 4);
    ix->up_col.upload(cols.data(), (int64_t)cols.size() * 4);
    g.up_ids = ix->up_ids.as<int>();
    g.up_rp = ix->up_rp.as<int64_t>();
    g.up_col = ix->up_col.as<int>();
    ix->g = g;
    ix->graph_n = n;
    ix->has_graph = true;
    ix->hg = std::move(hg);
}

void hnsw_insert_range(rvx_index* ix, int64_t first, int64_t count) {
    RVX_REQUIRE(ix->build_valid, RVX_ERR_UNSUPPORTED,
                "adding vectors to an HNSW index whose graph was loaded with rvx_index_load_graph is not supported");
    RVX_REQUIRE(ix->hyper ? (ix->cfg.m <= 128 && ix->m0 <= 256) : ix->cfg.m <= 128, RVX_ERR_UNSUPPORTED,
                "GPU HNSW construction supports layer-0 lists of <= 256 and upper lists of <= 128 neighbours");
    RVX_REQUIRE(ix->cfg.metric != RVX_METRIC_DOT, RVX_ERR_INVALID_PARAMETER, "DotProduct cannot be used with HNSW");
    if (count <= 0) return;
    const int M = ix->cfg.m, C0 = ix->hyper ? ix->m0 : 2 * M, max_layer = std::min(16, ix->cfg.dim);
    const int64_t end = first + count;
    RVX_REQUIRE(end < ((int64_t)1 << 31) - 1, RVX_ERR_INVALID_SHAPE, "too many points");
    for (int64_t i = first; i < end; ++i) {
        const int lev = ix->hyper ? hyper_level(ix->cfg.seed, ix->level_mult, i) : hnsw_level(ix->cfg.seed, M, max_layer, i);
        ix->h_level.push_back((uint8_t)lev);
        if (lev > 0) {
            ix->h_up_base.push_back(ix->n_upper);
            ix->n_upper += lev;
        } else {
            ix->h_up_base.push_back(-1);
        }
    }
    // capacity (lists keyed n_cap + upper index, so the reverse-edge heads are re-initialised on growth)
    if (end > ix->bn_cap || ix->n_upper > ix->bu_cap) {
        const int64_t ncap = std::max<int64_t>(end, ix->bn_cap * 2);
        const int64_t ucap = std::max<int64_t>(std::max<int64_t>(ix->n_upper, ix->bu_cap * 2), 64);
        grow<uint8_t>(ix->b_level, ix->bn_cap, ncap, 0);
        grow<int64_t>(ix->b_up_base, ix->bn_cap, ncap, 0xFF);
        grow<int>(ix->b_nb0, ix->bn_cap * C0, ncap * C0, 0);
        grow<float>(ix->b_nbd0, ix->bn_cap * C0, ncap * C0, 0);
        grow<int>(ix->b_cnt0, ix->bn_cap, ncap, 0);
        grow<int>(ix->b_nbu, ix->bu_cap * M, ucap * M, 0);
        grow<float>(ix->b_nbud, ix->bu_cap * M, ucap * M, 0);
        grow<int>(ix->b_cntu, ix->bu_cap, ucap, 0);
        ix->b_rev_head.reset((ncap + ucap) * 4);
        RVX_HIP(hipMemsetAsync(ix->b_rev_head.p, 0xFF, (size_t)(ncap + ucap) * 4, stream()));
        ix->bn_cap = ncap;
        ix->bu_cap = ucap;
    }
    ix->b_level.upload(ix->h_level.data() + first, count, first);
    ix->b_up_base.upload(ix->h_up_base.data() + first, count * 8, first * 8);
    BuildGraph G = build_view(ix);
    BuildScratch S;
    S.rev_head = ix->b_rev_head.as<int>();

    int64_t i = first;
    if (ix->entry < 0) {  // first point: it becomes the entry, no links (hnsw.rs:1084-1102)
        ix->entry = (int)i;
        ix->entry_level = ix->h_level[i];
        ix->level_mask |= 1u << ix->h_level[i];
        ++i;
    }
    while (i < end) {
        int64_t b = std::max<int64_t>(1, std::min<int64_t>(8192, i / 16));
        b = std::min(b, end - i);
        unsigned mask = ix->level_mask;
        for (int64_t p = i; p < i + b; ++p) mask |= 1u << ix->h_level[p];
        // HyperbolicHnsw::search_layer has no per-layer emptiness test: every
        // layer up to max_level holds the entry point
        const unsigned search_mask = ix->hyper ? 0xFFFFFFFFu : mask;
        build_insert_batch(G, ix->cfg.metric, ix->vecs.as<float>(), ix->norms.as<float>(), ix->cfg.dim, i, (int)b,
                           ix->entry, ix->entry_level, search_mask, ix->cfg.ef_construction, S, ix->curv,
                           ix->hyper ? 1 : 0);
        for (int64_t p = i; p < i + b; ++p)  // check_entry_point (hnsw.rs:529-552), first higher level wins
            if ((int)ix->h_level[p] > ix->entry_level) { ix->entry = (int)p; ix->entry_level = ix->h_level[p]; }
        ix->level_mask = mask;
        i += b;
    }
    hnsw_install(ix, build_to_host(ix, end));
}

}  // namespace rvx
