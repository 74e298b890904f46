// api_hnswio.cpp — hnsw_rs dump files (`<base>.hnsw.graph` + `<base>.hnsw.data`)
// for the HNSW index: write the searchable graph in the format
// patches/hnsw_rs/src/hnswio.rs reloads, and load such a dump onto the GPU.
//
// Format (hnswio.rs, native-endian; all counts `usize` = u64 here):
//   graph: Description::dump (:878-919) — MAGICDESCR_4 u32, dumpmode u8,
//          max_nb_connection u8, level_scale f64, nb_layer u8 (must be
//          NB_LAYER_MAX = 16), ef usize, nb_point usize, dimension usize,
//          distname (usize len + bytes), T name (usize len + bytes);
//          PointIndexation::dump (:1301-1332) — nb_layer u8, then per layer
//          MAGICLAYER u32 + nb_point usize + the layer's points in rank order;
//          a point (dump_point :1063-1095) is MAGICPOINT u32, origin_id usize,
//          [Full: layer u8, rank i32], then for each of nb_layer layers a
//          neighbour count usize and per neighbour d_id usize, [Full: layer
//          u8, rank i32], distance f32; finally the entry point's origin_id,
//          [Full: layer u8, rank i32].
//   data:  MAGICDATAP u32, dimension usize (:1349-1350), then per point in
//          graph order MAGICDATAP u32, origin_id u64, byte length u64, the
//          f32 values (:1099-1110).
// The reloader reads the point and neighbour PointIds unconditionally
// (load_point_graph :1221-1290, load_point_indexation :700-716), so only Full
// mode (dumpmode 1) round-trips; that is what is written and required here.
//
// Point ranks: hnsw_rs groups points by level (points_by_layer[l]) in
// insertion order; here the level-l points in ascending row order. A point
// may hold lists above its own level (entry-point links of insert, hnsw.rs:
// 1131-1135) and appear in upper lists (an early entry point found by the
// upper-layer descent); search traverses those, so every list round-trips.
#include <cstdio>
#include <cstring>
#include <string>

#include "graph.hpp"
#include "index.hpp"
#include "kernels.hpp"
#include "scan.hpp"

namespace rvx {
namespace {

constexpr uint32_t MAGICPOINT = 0x000a678f;
constexpr uint32_t MAGICDESCR_2 = 0x002a677f;
constexpr uint32_t MAGICDESCR_3 = 0x002a6771;
constexpr uint32_t MAGICDESCR_4 = 0x002a6779;
constexpr uint32_t MAGICLAYER = 0x000a676f;
constexpr uint32_t MAGICDATAP = 0xa67f0000;
constexpr int NB_LAYER_MAX = 16;

std::string path_of(const char* dir, const char* base, const char* suffix) {
    std::string p = dir && *dir ? std::string(dir) : std::string(".");
    if (p.back() != '/') p += '/';
    return p + base + suffix;
}

struct File {
    FILE* f = nullptr;
    std::string path;
    File(const std::string& p, const char* mode) : path(p) {
        f = std::fopen(p.c_str(), mode);
        RVX_REQUIRE(f, RVX_ERR_SERIALIZATION, "cannot open " + p);
        std::setvbuf(f, nullptr, _IOFBF, 1 << 22);
    }
    ~File() {
        if (f) std::fclose(f);
    }
    void put(const void* p, size_t n) {
        RVX_REQUIRE(std::fwrite(p, 1, n, f) == n, RVX_ERR_SERIALIZATION, "write failed: " + path);
    }
    void get(void* p, size_t n) {
        RVX_REQUIRE(std::fread(p, 1, n, f) == n, RVX_ERR_SERIALIZATION, "truncated file: " + path);
    }
    template <class T> void w(T v) { put(&v, sizeof v); }
    template <class T> T r() {
        T v;
        get(&v, sizeof v);
        return v;
    }
    void close() {
        RVX_REQUIRE(std::fclose(f) == 0, RVX_ERR_SERIALIZATION, "close failed: " + path);
        f = nullptr;
    }
};

const char* dist_name(int metric) {
    switch (metric) {
        case RVX_METRIC_L2: return "anndists::dist::distances::DistL2";
        case RVX_METRIC_COSINE: return "anndists::dist::distances::DistCosine";
        case RVX_METRIC_DOT: return "anndists::dist::distances::DistDot";
        case RVX_METRIC_L1: return "anndists::dist::distances::DistL1";
        default: return "";
    }
}

int metric_of(const std::string& name) {
    auto ends = [&](const char* s) {
        const size_t n = std::strlen(s);
        return name.size() >= n && name.compare(name.size() - n, n, s) == 0;
    };
    if (ends("DistL2")) return RVX_METRIC_L2;
    if (ends("DistCosine")) return RVX_METRIC_COSINE;
    if (ends("DistDot")) return RVX_METRIC_DOT;
    if (ends("DistL1")) return RVX_METRIC_L1;
    return -1;
}

// The names are Rust Strings in hnsw_rs (load_description decodes them as UTF-8 and
// errors otherwise, hnswio.rs:937-1040); a damaged dump is rejected the same way.
bool valid_utf8(const unsigned char* s, size_t n) {
    size_t i = 0;
    while (i < n) {
        const unsigned c = s[i];
        const int len = c < 0x80 ? 1 : (c >> 5) == 0x6 ? 2 : (c >> 4) == 0xE ? 3 : (c >> 3) == 0x1E ? 4 : 0;
        if (len == 0 || i + (size_t)len > n) return false;
        for (int k = 1; k < len; ++k)
            if ((s[i + k] & 0xC0) != 0x80) return false;
        i += (size_t)len;
    }
    return true;
}

void read_description(File& g, rvx_hnswio_description* d) {
    std::memset(d, 0, sizeof *d);
    const uint32_t magic = g.r<uint32_t>();
    if (magic == MAGICDESCR_2) d->format_version = 2;
    else if (magic == MAGICDESCR_3) d->format_version = 3;
    else if (magic == MAGICDESCR_4) d->format_version = 4;
    else fail(RVX_ERR_SERIALIZATION, "bad magic at description beginning");
    d->dump_mode = g.r<uint8_t>();
    d->max_nb_connection = g.r<uint8_t>();
    d->level_scale = d->format_version == 4 ? g.r<double>() : 1.0;
    d->nb_layer = g.r<uint8_t>();
    d->ef_construction = (int64_t)g.r<uint64_t>();
    d->nb_point = (int64_t)g.r<uint64_t>();
    d->dimension = (int64_t)g.r<uint64_t>();
    for (char* dst : {d->distname, d->t_name}) {
        const uint64_t len = g.r<uint64_t>();
        RVX_REQUIRE(len <= 256, RVX_ERR_SERIALIZATION, "name longer than 256 bytes");
        g.get(dst, (size_t)len);
        dst[len] = 0;
        RVX_REQUIRE(valid_utf8(reinterpret_cast<const unsigned char*>(dst), (size_t)len), RVX_ERR_SERIALIZATION,
                    "name in the dump description is not UTF-8");
    }
}

struct Nb {
    uint64_t d_id;
    uint8_t layer;
    int32_t rank;
    float dist;
};

}  // namespace
}  // namespace rvx

using namespace rvx;

extern "C" {

rvx_status rvx_hnswio_describe(const char* dir, const char* basename, rvx_hnswio_description* out) {
    return guard([&] {
        RVX_REQUIRE(basename && out, RVX_ERR_INVALID_PARAMETER, "null argument");
        File g(path_of(dir, basename, ".hnsw.graph"), "rb");
        read_description(g, out);
    });
}

rvx_status rvx_index_file_dump(const rvx_index* ix, const char* dir, const char* basename) {
    return guard([&] {
        RVX_REQUIRE(ix && basename, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(ix->cfg.kind == RVX_INDEX_HNSW && !ix->hyper, RVX_ERR_INVALID_PARAMETER,
                    "file_dump needs a (Euclidean-space) HNSW index");
        RVX_REQUIRE(ix->cfg.m <= 255, RVX_ERR_INVALID_PARAMETER, "max_nb_connection is dumped as u8");
        std::shared_lock<std::shared_mutex> lk(ix->mu);
        RVX_REQUIRE(ix->has_graph && ix->graph_n == ix->n, RVX_ERR_INDEX, "no HNSW graph over all points");
        ComputeLock cl;
        const HostGraph& h = ix->hg;
        const int64_t n = h.n;
        const int d = ix->cfg.dim;

        // ranks: level-l points in ascending row order
        std::vector<int32_t> rank(n);
        std::vector<std::vector<int64_t>> by_level(NB_LAYER_MAX);
        for (int64_t i = 0; i < n; ++i) {
            const int l = std::min<int>(h.levels[i], NB_LAYER_MAX - 1);
            rank[i] = (int32_t)by_level[l].size();
            by_level[l].push_back(i);
        }
        // edge distances (owner, neighbour) in the reference order, per layer
        std::vector<std::vector<float>> dist(h.max_level + 1);
        auto layer_dist = [&](const std::vector<int64_t>& rp, const std::vector<int32_t>& col, std::vector<float>& out) {
            const int64_t e = rp.back();
            out.resize(e);
            if (e == 0) return;
            auto* drp = (int64_t*)scratch_bytes("dump_rp", (n + 1) * 8);
            auto* dcol = (int32_t*)scratch_bytes("dump_col", e * 4);
            float* dd = scratch_f32("dump_dist", e);
            RVX_HIP(hipMemcpyAsync(drp, rp.data(), (size_t)(n + 1) * 8, hipMemcpyHostToDevice, stream()));
            RVX_HIP(hipMemcpyAsync(dcol, col.data(), (size_t)e * 4, hipMemcpyHostToDevice, stream()));
            edge_distances(ix->cfg.metric, ix->vecs.as<float>(), ix->norms.as<float>(), drp, dcol, n, d, dd);
            RVX_HIP(hipMemcpyAsync(out.data(), dd, (size_t)e * 4, hipMemcpyDeviceToHost, stream()));
            sync();
        };
        layer_dist(h.rp0, h.col0, dist[0]);
        // upper layer l as a CSR over all rows (rows without a list are empty)
        std::vector<std::vector<int64_t>> up_full(h.max_level + 1);
        for (int l = 1; l <= h.max_level; ++l) {
            std::vector<int64_t> rp(n + 1, 0);
            for (size_t j = 0; j < h.up_ids[l].size(); ++j)
                rp[h.up_ids[l][j] + 1] = h.up_rp[l][j + 1] - h.up_rp[l][j];
            for (int64_t i = 0; i < n; ++i) rp[i + 1] += rp[i];
            layer_dist(rp, h.up_col[l], dist[l]);
            up_full[l] = std::move(rp);
        }
        std::vector<float> vecs((size_t)n * d);
        if (n) ix->vecs.download(vecs.data(), n * d * 4);

        File gf(path_of(dir, basename, ".hnsw.graph"), "wb");
        File df(path_of(dir, basename, ".hnsw.data"), "wb");
        // Description (format 4, Full mode)
        gf.w<uint32_t>(MAGICDESCR_4);
        gf.w<uint8_t>(1);
        gf.w<uint8_t>((uint8_t)ix->cfg.m);
        gf.w<double>(1.0 / std::log((double)ix->cfg.m));  // LayerGenerator scale (hnsw.rs:336-356)
        gf.w<uint8_t>(NB_LAYER_MAX);
        gf.w<uint64_t>((uint64_t)ix->cfg.ef_construction);
        gf.w<uint64_t>((uint64_t)n);
        gf.w<uint64_t>((uint64_t)d);
        const std::string dn = dist_name(ix->cfg.metric), tn = "f32";
        gf.w<uint64_t>(dn.size());
        gf.put(dn.data(), dn.size());
        gf.w<uint64_t>(tn.size());
        gf.put(tn.data(), tn.size());
        df.w<uint32_t>(MAGICDATAP);
        df.w<uint64_t>((uint64_t)d);
        // PointIndexation
        gf.w<uint8_t>(NB_LAYER_MAX);
        auto put_id = [&](int64_t row) {
            gf.w<uint64_t>(ix->ids[row]);
            gf.w<uint8_t>((uint8_t)std::min<int>(h.levels[row], NB_LAYER_MAX - 1));
            gf.w<int32_t>(rank[row]);
        };
        for (int l = 0; l < NB_LAYER_MAX; ++l) {
            gf.w<uint32_t>(MAGICLAYER);
            gf.w<uint64_t>(by_level[l].size());
            for (int64_t row : by_level[l]) {
                gf.w<uint32_t>(MAGICPOINT);
                put_id(row);
                for (int ll = 0; ll < NB_LAYER_MAX; ++ll) {
                    int64_t b = 0, e = 0;
                    const int32_t* col = nullptr;
                    if (ll == 0) {
                        b = h.rp0[row]; e = h.rp0[row + 1]; col = h.col0.data();
                    } else if (ll <= h.max_level) {
                        b = up_full[ll][row]; e = up_full[ll][row + 1]; col = h.up_col[ll].data();
                    }
                    gf.w<uint64_t>((uint64_t)(e - b));
                    for (int64_t p = b; p < e; ++p) {
                        put_id(col[p]);
                        gf.w<float>(dist[ll][p]);
                    }
                }
                df.w<uint32_t>(MAGICDATAP);
                df.w<uint64_t>(ix->ids[row]);
                df.w<uint64_t>((uint64_t)d * 4);
                df.put(vecs.data() + (size_t)row * d, (size_t)d * 4);
            }
        }
        if (n) put_id(h.entry);
        gf.close();
        df.close();
    });
}

rvx_status rvx_index_file_load(const char* dir, const char* basename, int32_t metric, int32_t ef_search,
                               uint64_t seed, rvx_index** out) {
    return guard([&] {
        RVX_REQUIRE(basename && out, RVX_ERR_INVALID_PARAMETER, "null argument");
        File gf(path_of(dir, basename, ".hnsw.graph"), "rb");
        File df(path_of(dir, basename, ".hnsw.data"), "rb");
        rvx_hnswio_description ds;
        read_description(gf, &ds);
        RVX_REQUIRE(ds.dump_mode == 1, RVX_ERR_SERIALIZATION,
                    "only Full-mode dumps reload (hnswio.rs load_point_graph reads PointIds unconditionally)");
        RVX_REQUIRE(std::string(ds.t_name) == "f32", RVX_ERR_SERIALIZATION, "data type is not f32");
        RVX_REQUIRE(ds.format_version >= 3, RVX_ERR_UNSUPPORTED, "format 2 (bincode point data) is not supported");
        // description fields are untrusted: bound them before sizing anything by them
        RVX_REQUIRE(ds.dimension > 0 && ds.dimension <= ((int64_t)1 << 24) && ds.nb_layer >= 1 &&
                        ds.nb_layer <= NB_LAYER_MAX && ds.nb_point >= 0 && ds.nb_point <= ((int64_t)1 << 40),
                    RVX_ERR_SERIALIZATION, "bad description");
        if (metric < 0) metric = metric_of(ds.distname);
        RVX_REQUIRE(metric >= 0, RVX_ERR_INVALID_PARAMETER,
                    std::string("distance '") + ds.distname + "' does not name a metric; pass one");
        const int64_t d = ds.dimension;
        RVX_REQUIRE(df.r<uint32_t>() == MAGICDATAP, RVX_ERR_SERIALIZATION, "bad data file magic");
        RVX_REQUIRE((int64_t)df.r<uint64_t>() == d, RVX_ERR_SERIALIZATION, "data dimension != description");

        const int nl = gf.r<uint8_t>();
        RVX_REQUIRE(nl >= 1 && nl <= NB_LAYER_MAX, RVX_ERR_SERIALIZATION, "inconsistent number of layers");
        std::vector<int64_t> layer_off(NB_LAYER_MAX + 1, 0);
        std::vector<uint64_t> ids;
        std::vector<uint8_t> levels;
        std::vector<float> vecs;
        // per row and layer <= level: neighbour (layer, rank) and distance
        std::vector<std::vector<std::vector<Nb>>> nbs;
        for (int l = 0; l < nl; ++l) {
            RVX_REQUIRE(gf.r<uint32_t>() == MAGICLAYER, RVX_ERR_SERIALIZATION, "bad magic at layer beginning");
            const int64_t cnt = (int64_t)gf.r<uint64_t>();
            RVX_REQUIRE(cnt >= 0 && (int64_t)ids.size() + cnt <= ds.nb_point, RVX_ERR_SERIALIZATION,
                        "more points than described");
            layer_off[l] = (int64_t)ids.size();
            for (int64_t r = 0; r < cnt; ++r) {
                RVX_REQUIRE(gf.r<uint32_t>() == MAGICPOINT, RVX_ERR_SERIALIZATION, "bad magic at point beginning");
                const uint64_t origin = gf.r<uint64_t>();
                const int pl = gf.r<uint8_t>();
                const int32_t pr = gf.r<int32_t>();
                RVX_REQUIRE(pl == l && pr == r, RVX_ERR_SERIALIZATION, "point id out of layer/rank order");
                std::vector<std::vector<Nb>> lists(ds.nb_layer);
                for (int ll = 0; ll < ds.nb_layer; ++ll) {
                    const uint64_t k = gf.r<uint64_t>();
                    RVX_REQUIRE(k < ((uint64_t)1 << 31), RVX_ERR_SERIALIZATION, "neighbour count too large");
                    for (uint64_t j = 0; j < k; ++j) {
                        Nb nb;
                        nb.d_id = gf.r<uint64_t>();
                        nb.layer = gf.r<uint8_t>();
                        nb.rank = gf.r<int32_t>();
                        nb.dist = gf.r<float>();
                        lists[ll].push_back(nb);
                    }
                }
                nbs.push_back(std::move(lists));
                ids.push_back(origin);
                levels.push_back((uint8_t)l);
                RVX_REQUIRE(df.r<uint32_t>() == MAGICDATAP, RVX_ERR_SERIALIZATION, "bad magic in data file");
                RVX_REQUIRE(df.r<uint64_t>() == origin, RVX_ERR_SERIALIZATION, "origin_id incoherent between graph and data");
                RVX_REQUIRE(df.r<uint64_t>() == (uint64_t)d * 4, RVX_ERR_SERIALIZATION, "vector length != dimension");
                const size_t at = vecs.size();
                vecs.resize(at + (size_t)d);
                df.get(vecs.data() + at, (size_t)d * 4);
            }
        }
        for (int l = nl; l <= NB_LAYER_MAX; ++l) layer_off[l] = (int64_t)ids.size();
        const int64_t n = (int64_t)ids.size();
        RVX_REQUIRE(n == ds.nb_point, RVX_ERR_SERIALIZATION, "fewer points than described");
        auto row_of = [&](int layer, int32_t r) -> int64_t {
            RVX_REQUIRE(layer < nl && r >= 0 && r < layer_off[layer + 1] - layer_off[layer], RVX_ERR_SERIALIZATION,
                        "neighbour point id out of range");
            return layer_off[layer] + r;
        };

        HostGraph hg;
        hg.n = n;
        hg.levels = levels;
        hg.max_level = 0;
        for (int64_t i = 0; i < n; ++i) hg.max_level = std::max<int>(hg.max_level, levels[i]);
        hg.rp0.assign(n + 1, 0);
        for (int64_t i = 0; i < n; ++i) {
            for (const Nb& nb : nbs[i][0]) {
                hg.col0.push_back((int32_t)row_of(nb.layer, nb.rank));
                hg.dist0.push_back(nb.dist);
            }
            hg.rp0[i + 1] = (int64_t)hg.col0.size();
        }
        hg.up_ids.assign(hg.max_level + 1, {});
        hg.up_rp.assign(hg.max_level + 1, {});
        hg.up_col.assign(hg.max_level + 1, {});
        // layer l >= 1: every point holding a non-empty layer-l list, whatever
        // its level (layers above the entry's level are never searched)
        for (int l = 1; l <= hg.max_level; ++l) {
            hg.up_rp[l].push_back(0);
            for (int64_t i = 0; i < n; ++i) {
                if (l >= (int)nbs[i].size() || nbs[i][l].empty()) continue;
                hg.up_ids[l].push_back((int32_t)i);
                for (const Nb& nb : nbs[i][l]) hg.up_col[l].push_back((int32_t)row_of(nb.layer, nb.rank));
                hg.up_rp[l].push_back((int64_t)hg.up_col[l].size());
            }
        }
        nbs.clear();
        if (n) {
            const uint64_t e_origin = gf.r<uint64_t>();
            const int el = gf.r<uint8_t>();
            const int32_t er = gf.r<int32_t>();
            hg.entry = row_of(el, er);
            RVX_REQUIRE(ids[hg.entry] == e_origin, RVX_ERR_SERIALIZATION, "entry point id mismatch");
        }

        rvx_index_config cfg{};
        cfg.kind = RVX_INDEX_HNSW;
        cfg.dim = (int32_t)d;
        cfg.metric = metric;
        cfg.m = std::max(1, ds.max_nb_connection);
        cfg.ef_construction = (int32_t)std::max<int64_t>(1, ds.ef_construction);
        cfg.ef_search = ef_search > 0 ? ef_search : 100;
        cfg.max_elements = std::max<int64_t>(n, 1);
        cfg.seed = seed;
        rvx_index* raw = nullptr;
        if (rvx_index_create(&cfg, &raw) != RVX_OK) fail(RVX_ERR_INVALID_PARAMETER, "index configuration rejected");
        std::unique_ptr<rvx_index, rvx_status (*)(rvx_index*)> ix(raw, rvx_index_destroy);
        {
            std::unique_lock<std::shared_mutex> lk(ix->mu);
            ComputeLock cl;
            if (n) index_append_rows(ix.get(), vecs.data(), ids.data(), n, false);
            ix->build_valid = false;
            hnsw_install(ix.get(), std::move(hg));
        }
        *out = ix.release();
    });
}

}  // extern "C"
