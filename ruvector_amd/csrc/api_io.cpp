// api_io.cpp — node-feature files into / out of HBM, and stored rows back out
// of an index.
//
// Layouts of the reference's on-disk embedding tables:
//   RVX_FEATURE_RAW: MmapManager (crates/ruvector-gnn/src/mmap.rs:147-218) —
//     row i at byte i*dim*4, native f32, no header.
//   RVX_FEATURE_COLD_TIER: FeatureStorage (crates/ruvector-gnn/src/cold_tier.rs:
//     17-151) — 24-byte header {dim, num_nodes, block_size} (u64 LE), row i at
//     24 + i*block_size, block_size = dim*4 rounded up to the page size.
// Loads stream through two pinned staging buffers: pread of chunk c+1
// overlaps the DMA of chunk c; padded blocks are unpacked by a 2-D copy.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <string>

#include "common.hpp"
#include "gnn.hpp"
#include "graph.hpp"
#include "index.hpp"

namespace rvx {
namespace {

constexpr int64_t COLD_HEADER = 24;
constexpr int64_t STAGE_BYTES = 64ll << 20;

struct Fd {
    int fd = -1;
    std::string path;
    Fd(const char* p, int flags) : path(p) {
        fd = ::open(p, flags, 0644);
        RVX_REQUIRE(fd >= 0, RVX_ERR_SERIALIZATION, std::string("cannot open ") + p);
    }
    ~Fd() {
        if (fd >= 0) ::close(fd);
    }
    int64_t size() const {
        struct stat st;
        RVX_REQUIRE(::fstat(fd, &st) == 0, RVX_ERR_SERIALIZATION, "stat failed: " + path);
        return (int64_t)st.st_size;
    }
    void pread_all(void* dst, int64_t n, int64_t off) const {
        auto* p = static_cast<char*>(dst);
        while (n > 0) {
            const ssize_t r = ::pread(fd, p, (size_t)n, (off_t)off);
            RVX_REQUIRE(r > 0, RVX_ERR_SERIALIZATION, "short read: " + path);
            p += r; off += r; n -= r;
        }
    }
    void pwrite_all(const void* src, int64_t n, int64_t off) const {
        auto* p = static_cast<const char*>(src);
        while (n > 0) {
            const ssize_t r = ::pwrite(fd, p, (size_t)n, (off_t)off);
            RVX_REQUIRE(r > 0, RVX_ERR_SERIALIZATION, "short write: " + path);
            p += r; off += r; n -= r;
        }
    }
};

struct Layout {
    int64_t dim = 0, rows = 0, block = 0, base = 0;  // row i at base + i*block
};

Layout layout_of(const Fd& f, int32_t layout, int64_t dim) {
    Layout L;
    constexpr int64_t MAX_DIM = (int64_t)1 << 28, MAX_BLOCK = (int64_t)1 << 36;  // keep every product in int64
    if (layout == RVX_FEATURE_RAW) {
        RVX_REQUIRE(dim > 0 && dim <= MAX_DIM, RVX_ERR_INVALID_PARAMETER, "raw feature files need a dimension in [1, 2^28]");
        L.dim = dim;
        L.block = dim * 4;
        L.rows = f.size() / L.block;
    } else if (layout == RVX_FEATURE_COLD_TIER) {
        uint64_t h[3];
        RVX_REQUIRE(f.size() >= COLD_HEADER, RVX_ERR_SERIALIZATION, "file shorter than the cold-tier header");
        f.pread_all(h, COLD_HEADER, 0);  // little-endian host
        L.dim = (int64_t)h[0];
        L.rows = (int64_t)h[1];
        L.block = (int64_t)h[2];
        L.base = COLD_HEADER;
        // header fields are untrusted: bound them before any arithmetic on them
        RVX_REQUIRE(h[0] > 0 && h[0] <= (uint64_t)MAX_DIM && h[2] <= (uint64_t)MAX_BLOCK && h[1] <= (uint64_t)INT64_MAX,
                    RVX_ERR_SERIALIZATION, "bad cold-tier header");
        RVX_REQUIRE(L.block >= L.dim * 4, RVX_ERR_SERIALIZATION, "bad cold-tier header");
        RVX_REQUIRE(L.rows <= (f.size() - COLD_HEADER) / L.block, RVX_ERR_SERIALIZATION,
                    "cold-tier header claims more rows than the file holds");
        RVX_REQUIRE(dim <= 0 || dim == L.dim, RVX_ERR_DIMENSION_MISMATCH, "dimension differs from the file header");
    } else {
        fail(RVX_ERR_INVALID_PARAMETER, "unknown feature-file layout");
    }
    return L;
}

struct Pinned {
    void* p = nullptr;
    explicit Pinned(int64_t b) { RVX_HIP(hipHostMalloc(&p, (size_t)b, hipHostMallocDefault)); }
    ~Pinned() {
        if (p) (void)hipHostFree(p);
    }
};

}  // namespace
}  // namespace rvx

using namespace rvx;

extern "C" {

rvx_status rvx_feature_file_info(const char* path, int32_t layout, int64_t dim, int64_t* rows, int64_t* dim_out,
                                 int64_t* block_size) {
    return guard([&] {
        RVX_REQUIRE(path, RVX_ERR_INVALID_PARAMETER, "null path");
        Fd f(path, O_RDONLY);
        const Layout L = layout_of(f, layout, dim);
        if (rows) *rows = L.rows;
        if (dim_out) *dim_out = L.dim;
        if (block_size) *block_size = L.block;
    });
}

rvx_status rvx_feature_file_load(const char* path, int32_t layout, int64_t dim, int64_t row0, int64_t nrows,
                                 rvx_buffer* dst, int64_t dst_row0) {
    return guard([&] {
        RVX_REQUIRE(path && dst && row0 >= 0 && nrows >= 0 && dst_row0 >= 0, RVX_ERR_INVALID_PARAMETER, "bad argument");
        Fd f(path, O_RDONLY);
        const Layout L = layout_of(f, layout, dim);
        RVX_REQUIRE(row0 <= L.rows && nrows <= L.rows - row0, RVX_ERR_INDEX, "rows past the end of the file");
        const int64_t rb = L.dim * 4;
        RVX_REQUIRE(dst_row0 <= dst->mem.bytes / rb && nrows <= dst->mem.bytes / rb - dst_row0,
                    RVX_ERR_DIMENSION_MISMATCH, "buffer smaller than rows*dim");
        RVX_REQUIRE(f.size() >= L.base + (row0 + nrows - 1) * L.block + rb || nrows == 0, RVX_ERR_SERIALIZATION,
                    "file shorter than its rows");
        if (nrows == 0) return;
        const int64_t per = std::max<int64_t>(1, STAGE_BYTES / L.block);
        Pinned st0(per * L.block), st1(per * L.block);
        void* stage[2] = {st0.p, st1.p};
        hipEvent_t done[2];
        RVX_HIP(hipEventCreateWithFlags(&done[0], hipEventDisableTiming));
        RVX_HIP(hipEventCreateWithFlags(&done[1], hipEventDisableTiming));
        char* out = dst->mem.as<char>() + dst_row0 * rb;
        int s = 0;
        for (int64_t r = 0; r < nrows; r += per, s ^= 1) {
            const int64_t cnt = std::min(per, nrows - r);
            RVX_HIP(hipEventSynchronize(done[s]));  // the copy that last used this stage is finished
            // the last block of a cold-tier file may stop at the row's end
            const int64_t bytes = (cnt - 1) * L.block + rb;
            f.pread_all(stage[s], bytes, L.base + (row0 + r) * L.block);
            if (L.block == rb)
                RVX_HIP(hipMemcpyAsync(out + r * rb, stage[s], (size_t)bytes, hipMemcpyHostToDevice, stream()));
            else
                RVX_HIP(hipMemcpy2DAsync(out + r * rb, (size_t)rb, stage[s], (size_t)L.block, (size_t)rb, (size_t)cnt,
                                         hipMemcpyHostToDevice, stream()));
            RVX_HIP(hipEventRecord(done[s], stream()));
        }
        rvx::sync();
        (void)hipEventDestroy(done[0]);
        (void)hipEventDestroy(done[1]);
    });
}

rvx_status rvx_feature_file_store(const char* path, int32_t layout, const rvx_buffer* src, int64_t dim, int64_t nrows,
                                  int64_t block_size) {
    return guard([&] {
        RVX_REQUIRE(path && src && dim > 0 && nrows >= 0, RVX_ERR_INVALID_PARAMETER, "bad argument");
        const int64_t rb = dim * 4;
        RVX_REQUIRE(nrows * rb <= src->mem.bytes, RVX_ERR_DIMENSION_MISMATCH, "buffer smaller than rows*dim");
        RVX_REQUIRE(layout == RVX_FEATURE_RAW || layout == RVX_FEATURE_COLD_TIER, RVX_ERR_INVALID_PARAMETER,
                    "unknown feature-file layout");
        int64_t block = rb, base = 0;
        if (layout == RVX_FEATURE_COLD_TIER) {
            // FeatureStorage::create: block = align_up(dim*4, page size) (cold_tier.rs:45-66)
            const int64_t page = block_size > 0 ? block_size : (int64_t)::sysconf(_SC_PAGESIZE);
            block = (rb + page - 1) / page * page;
            base = COLD_HEADER;
        }
        Fd f(path, O_WRONLY | O_CREAT | O_TRUNC);
        if (layout == RVX_FEATURE_COLD_TIER) {
            const uint64_t h[3] = {(uint64_t)dim, (uint64_t)nrows, (uint64_t)block};
            f.pwrite_all(h, COLD_HEADER, 0);
        }
        RVX_REQUIRE(::ftruncate(f.fd, (off_t)(base + nrows * block)) == 0, RVX_ERR_SERIALIZATION, "cannot size file");
        if (nrows == 0) return;
        const int64_t per = std::max<int64_t>(1, STAGE_BYTES / block);
        Pinned st(per * block);
        std::memset(st.p, 0, (size_t)(per * block));
        const char* in = src->mem.as<char>();
        for (int64_t r = 0; r < nrows; r += per) {
            const int64_t cnt = std::min(per, nrows - r);
            if (block == rb)
                RVX_HIP(hipMemcpyAsync(st.p, in + r * rb, (size_t)(cnt * rb), hipMemcpyDeviceToHost, stream()));
            else
                RVX_HIP(hipMemcpy2DAsync(st.p, (size_t)block, in + r * rb, (size_t)rb, (size_t)rb, (size_t)cnt,
                                         hipMemcpyDeviceToHost, stream()));
            rvx::sync();
            f.pwrite_all(st.p, (cnt - 1) * block + rb, base + r * block);
        }
    });
}

rvx_status rvx_index_export_rows(const rvx_index* ix, int64_t row0, int64_t count, float* vecs, uint64_t* ids,
                                 uint8_t* deleted, int64_t* total_rows) {
    return guard([&] {
        RVX_REQUIRE(ix && row0 >= 0 && count >= 0, RVX_ERR_INVALID_PARAMETER, "bad argument");
        std::shared_lock<std::shared_mutex> lk(ix->mu);
        if (total_rows) *total_rows = ix->n;
        RVX_REQUIRE(row0 + count <= ix->n, RVX_ERR_INDEX, "rows past the end of the index");
        if (count == 0) return;
        const int64_t d = ix->cfg.dim;
        if (vecs) ix->vecs.download(vecs, count * d * 4, row0 * d * 4);
        if (ids) std::copy(ix->ids.begin() + row0, ix->ids.begin() + row0 + count, ids);
        if (deleted) std::copy(ix->deleted_h.begin() + row0, ix->deleted_h.begin() + row0 + count, deleted);
    });
}

rvx_status rvx_buffer_gather_rows_f32(const rvx_buffer* table, int64_t rows, int32_t dim, const int64_t* ids,
                                     int64_t n, float* out) {
    return guard([&] {
        RVX_REQUIRE(table && dim > 0 && rows >= 0 && n >= 0 && (n == 0 || (ids && out)), RVX_ERR_INVALID_PARAMETER,
                    "bad arguments");
        RVX_REQUIRE(table->mem.bytes >= rows * (int64_t)dim * 4, RVX_ERR_DIMENSION_MISMATCH,
                    "table smaller than rows*dim");
        for (int64_t i = 0; i < n; ++i)
            RVX_REQUIRE(ids[i] >= 0 && ids[i] < rows, RVX_ERR_INDEX, "row id out of range");
        ComputeLock cl;
        const int64_t step = std::max<int64_t>(1, std::min<int64_t>(n, ((int64_t)256 << 20) / ((int64_t)dim * 4)));
        auto* dids = (int64_t*)scratch_bytes("gather_ids", step * 8);
        float* dst = scratch_f32("gather_rows", step * dim);
        for (int64_t r0 = 0; r0 < n; r0 += step) {
            const int64_t m = std::min(step, n - r0);
            RVX_HIP(hipMemcpyAsync(dids, ids + r0, (size_t)m * 8, hipMemcpyHostToDevice, stream()));
            star_gather(nullptr, 1, table->mem.as<float>(), rows, dids, (int)m, dim, dst);
            RVX_HIP(hipMemcpyAsync(out + r0 * dim, dst, (size_t)(m * dim * 4), hipMemcpyDeviceToHost, stream()));
            rvx::sync();
        }
    });
}

}  // extern "C"
