// api_shard.cpp — the merge step of node-range-sharded index search across GPUs
// (SURVEY.md §8e option 2; ShardedHyperbolicHnsw::search, crates/ruvector-
// hyperbolic-hnsw/src/shard.rs:354-373): every rank's per-query top-k travels in
// one all-gather (RCCL over xGMI, or the host-staged transport) and every rank
// merges the world lists on the GPU.
#include "comm.hpp"
#include "graph.hpp"

using namespace rvx;

namespace {

// One hit as it travels between ranks (24 B): the reported distance and the merge key.
// The key orders real hits by distance (NaN as +inf) and every empty slot (gid -1) after
// every real hit, +inf and NaN hits included: the high word is 1 for an empty slot, the
// low word the order-preserving image of the distance. Every rank's list is ascending in
// that key, so each output slot is written exactly once and the first `count` slots are
// real hits.
struct Hit {
    int64_t gid;
    int64_t lid;
    float d;
    uint32_t key_lo;  // order-preserving bits of the distance (NaN -> +inf)
};

__device__ __forceinline__ uint64_t hit_key(const Hit& h) {
    return ((uint64_t)(h.gid == -1 ? 1u : 0u) << 32) | h.key_lo;
}

__global__ void k_pack_hits(const int64_t* gid, const int64_t* lid, const float* d, int64_t total, Hit* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    Hit h;
    h.gid = gid[i];
    h.lid = lid ? lid[i] : 0;
    h.d = h.gid == -1 ? INFINITY : d[i];
    const float kv = isnan(h.d) ? INFINITY : h.d;
    const uint32_t b = __float_as_uint(kv);
    h.key_lo = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    out[i] = h;
}

// count of entries of the ascending list l[0..k) with key' < v (strict) or key' <= v
__device__ __forceinline__ int count_before(const Hit* l, int k, uint64_t v, bool inclusive) {
    int lo = 0, hi = k;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const uint64_t x = hit_key(l[mid]);
        if (inclusive ? (x <= v) : (x < v)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Thread per (rank r, query q, slot j) of all[r][q][j]: its merged position is j
// plus, over every other rank's ascending list, the entries that order before it
// (ranks before r win distance ties). Positions < k are written; the (r 0, j 0)
// thread also writes the query's result count.
__global__ void k_merge_hits(const Hit* all, int w, int64_t nq, int k, int64_t* out_gid, int64_t* out_lid,
                             float* out_d, int32_t* out_n) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per_rank = nq * k;
    if (t >= per_rank * w) return;
    const int r = (int)(t / per_rank);
    const int64_t rem = t - (int64_t)r * per_rank;
    const int64_t q = rem / k;
    const int j = (int)(rem - q * k);
    const Hit h = all[t];
    int pos = j;
    for (int p = 0; p < w && pos < k; ++p) {
        if (p == r) continue;
        pos += count_before(all + (int64_t)p * per_rank + q * k, k, hit_key(h), p < r);
    }
    if (pos < k) {
        out_gid[q * k + pos] = h.gid;
        if (out_lid) out_lid[q * k + pos] = h.gid == -1 ? -1 : h.lid;
        out_d[q * k + pos] = h.d;
    }
    if (out_n && r == 0 && j == 0) {
        int64_t valid = 0;
        for (int p = 0; p < w; ++p) {
            const Hit* l = all + (int64_t)p * per_rank + q * k;
            for (int s = 0; s < k; ++s) valid += l[s].gid != -1;
        }
        out_n[q] = (int32_t)(valid < k ? valid : k);
    }
}

}  // namespace

namespace rvx {

void shard_agree(rvx_comm* c, rvx_status status, const std::string& why, const int64_t (&args)[5]) {
    const int w = comm_size(c), me = comm_rank(c);
    if (w <= 1 && !comm_self_p2p(c)) {
        if (status != RVX_OK) fail(status, why);
        return;
    }
    // fixed-size all-gather: {status, args...} per rank, so ranks that disagree on the
    // arguments (or failed before any collective) still exchange the same byte count
    constexpr int F = 8;
    ComputeLock cl;  // the scratch slot is only valid under the device's compute lock
    int64_t mine[F] = {(int64_t)status, args[0], args[1], args[2], args[3], args[4], 0, 0};
    auto* dev = (int64_t*)scratch_bytes("shard_agree", (int64_t)(w + 1) * F * 8);
    RVX_HIP(hipMemcpyAsync(dev, mine, sizeof mine, hipMemcpyHostToDevice, stream()));
    comm_allgather_bytes(c, dev, dev + F, F * 8, stream());
    std::vector<int64_t> all((size_t)w * F);
    RVX_HIP(hipMemcpyAsync(all.data(), dev + F, all.size() * 8, hipMemcpyDeviceToHost, stream()));
    sync();
    for (int p = 0; p < w; ++p)
        if (all[(size_t)p * F] != RVX_OK)
            fail((rvx_status)all[(size_t)p * F],
                 p == me ? why : "sharded search failed on rank " + std::to_string(p) + " (status " +
                                     std::to_string(all[(size_t)p * F]) + ")");
    for (int p = 1; p < w; ++p)
        for (int f = 1; f <= 5; ++f)
            RVX_REQUIRE(all[(size_t)p * F + f] == all[(size_t)f], RVX_ERR_INVALID_PARAMETER,
                        "sharded search arguments (nq, k, ef, mode, dim) differ between rank 0 and rank " +
                            std::to_string(p));
}

void sharded_merge(rvx_comm* c, const int64_t* gid, const int64_t* lid, const float* dist, int64_t nq, int k,
                   int64_t* out_gid, int64_t* out_lid, float* out_dist, int32_t* out_count) {
    if (nq <= 0) return;
    const int w = comm_size(c);
    const int64_t per_rank = nq * k;
    auto* mine = (Hit*)scratch_bytes("shard_hits", per_rank * (int64_t)sizeof(Hit));
    auto* all = (Hit*)scratch_bytes("shard_hits_all", per_rank * w * (int64_t)sizeof(Hit));
    {
        ProfScope ps("shard_pack");
        hipLaunchKernelGGL(k_pack_hits, dim3((unsigned)((per_rank + 255) / 256)), dim3(256), 0, stream(), gid, lid,
                           dist, per_rank, mine);
        RVX_HIP(hipGetLastError());
    }
    {
        ProfScope ps("shard_allgather");
        comm_allgather_bytes(c, mine, all, per_rank * (int64_t)sizeof(Hit), stream());
    }
    ProfScope ps("shard_merge");
    const int64_t threads = per_rank * w;
    hipLaunchKernelGGL(k_merge_hits, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, stream(), all, w, nq, k,
                       out_gid, out_lid, out_dist, out_count);
    RVX_HIP(hipGetLastError());
}

}  // namespace rvx
