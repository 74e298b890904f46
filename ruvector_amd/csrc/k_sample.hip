// k_sample.hip — GraphSAGE neighbour sampling as a sampled CSR.
//
// GraphSAGELayer::sample_neighbors (crates/ruvector-postgres/src/gnn/graphsage.rs:92-102)
// re-seeds `StdRng::seed_from_u64(42)` for every node and keeps
// `sampled[..k]` after `partial_shuffle(rng, k)`. The draw sequence therefore
// depends only on the list length L, so the kept positions are one table per
// distinct degree L > k. The host computes those tables (rand 0.8.5 /
// rand_chacha 0.3.1 / rand_core 0.6 restated below; not vendored under the
// reference, Cargo.lock:6952,6993), and one kernel pass writes the sampled CSR
// (row i keeps min(deg_i, k) ids, in the reference's kept order). The
// aggregate kernels then run unchanged over it, so every sum is the
// reference's sequential sum over the sampled list.
#include <algorithm>
#include <unordered_map>

#include "common.hpp"
#include "graph.hpp"

namespace rvx {
namespace {

// StdRng = ChaCha12Rng: 256-bit key = seed, 64-bit block counter from 0, zero
// nonce, next_u32 = keystream words in order.
struct StdRng {
    uint32_t key[8];
    uint64_t counter = 0;
    uint32_t buf[16];
    int idx = 16;

    static uint32_t rotl(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }
    void refill() {
        const uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                                key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                                (uint32_t)counter, (uint32_t)(counter >> 32), 0u, 0u};
        uint32_t x[16];
        for (int i = 0; i < 16; ++i) x[i] = s[i];
#define RVX_QR(a, b, c, d)                   \
    x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 16); \
    x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 12); \
    x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 8);  \
    x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 7);
        for (int r = 0; r < 6; ++r) {  // 12 rounds = 6 column + diagonal double rounds
            RVX_QR(0, 4, 8, 12) RVX_QR(1, 5, 9, 13) RVX_QR(2, 6, 10, 14) RVX_QR(3, 7, 11, 15)
            RVX_QR(0, 5, 10, 15) RVX_QR(1, 6, 11, 12) RVX_QR(2, 7, 8, 13) RVX_QR(3, 4, 9, 14)
        }
#undef RVX_QR
        for (int i = 0; i < 16; ++i) buf[i] = x[i] + s[i];
        ++counter;
        idx = 0;
    }
    uint32_t next_u32() {
        if (idx >= 16) refill();
        return buf[idx++];
    }
    // SeedableRng::seed_from_u64: eight PCG32 outputs form the 32-byte seed.
    explicit StdRng(uint64_t state) {
        for (int i = 0; i < 8; ++i) {
            state = state * 6364136223846793005ull + 11634580027462260723ull;
            const uint32_t xs = (uint32_t)(((state >> 18) ^ state) >> 27);
            const uint32_t rot = (uint32_t)(state >> 59);
            key[i] = (xs >> rot) | (xs << ((32u - rot) & 31u));
        }
    }
    // gen_index(ub) = gen_range(0..ub as u32): UniformInt::sample_single_inclusive
    // with the widening-multiply rejection zone (range << lzcnt(range)) - 1.
    uint32_t gen_index(uint32_t ub) {
        const uint32_t zone = (ub << __builtin_clz(ub)) - 1u;
        for (;;) {
            const uint64_t m = (uint64_t)next_u32() * ub;
            if ((uint32_t)m <= zone) return (uint32_t)(m >> 32);
        }
    }
};

// Kept positions for a list of length len > k: Durstenfeld swaps of
// partial_shuffle over the tail, then the prefix [0, k). Positions untouched
// by a swap keep their index, so a sparse map suffices (O(k) per length).
void sample_positions(int32_t len, int32_t k, int32_t* out) {
    StdRng rng(42);
    std::unordered_map<int32_t, int32_t> moved;
    auto at = [&](int32_t p) {
        auto it = moved.find(p);
        return it == moved.end() ? p : it->second;
    };
    for (int32_t i = len - 1; i >= len - k; --i) {
        const int32_t j = (int32_t)rng.gen_index((uint32_t)i + 1);
        const int32_t vi = at(i), vj = at(j);
        moved[i] = vj;
        moved[j] = vi;
    }
    for (int32_t t = 0; t < k; ++t) out[t] = at(t);
}

// One wave per row: copy min(deg, k) ids, through the row's position table
// when deg > k.
__global__ __launch_bounds__(256) void k_sample_csr(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                    int64_t n, int32_t k, const int32_t* __restrict__ table_off,
                                                    int32_t max_deg, const int32_t* __restrict__ table,
                                                    const int64_t* __restrict__ rp_s, int32_t* __restrict__ col_s) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    const int64_t beg = rp[row];
    const int32_t deg = (int32_t)(rp[row + 1] - beg);
    const int64_t out0 = rp_s[row];
    if (deg <= k) {
        for (int t = lane; t < deg; t += 64) col_s[out0 + t] = col[beg + t];
    } else {
        const int32_t* pos = table + (int64_t)table_off[deg - k - 1] * k;
        for (int t = lane; t < k; t += 64) col_s[out0 + t] = col[beg + pos[t]];
    }
    (void)max_deg;
}

}  // namespace

void sage_sample_positions(int32_t len, int32_t k, int32_t* out) { sample_positions(len, k, out); }

// The sampled CSR of g for num_samples = k (cached on the graph handle).
const rvx_graph* sampled_graph(const rvx_graph* g, int32_t k) {
    if (g->max_deg <= k) return g;
    std::lock_guard<std::mutex> lk(g->sampled_mu);
    auto& slot = g->sampled[k];
    if (slot) return slot.get();
    std::vector<int64_t> rp(g->n + 1);
    sync();
    RVX_HIP(hipMemcpy(rp.data(), g->row_ptr, (size_t)(g->n + 1) * 8, hipMemcpyDeviceToHost));
    // one position table per distinct degree above k
    std::vector<int32_t> off((size_t)(g->max_deg - k), -1);
    std::vector<int64_t> rp_s(g->n + 1, 0);
    int32_t tables = 0;
    for (int64_t i = 0; i < g->n; ++i) {
        const int64_t d = rp[i + 1] - rp[i];
        if (d > k && off[(size_t)(d - k - 1)] < 0) off[(size_t)(d - k - 1)] = tables++;
        rp_s[i + 1] = rp_s[i] + std::min<int64_t>(d, k);
    }
    std::vector<int32_t> table((size_t)tables * k);
    for (int32_t d = k + 1; d <= g->max_deg; ++d)
        if (off[(size_t)(d - k - 1)] >= 0) sample_positions(d, k, table.data() + (size_t)off[(size_t)(d - k - 1)] * k);
    auto s = std::make_unique<rvx_graph>();
    s->n = g->n;
    s->e = rp_s[g->n];
    s->max_deg = k;
    s->row_ptr_mem.reset((g->n + 1) * 8);
    s->row_ptr_mem.upload(rp_s.data(), (g->n + 1) * 8);
    s->row_ptr = s->row_ptr_mem.as<int64_t>();
    s->col_mem.reset(std::max<int64_t>(s->e, 1) * 4);
    s->col = s->col_mem.as<int32_t>();
    DevMem d_off((int64_t)off.size() * 4), d_table(std::max<int64_t>((int64_t)table.size(), 1) * 4);
    d_off.upload(off.data(), (int64_t)off.size() * 4);
    if (!table.empty()) d_table.upload(table.data(), (int64_t)table.size() * 4);
    const dim3 grid((unsigned)((g->n + 3) / 4)), block(256);
    RVX_LAUNCH("sage_sample_csr", k_sample_csr, grid, block, 0, g->row_ptr, g->col, g->n, k, d_off.as<int32_t>(),
               g->max_deg, d_table.as<int32_t>(), s->row_ptr, s->col_mem.as<int32_t>());
    sync();  // d_off / d_table are freed on return
    slot = std::move(s);
    return slot.get();
}

}  // namespace rvx
