// gemm_f32.hip — FP32 MFMA GEMM for gfx950 with fused epilogues.
//
// The dense feature-times-weight contraction of every GNN layer on the path:
//   Linear::forward        y = W x + b      (crates/ruvector-gnn/src/layer.rs:37-41)
//   GraphSAGE linear_transform  x·W         (crates/ruvector-postgres/src/gnn/graphsage.rs:105-115)
//   GCN linear_transform   x·W + b          (crates/ruvector-postgres/src/gnn/gcn.rs:64-81)
// batched over all nodes of the graph: C[M][N] = A[M][K] · B[N][K]^T (+ A1·B1^T).
// Both operands are K-contiguous ("NT"), which is the ndarray [out][in] weight
// layout of Linear; GraphSAGE/GCN [in][out] weights are transposed once at upload.
//
// Numerics: v_mfma_f32_32x32x2_f32 is an exact f32 fma chain (one rounding per
// product, cdna_hip_programming.md §3), so results differ from the reference's
// mul-then-add order only by rounding; parity is 1e-5 relative (north star).
//
// Tiling (CDNA4): 128x128 block tile, BK=32, 256 threads = 4 waves in a 2x2 grid,
// each wave a 64x64 tile of 2x2 MFMA 32x32 accumulators (64 AGPR/VGPR).
// Operands are staged through LDS with a +4-float row pad (144-B stride), which
// makes the per-lane ds_read_b128 fragment reads bank-conflict free. The K axis
// is permuted inside a BK tile so every lane reads 16 contiguous k values
// (lane half h owns k = 16h..16h+15); A and B use the same permutation, so the
// product is unchanged. Double-buffered LDS, one barrier per K tile, register
// prefetch of tile k+1 during the MFMAs of tile k, XCD-aware block swizzle so
// the column tiles of one row block share an XCD's L2.
#include <cstdio>
#include "common.hpp"
#include "graph.hpp"
#include "kernels.hpp"
#include "agg_row.hpp"
#include "gnn.hpp"

namespace rvx {

namespace {

constexpr int BM = 128, BN = 128, BK = 32, LDS_ROW = BK + 4;  // 36 floats = 144 B
constexpr int TILE_FLOATS = 128 * LDS_ROW;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct GemmArgs {
    const float* A0; const float* B0; int64_t lda0, ldb0; int K0;
    const float* A1; const float* B1; int64_t lda1, ldb1; int K1;
    const uint16_t* B0x3; const uint16_t* B1x3; int64_t B0x3_plane, B1x3_plane;  // split-bf16 weight planes
    const float* bias0; const float* bias1;
    const float* addend; int64_t ld_add;
    float* C; int64_t ldc;
    int64_t M; int N;
    int tiles_n; int64_t nblocks;
    float alpha;  // scale applied to acc before bias (dropout scale etc.)
    // split-f16 path (gemm_nt_h2g): per-row power-of-2 scale of A, per-column
    // inverse scale of B, and the two f16 planes of each B
    const float* a_scale; const float* b_inv;
    const _Float16* B0h; const _Float16* B1h; int64_t B0h_plane, B1h_plane;
    // pre-split A (gemm_nt_h2p): f16 planes [2][M][lda] written by the producer
    const _Float16* A0h; const _Float16* A1h; int64_t Ah_plane;
    // persistent split-f16 GEMM: per-XCD tile counters (stride 32 words), zeroed per launch
    unsigned* queue;
    int xsplit;  // queue mode: XCD pair (2i, 2i+1) shares a row range, each XCD takes half the column tiles
    // in-launch row normalisation (h2g): one arrival ticket per 128-row tile, zeroed per launch
    unsigned* row_tickets;
    // deferred normalisation (h2g): per-row partial sums of squares per column tile, and the
    // phase-1 operand's per-row multiplier
    float* row_sumsq; const float* a1_rowmul;
    // per-row max |v| per column tile for the next GEMM's row scale (h2g, h2w with WN = 1)
    float* row_absmax;
    // gemm_nt_h2w<..., HELP>: the next row chunk's gather, helped once the tiles run out
    AggHelp help;
    // AMX tiles: the gate columns (GemmEpilogue::gate_*)
    const float* gate_h; int64_t ld_gate_h; float* gate_out; int64_t ld_gate_out; int gate_col0;
};

// One row's max |v| over this column tile: lanes lr = 0..31 of a half-wave hold the row's
// columns; lane 0 writes slot tn, and the last column tile zeroes the slots past the tile
// count so a consumer reduces all ROWSUMSQ_SLOTS. fmaxf ignores NaN as k_row_scale_h2 does,
// and max is order-free, so the scale equals the one a pass over C computes.
__device__ __forceinline__ void row_absmax_store(const GemmArgs& g, int64_t row, int tn, int lr, float amx) {
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) amx = fmaxf(amx, __shfl_xor(amx, off));
    if (lr == 0 && row < g.M) {
        float* p = g.row_absmax + row * ROWSUMSQ_SLOTS;
        p[tn] = amx;
        if (tn == g.tiles_n - 1)
            for (int t = tn + 1; t < ROWSUMSQ_SLOTS; ++t) p[t] = 0.0f;
    }
}

__device__ __forceinline__ float epi_apply(int epi, float v) {
    if (epi == GEMM_EPI_RELU) return fmaxf(v, 0.0f);
    if (epi == GEMM_EPI_SIGMOID) {  // GRUCell::sigmoid, layer.rs:278-285
        if (v > 0.0f) return 1.0f / (1.0f + expf(-v));
        float ex = expf(v);
        return ex / (1.0f + ex);
    }
    if (epi == GEMM_EPI_TANH) return tanhf(v);
    return v;
}

template <bool DUAL, int DEPTH>
__global__ __launch_bounds__(256, 2) void gemm_nt_mfma(GemmArgs g, int epi) {
    __shared__ __attribute__((aligned(16))) float smem[2 * 2 * TILE_FLOATS];  // [stage][A|B]

    // XCD-aware bijective swizzle (cdna_hip_programming.md §5, T1): blocks b and
    // b+8 share an XCD; give each XCD a contiguous run of logical tiles so the
    // tiles_n column tiles of one row block hit the same L2.
    const int64_t nwg = g.nblocks;
    const int64_t bid = blockIdx.x;
    const int64_t xcd = bid % 8, q = nwg / 8, r = nwg % 8;
    const int64_t wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    const int64_t tm = wgid / g.tiles_n;
    const int tn = (int)(wgid % g.tiles_n);
    const int64_t m0 = tm * BM;
    const int n0 = tn * BN;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int lr = lane & 31, lh = lane >> 5;

    const int nk0 = (g.K0 + BK - 1) / BK;
    const int nk1 = DUAL ? (g.K1 + BK - 1) / BK : 0;
    const int nk = nk0 + nk1;

    // Global->register staging: 4 float4 of A and 4 of B per thread per K tile,
    // DEPTH register sets: tile kt+DEPTH is requested while tile kt is in the
    // MFMAs, so a load has DEPTH-1 full K tiles of compute (plus the current
    // one) to land — what keeps the GEMM fed when a concurrent gather has
    // HBM latency high.
    float4 ra[DEPTH][4], rb[DEPTH][4];
    auto load_tile = [&](int kt, float4 (&xa)[4], float4 (&xb)[4]) {
        const float* A; const float* B; int64_t lda, ldb; int K, k0;
        if (!DUAL || kt < nk0) { A = g.A0; B = g.B0; lda = g.lda0; ldb = g.ldb0; K = g.K0; k0 = kt * BK; }
        else { A = g.A1; B = g.B1; lda = g.lda1; ldb = g.ldb1; K = g.K1; k0 = (kt - nk0) * BK; }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int f = tid + 256 * i;
            const int row = f >> 3, c = (f & 7) * 4;
            const int k = k0 + c;
            const int64_t am = m0 + row;
            const int bn = n0 + row;
            float4 za = make_float4(0.f, 0.f, 0.f, 0.f), zb = za;
            if (am < g.M && k < K) za = *reinterpret_cast<const float4*>(A + am * lda + k);
            if (bn < g.N && k < K) zb = *reinterpret_cast<const float4*>(B + (int64_t)bn * ldb + k);
            xa[i] = za; xb[i] = zb;
        }
    };
    auto store_tile = [&](int stage, const float4 (&xa)[4], const float4 (&xb)[4]) {
        float* As = smem + stage * 2 * TILE_FLOATS;
        float* Bs = As + TILE_FLOATS;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int f = tid + 256 * i;
            const int row = f >> 3, c = (f & 7) * 4;
            *reinterpret_cast<float4*>(As + row * LDS_ROW + c) = xa[i];
            *reinterpret_cast<float4*>(Bs + row * LDS_ROW + c) = xb[i];
        }
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

    auto compute = [&](int stage) {
        const float* As = smem + stage * 2 * TILE_FLOATS;
        const float* Bs = As + TILE_FLOATS;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            float4 af[2][2], bf[2][2];
#pragma unroll
            for (int mi = 0; mi < 2; ++mi) {
                const float* p = As + (wm * 64 + mi * 32 + lr) * LDS_ROW + lh * 16 + half * 8;
                af[mi][0] = *reinterpret_cast<const float4*>(p);
                af[mi][1] = *reinterpret_cast<const float4*>(p + 4);
            }
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
                const float* p = Bs + (wn * 64 + ni * 32 + lr) * LDS_ROW + lh * 16 + half * 8;
                bf[ni][0] = *reinterpret_cast<const float4*>(p);
                bf[ni][1] = *reinterpret_cast<const float4*>(p + 4);
            }
#pragma unroll
            for (int s = 0; s < 8; ++s) {
#pragma unroll
                for (int mi = 0; mi < 2; ++mi) {
                    const float a = (s < 4) ? af[mi][0][s & 3] : af[mi][1][s & 3];
#pragma unroll
                    for (int ni = 0; ni < 2; ++ni) {
                        const float b = (s < 4) ? bf[ni][0][s & 3] : bf[ni][1][s & 3];
                        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[mi][ni], 0, 0, 0);
                    }
                }
            }
        }
    };

    if (DEPTH == 1) {
        load_tile(0, ra[0], rb[0]);
        store_tile(0, ra[0], rb[0]);
        __syncthreads();
        for (int kt = 0; kt < nk; ++kt) {
            const int stage = kt & 1;
            if (kt + 1 < nk) load_tile(kt + 1, ra[0], rb[0]);
            compute(stage);
            if (kt + 1 < nk) store_tile(stage ^ 1, ra[0], rb[0]);
            __syncthreads();
        }
    } else {
        // two register sets, loop unrolled by two so the set index is static
        load_tile(0, ra[0], rb[0]);
        store_tile(0, ra[0], rb[0]);
        if (nk > 1) load_tile(1, ra[1 % DEPTH], rb[1 % DEPTH]);
        __syncthreads();
        for (int kt = 0; kt < nk; kt += 2) {
            // even tile kt: compute stage 0; request tile kt+2 into set 0; publish tile kt+1 (set 1)
            if (kt + 2 < nk) load_tile(kt + 2, ra[0], rb[0]);
            compute(0);
            if (kt + 1 < nk) store_tile(1, ra[1 % DEPTH], rb[1 % DEPTH]);
            __syncthreads();
            if (kt + 1 >= nk) break;
            // odd tile kt+1: compute stage 1; request tile kt+3 into set 1; publish tile kt+2 (set 0)
            if (kt + 3 < nk) load_tile(kt + 3, ra[1 % DEPTH], rb[1 % DEPTH]);
            compute(1);
            if (kt + 2 < nk) store_tile(0, ra[0], rb[0]);
            __syncthreads();
        }
    }

    // Epilogue. 32x32 C/D map: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5).
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
            const int col = n0 + wn * 64 + ni * 32 + lr;
            if (col >= g.N) continue;
            float b = 0.0f;
            if (g.bias0) b = g.bias0[col];
            if (g.bias1) b += g.bias1[col];
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int64_t row = m0 + wm * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
                if (row < g.M) {
                    float v = acc[mi][ni][e];
                    if (g.alpha != 1.0f) v *= g.alpha;
                    if (g.bias0 || g.bias1) v += b;
                    if (g.addend) v += g.addend[row * g.ld_add + col];
                    g.C[row * g.ldc + col] = epi_apply(epi, v);
                }
            }
        }
    }
}


// ---------------------------------------------------------------------------
// Split-bf16 MFMA GEMM ("x3"). Every f32 operand is split exactly into three
// bf16 parts, a = a1 + a2 + a3 (truncation: a1 keeps the top 8 significand
// bits, a2 the next 8 of the exact remainder, a3 the rest; the sum is exact),
// and the six partial products whose weight is >= 2^-16 —
// a1b1, a1b2, a2b1, a1b3, a3b1, a2b2 — run on v_mfma_f32_32x32x16_bf16 with
// f32 accumulation. Each bf16 x bf16 product is exact in f32; the dropped
// terms (a2b3, a3b2, a3b3) are below 2^-23 |a b|, i.e. f32 rounding level, so
// the result is an f32 GEMM to within reordering error, at 6/16 of the
// FP32-MFMA cycle cost (bf16 MFMA is 16x the f32 rate on gfx950).
//
// Tile 128x128x32, 256 threads = 4 waves as 2(M) x 2(N), each wave 64x64 =
// 2x2 32x32 accumulators, two blocks per CU (8 waves). A is staged as f32
// and split into its three bf16 parts per fragment read (VALU work that
// issues in the MFMAs' shadow); B comes pre-split from HBM (weights are split
// once at upload). No row padding: 16-B chunks are XOR-swizzled so the
// per-lane 16-B fragment reads of 16 consecutive rows hit 16 distinct bank
// groups (A rows 128 B: chunk ^ (row>>1)&7; B plane rows 64 B: chunk ^
// (row>>2)&3). Double-buffered, 2 x 40 KB, register prefetch of tile k+1.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int XBM = 128, XBN = 128;
constexpr int XA_TILE = XBM * 128;                  // f32 A tile bytes
constexpr int XB_PLANE = XBN * 64;                  // one bf16 B plane tile bytes
constexpr int X_STAGE = XA_TILE + 3 * XB_PLANE;     // 40,960 B
constexpr int X_LDS = 2 * X_STAGE;                  // 81,920 B -> 2 blocks / CU

__device__ __forceinline__ int xa_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
__device__ __forceinline__ int xb_off(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4); }

// exact three-way bf16 split of 8 floats into packed bf16x8 parts
__device__ __forceinline__ void split8(const float4& lo, const float4& hi, bf16x8& p1, bf16x8& p2, bf16x8& p3) {
    const float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    u32x4 w1, w2, w3;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float a0 = v[2 * j], a1 = v[2 * j + 1];
        const unsigned h0 = __float_as_uint(a0) & 0xFFFF0000u, h1 = __float_as_uint(a1) & 0xFFFF0000u;
        const float r0 = a0 - __uint_as_float(h0), r1 = a1 - __uint_as_float(h1);
        const unsigned m0 = __float_as_uint(r0) & 0xFFFF0000u, m1 = __float_as_uint(r1) & 0xFFFF0000u;
        // the remainder r - m has at most 8 significant bits: its top half is exact
        const unsigned l0 = __float_as_uint(r0 - __uint_as_float(m0)), l1 = __float_as_uint(r1 - __uint_as_float(m1));
        w1[j] = __builtin_amdgcn_perm(h1, h0, 0x07060302u);
        w2[j] = __builtin_amdgcn_perm(m1, m0, 0x07060302u);
        w3[j] = __builtin_amdgcn_perm(l1, l0, 0x07060302u);
    }
    p1 = __builtin_bit_cast(bf16x8, w1);
    p2 = __builtin_bit_cast(bf16x8, w2);
    p3 = __builtin_bit_cast(bf16x8, w3);
}

// One packed pair (two k-adjacent values) of split8: words of planes 1..3.
__device__ __forceinline__ void split_pair(float a0, float a1, unsigned& w1, unsigned& w2, unsigned& w3) {
    const unsigned h0 = __float_as_uint(a0) & 0xFFFF0000u, h1 = __float_as_uint(a1) & 0xFFFF0000u;
    const float r0 = a0 - __uint_as_float(h0), r1 = a1 - __uint_as_float(h1);
    const unsigned m0 = __float_as_uint(r0) & 0xFFFF0000u, m1 = __float_as_uint(r1) & 0xFFFF0000u;
    const unsigned l0 = __float_as_uint(r0 - __uint_as_float(m0)), l1 = __float_as_uint(r1 - __uint_as_float(m1));
    w1 = __builtin_amdgcn_perm(h1, h0, 0x07060302u);
    w2 = __builtin_amdgcn_perm(m1, m0, 0x07060302u);
    w3 = __builtin_amdgcn_perm(l1, l0, 0x07060302u);
}

__device__ __forceinline__ float f4_at(const float4& lo, const float4& hi, int i) {
    switch (i) {
        case 0: return lo.x; case 1: return lo.y; case 2: return lo.z; case 3: return lo.w;
        case 4: return hi.x; case 5: return hi.y; case 6: return hi.z; default: return hi.w;
    }
}

template <bool DUAL>
__global__ __launch_bounds__(256, 2) void gemm_nt_x3(GemmArgs g, int epi) {
    extern __shared__ __attribute__((aligned(16))) unsigned char xsm[];

    const int64_t nwg = g.nblocks;
    const int64_t bid = blockIdx.x;
    const int64_t xcd = bid % 8, q = nwg / 8, r = nwg % 8;
    const int64_t wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    const int64_t tm = wgid / g.tiles_n;
    const int tn = (int)(wgid % g.tiles_n);
    const int64_t m0 = tm * XBM;
    const int n0 = tn * XBN;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int lr = lane & 31, lh = lane >> 5;

    const int nk0 = (g.K0 + 31) / 32;
    const int nk1 = DUAL ? (g.K1 + 31) / 32 : 0;
    const int nk = nk0 + nk1;

    float4 ra[4];
    u32x4 rb[3][2];
    auto load_tile = [&](int kt) {
        const float* A; const uint16_t* B; int64_t lda, ldb, bpl; int K, k0;
        if (!DUAL || kt < nk0) { A = g.A0; B = g.B0x3; lda = g.lda0; ldb = g.ldb0; bpl = g.B0x3_plane; K = g.K0; k0 = kt * 32; }
        else { A = g.A1; B = g.B1x3; lda = g.lda1; ldb = g.ldb1; bpl = g.B1x3_plane; K = g.K1; k0 = (kt - nk0) * 32; }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int f = tid + 256 * i;
            const int row = f >> 3, k = k0 + (f & 7) * 4;
            const int64_t am = m0 + row;
            ra[i] = (am < g.M && k < K) ? *reinterpret_cast<const float4*>(A + am * lda + k) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int f = tid + 256 * i;
            const int brow = f >> 2, bk = k0 + (f & 3) * 8;
            const bool bin = (n0 + brow < g.N) && (bk < K);
#pragma unroll
            for (int p = 0; p < 3; ++p)
                rb[p][i] = bin ? *reinterpret_cast<const u32x4*>(B + p * bpl + (int64_t)(n0 + brow) * ldb + bk)
                               : u32x4{0, 0, 0, 0};
        }
    };
    auto store_tile = [&](int stage) {
        unsigned char* base = xsm + stage * X_STAGE;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int f = tid + 256 * i;
            *reinterpret_cast<float4*>(base + xa_off(f >> 3, f & 7)) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int f = tid + 256 * i;
#pragma unroll
            for (int p = 0; p < 3; ++p)
                *reinterpret_cast<u32x4*>(base + XA_TILE + p * XB_PLANE + xb_off(f >> 2, f & 3)) = rb[p][i];
        }
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int stage = kt & 1;
        if (kt + 1 < nk) load_tile(kt + 1);
        const unsigned char* base = xsm + stage * X_STAGE;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            bf16x8 af[2][3], bf[2][3];
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
                const int off = xb_off(wn * 64 + ni * 32 + lr, 2 * s + lh);
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    bf[ni][p] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(base + XA_TILE + p * XB_PLANE + off));
            }
#pragma unroll
            for (int mi = 0; mi < 2; ++mi) {
                const int row = wm * 64 + mi * 32 + lr;
                const int c = 4 * s + 2 * lh;  // k = 16s + 8lh .. +7 = chunks c, c+1
                const float4 lo = *reinterpret_cast<const float4*>(base + xa_off(row, c));
                const float4 hi = *reinterpret_cast<const float4*>(base + xa_off(row, c + 1));
                split8(lo, hi, af[mi][0], af[mi][1], af[mi][2]);
            }
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int ni = 0; ni < 2; ++ni) {
                    f32x16 c = acc[mi][ni];
                    // small terms first
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi][1], bf[ni][1], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi][2], bf[ni][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi][0], bf[ni][2], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi][1], bf[ni][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi][0], bf[ni][1], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi][0], bf[ni][0], c, 0, 0, 0);
                    acc[mi][ni] = c;
                }
        }
        if (kt + 1 < nk) store_tile(stage ^ 1);
        __syncthreads();
    }

#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
            const int col = n0 + wn * 64 + ni * 32 + lr;
            if (col >= g.N) continue;
            float b = 0.0f;
            if (g.bias0) b = g.bias0[col];
            if (g.bias1) b += g.bias1[col];
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int64_t row = m0 + wm * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
                if (row < g.M) {
                    float v = acc[mi][ni][e];
                    if (g.alpha != 1.0f) v *= g.alpha;
                    if (g.bias0 || g.bias1) v += b;
                    if (g.addend) v += g.addend[row * g.ld_add + col];
                    g.C[row * g.ldc + col] = epi_apply(epi, v);
                }
            }
        }
    }
}

// Same tile and MFMA schedule as gemm_nt_x3, but the stage fill is LDS-DMA
// (global_load_lds_dwordx4): no register staging and no ds_write pass. One
// wave-instruction writes 1 KiB lane-linear, so the XOR swizzle goes on the
// per-lane SOURCE address: LDS slot p of row r receives global chunk
// p ^ swz(r). Waves are 4(M) x 1(N) — each owns 32 rows x all 128 columns —
// so every A fragment is split by exactly one wave. Requires K % 32 == 0 (no
// tail tile: the DMA has no zero fill); rows past M / N are clamped to a
// valid row and never stored.
template <bool DUAL, int WM, bool S16>
__global__ __launch_bounds__(64 * WM, WM == 4 ? 2 : 1) void gemm_nt_x3g(GemmArgs g, int epi) {
    constexpr int BM = 32 * WM;               // rows per block: one 32-row strip per wave
    constexpr int XA = BM * 128;              // f32 A tile bytes per stage
    constexpr int STG = XA + 3 * XB_PLANE;    // stage bytes
    constexpr int NB = 24 / WM;               // B DMA pieces per wave (3 planes x 8 pieces)
    extern __shared__ __attribute__((aligned(16))) unsigned char xsm[];

    const int64_t nwg = g.nblocks;
    const int64_t bid = blockIdx.x;
    const int64_t xcd = bid % 8, q = nwg / 8, r = nwg % 8;
    const int64_t wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    const int64_t tm = wgid / g.tiles_n;
    const int tn = (int)(wgid % g.tiles_n);
    const int64_t m0 = tm * BM;
    const int n0 = tn * XBN;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: LDS DMA targets go to M0 directly
    const int lr = lane & 31, lh = lane >> 5;

    const int nk0 = g.K0 / 32;
    const int nk1 = DUAL ? g.K1 / 32 : 0;

    // LDS XOR swizzles (16-B chunk ^ f(row)), conflict-free for the fragment
    // reads of each MFMA shape (checked against the ds_read_b128 lane groups)
    auto sw_a = [](int row) { return S16 ? (row >> 1) & 5 : (row >> 1) & 7; };
    auto sw_b = [](int row) { return S16 ? (4 - (row >> 2)) & 3 : (row >> 2) & 3; };

    // DMA sources: a scalar tile base (advanced 128 B / 64 B per k-tile) plus a
    // per-lane 32-bit byte offset fixed over k (host guarantees it fits), so the
    // k-loop carries no 64-bit address arithmetic.
    // A: pieces 4*wave .. 4*wave+3, each 8 rows x 8 chunks of 16 B
    // B: pieces NB*wave .. NB*wave+NB-1 over 3 planes x 8 pieces, each 16 rows x 4 chunks
    uint32_t a_off[2][4], b_off[2][NB];
    const char* a_base[2];
    const char* b_base[2];
#pragma unroll
    for (int ph = 0; ph < (DUAL ? 2 : 1); ++ph) {
        const float* A = ph ? g.A1 : g.A0;
        const uint16_t* B = ph ? g.B1x3 : g.B0x3;
        const int64_t lda = ph ? g.lda1 : g.lda0, ldb = ph ? g.ldb1 : g.ldb0, bpl = ph ? g.B1x3_plane : g.B0x3_plane;
        a_base[ph] = reinterpret_cast<const char*>(A + m0 * lda);
        b_base[ph] = reinterpret_cast<const char*>(B + (int64_t)n0 * ldb);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = 8 * (4 * wave + j) + (lane >> 3);
            const int chunk = (lane & 7) ^ sw_a(row);
            const int64_t r = std::min<int64_t>(m0 + row, g.M - 1) - m0;
            a_off[ph][j] = (uint32_t)((r * lda + 4 * chunk) * 4);
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const int piece = NB * wave + j;
            const int row = 16 * (piece & 7) + (lane >> 2);
            const int chunk = (lane & 3) ^ sw_b(row);
            const int64_t r = std::min<int64_t>(n0 + row, (int64_t)g.N - 1) - n0;
            b_off[ph][j] = (uint32_t)(((piece >> 3) * bpl + r * ldb + 8 * chunk) * 2);
        }
    }

    auto fill_ph = [&](int ph, int k0, unsigned char* base) {
        const char* ab = a_base[ph] + (int64_t)k0 * 4;
        const char* bb = b_base[ph] + (int64_t)k0 * 2;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            __builtin_amdgcn_global_load_lds((const void*)(ab + a_off[ph][j]),
                                             (__attribute__((address_space(3))) void*)(base + (4 * wave + j) * 1024),
                                             16, 0, 0);
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const int piece = NB * wave + j;
            __builtin_amdgcn_global_load_lds(
                (const void*)(bb + b_off[ph][j]),
                (__attribute__((address_space(3))) void*)(base + XA + (piece >> 3) * XB_PLANE + (piece & 7) * 1024),
                16, 0, 0);
        }
    };
    auto xa_sw = [&](int row, int chunk) { return row * 128 + ((chunk ^ sw_a(row)) << 4); };
    auto xb_sw = [&](int row, int chunk) { return row * 64 + ((chunk ^ sw_b(row)) << 4); };
    if constexpr (S16) {
    // 16x16x32 form: per k-tile each wave owns 2 (M) x 8 (N) 16x16 tiles; one
    // MFMA consumes the whole 32-deep k-tile, so both A row halves are split
    // up front and the eight column groups run 12 MFMAs each
    f32x4 acc[2][8];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const int l16 = lane & 15, lq = lane >> 4;
    int a_rd[2][2], b_rd[8];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
        a_rd[mi][0] = xa_sw(wave * 32 + 16 * mi + l16, 2 * lq);
        a_rd[mi][1] = xa_sw(wave * 32 + 16 * mi + l16, 2 * lq + 1);
    }
#pragma unroll
    for (int nj = 0; nj < 8; ++nj) b_rd[nj] = XA + xb_sw(16 * nj + l16, lq);

    auto tile = [&](const unsigned char* __restrict__ cur, unsigned char* __restrict__ nxt, int fph, int fk0) {
        if (fph == 0) fill_ph(0, fk0, nxt);
        else if (DUAL && fph == 1) fill_ph(1, fk0, nxt);
        bf16x8 af[2][3];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
            const float4 lo = *reinterpret_cast<const float4*>(cur + a_rd[mi][0]);
            const float4 hi = *reinterpret_cast<const float4*>(cur + a_rd[mi][1]);
            split8(lo, hi, af[mi][0], af[mi][1], af[mi][2]);
        }
        u32x4 bq[2][3];
#pragma unroll
        for (int p = 0; p < 3; ++p) bq[0][p] = *reinterpret_cast<const u32x4*>(cur + b_rd[0] + p * XB_PLANE);
#pragma unroll
        for (int nj = 0; nj < 8; ++nj) {
            if (nj + 1 < 8) {
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    bq[(nj + 1) & 1][p] = *reinterpret_cast<const u32x4*>(cur + b_rd[nj + 1] + p * XB_PLANE);
            }
            bf16x8 bf[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) bf[p] = __builtin_bit_cast(bf16x8, bq[nj & 1][p]);
#pragma unroll
            for (int mi = 0; mi < 2; ++mi) {
                f32x4 c = acc[mi][nj];
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi][1], bf[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi][2], bf[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi][0], bf[2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi][1], bf[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi][0], bf[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi][0], bf[0], c, 0, 0, 0);
                acc[mi][nj] = c;
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    // one k-loop per phase (compile-time ph: no per-tile operand selection);
    // the last tile of phase 0 prefetches the first tile of phase 1
    fill_ph(0, 0, xsm);
    __syncthreads();
    int stage = 0;
#pragma unroll
    for (int ph = 0; ph < (DUAL ? 2 : 1); ++ph) {
        const int nkp = ph ? nk1 : nk0;
        for (int kt = 0; kt < nkp; ++kt) {
            // the other stage was last read in the previous tile, before the barrier
            int fph = -1, fk0 = 0;
            if (kt + 1 < nkp) { fph = ph; fk0 = (kt + 1) * 32; }
            else if (DUAL && ph == 0 && nk1 > 0) fph = 1;
            tile(xsm + stage * STG, xsm + (stage ^ 1) * STG, fph, fk0);
            __syncthreads();  // retires the DMA of the next tile (vmcnt) for all waves
            stage ^= 1;
        }
    }

#pragma unroll
    for (int nj = 0; nj < 8; ++nj) {
        const int col = n0 + nj * 16 + l16;
        if (col >= g.N) continue;
        float b = 0.0f;
        if (g.bias0) b = g.bias0[col];
        if (g.bias1) b += g.bias1[col];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t row = m0 + wave * 32 + 16 * mi + 4 * lq + e;
                if (row < g.M) {
                    float v = acc[mi][nj][e];
                    if (g.alpha != 1.0f) v *= g.alpha;
                    if (g.bias0 || g.bias1) v += b;
                    if (g.addend) v += g.addend[row * g.ld_add + col];
                    g.C[row * g.ldc + col] = epi_apply(epi, v);
                }
            }
    }
    } else {
    f32x16 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][e] = 0.0f;

    // per-lane LDS read offsets, fixed over k (stage offsets fold into immediates)
    const int arow = wave * 32 + lr;
    int a_rd[2][2], b_rd[2][4];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        a_rd[s][0] = xa_sw(arow, 4 * s + 2 * lh);
        a_rd[s][1] = xa_sw(arow, 4 * s + 2 * lh + 1);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) b_rd[s][ni] = XA + xb_sw(ni * 32 + lr, 2 * s + lh);
    }

    // One k-tile: issue the next tile's DMA into `nxt`, then read `cur`
    // fragment by fragment interleaved with the split and the MFMAs. The
    // __restrict__ parameters give the inlined accesses disjoint alias scopes,
    // which lets the waitcnt pass see that the reads of `cur` do not depend on
    // the DMA into `nxt` (otherwise every read waits vmcnt(0) for it).
    auto tile = [&](const unsigned char* __restrict__ cur, unsigned char* __restrict__ nxt, int fph, int fk0) {
        if (fph == 0) fill_ph(0, fk0, nxt);
        else if (DUAL && fph == 1) fill_ph(1, fk0, nxt);
        // A fragments of both k-halves; the second half is split in four
        // slices beside the first half's four 6-MFMA groups (software
        // pipelined: only the first half's split precedes an MFMA)
        float4 alo[2], ahi[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            alo[s] = *reinterpret_cast<const float4*>(cur + a_rd[s][0]);
            ahi[s] = *reinterpret_cast<const float4*>(cur + a_rd[s][1]);
        }
        unsigned w[2][3][4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            split_pair(f4_at(alo[0], ahi[0], 2 * j), f4_at(alo[0], ahi[0], 2 * j + 1), w[0][0][j], w[0][1][j], w[0][2][j]);
        // B fragments double-buffered across the eight (k-half, column) groups:
        // group g+1's reads are in flight during group g's MFMAs
        u32x4 bq[2][3];
#pragma unroll
        for (int p = 0; p < 3; ++p) bq[0][p] = *reinterpret_cast<const u32x4*>(cur + b_rd[0][0] + p * XB_PLANE);
#pragma unroll
        for (int gi = 0; gi < 8; ++gi) {
            const int s = gi >> 2, ni = gi & 3;
            if (gi + 1 < 8) {
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    bq[(gi + 1) & 1][p] =
                        *reinterpret_cast<const u32x4*>(cur + b_rd[(gi + 1) >> 2][(gi + 1) & 3] + p * XB_PLANE);
            }
            bf16x8 af[3], bf[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                af[p] = __builtin_bit_cast(bf16x8, u32x4{w[s][p][0], w[s][p][1], w[s][p][2], w[s][p][3]});
                bf[p] = __builtin_bit_cast(bf16x8, bq[gi & 1][p]);
            }
            if (s == 0)
                split_pair(f4_at(alo[1], ahi[1], 2 * ni), f4_at(alo[1], ahi[1], 2 * ni + 1), w[1][0][ni], w[1][1][ni],
                           w[1][2][ni]);
            f32x16 c = acc[ni];
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1], bf[1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[2], bf[0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bf[2], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1], bf[0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bf[1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bf[0], c, 0, 0, 0);
            acc[ni] = c;
            // fence per 6-MFMA group: the scheduler otherwise hoists the second
            // half's split into one VALU block ahead of its MFMAs
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    // one k-loop per phase (compile-time ph: no per-tile operand selection);
    // the last tile of phase 0 prefetches the first tile of phase 1
    fill_ph(0, 0, xsm);
    __syncthreads();
    int stage = 0;
#pragma unroll
    for (int ph = 0; ph < (DUAL ? 2 : 1); ++ph) {
        const int nkp = ph ? nk1 : nk0;
        for (int kt = 0; kt < nkp; ++kt) {
            // the other stage was last read in the previous tile, before the barrier
            int fph = -1, fk0 = 0;
            if (kt + 1 < nkp) { fph = ph; fk0 = (kt + 1) * 32; }
            else if (DUAL && ph == 0 && nk1 > 0) fph = 1;
            tile(xsm + stage * STG, xsm + (stage ^ 1) * STG, fph, fk0);
            __syncthreads();  // retires the DMA of the next tile (vmcnt) for all waves
            stage ^= 1;
        }
    }

#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
        const int col = n0 + ni * 32 + lr;
        if (col >= g.N) continue;
        float b = 0.0f;
        if (g.bias0) b = g.bias0[col];
        if (g.bias1) b += g.bias1[col];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int64_t row = m0 + wave * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
            if (row < g.M) {
                float v = acc[ni][e];
                if (g.alpha != 1.0f) v *= g.alpha;
                if (g.bias0 || g.bias1) v += b;
                if (g.addend) v += g.addend[row * g.ld_add + col];
                g.C[row * g.ldc + col] = epi_apply(epi, v);
            }
        }
    }
    }
}

// Split a [rows][cols] f32 matrix into three bf16 planes (plane stride rows*cols).
__global__ void k_split_x3(const float* __restrict__ src, int64_t n, uint16_t* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float a = src[i];
    const unsigned h = __float_as_uint(a) & 0xFFFF0000u;
    const float r = a - __uint_as_float(h);
    const unsigned m = __float_as_uint(r) & 0xFFFF0000u;
    const float s = r - __uint_as_float(m);
    dst[i] = (uint16_t)(h >> 16);
    dst[n + i] = (uint16_t)(m >> 16);
    dst[2 * n + i] = (uint16_t)(__float_as_uint(s) >> 16);
}

// ---------------------------------------------------------------------------
// Split-f16 MFMA GEMM ("h2"), the GraphSAGE layer's dual GEMM. Each f32
// operand row is scaled by a power of two (exact) so its largest magnitude
// lands in [2^14, 2^15) — A rows by the gather kernel (row_scale of
// aggregate_rows, over the aggregate AND the self row of the dual GEMM), B
// rows (output features) once at upload — then split with round-to-nearest
// into two f16 parts, x = x1 + x2 + r with |r| <= 2^-22 |x|. Three f16 MFMA
// products per fragment pair, a2b1 + a1b2 + a1b1 (the dropped a2b2 is
// <= 2^-22 |ab|), accumulate in f32; the epilogue undoes the two scales
// exactly. Per product that is f32-level accuracy at half the MFMA work of the
// six-product bf16 split (x3) and two thirds of its B operand bytes.
// Tiling as gemm_nt_x3g<.., 4, false>: 128x128x32, waves 4(M) x 1(N), LDS-DMA
// stage fill with source-address XOR swizzle, 2 x 32 KB stages.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
// packed form: v_pk_mul_f32, v_cvt_pk_f16_f32 (RNE) for the high parts, the exact residual
// x - f32(h) (v_pk_add_f32) rounded the same way for the low parts — 6 VALU per pair
__device__ __forceinline__ void split_h2_pair(float a0, float a1, float sc, unsigned& w1, unsigned& w2) {
    const f32x2 x = f32x2{a0, a1} * sc;
    const f16x2 h = __builtin_convertvector(x, f16x2);
    const f16x2 l = __builtin_convertvector(x - __builtin_convertvector(h, f32x2), f16x2);
    w1 = __builtin_bit_cast(unsigned, h);
    w2 = __builtin_bit_cast(unsigned, l);
}

// XCD x (= block id % 8: workgroups are dealt round-robin over the 8 XCDs)
// owns the contiguous tile range [xcd_first(x), xcd_first(x) + xcd_count(x)).
__device__ __forceinline__ int64_t xcd_first(int64_t nwg, int64_t xcd) {
    const int64_t q = nwg / 8, r = nwg % 8;
    return xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
}
__device__ __forceinline__ int64_t xcd_count(int64_t nwg, int64_t xcd) { return nwg / 8 + (xcd < nwg % 8 ? 1 : 0); }
__device__ __forceinline__ int64_t part_first(int64_t n, int64_t parts, int64_t i) {
    const int64_t q = n / parts, r = n % parts;
    return i < r ? i * (q + 1) : r * (q + 1) + (i - r) * q;
}
__device__ __forceinline__ int64_t part_count(int64_t n, int64_t parts, int64_t i) { return n / parts + (i < n % parts ? 1 : 0); }

// End of a tile episode with in-launch row normalisation: every column tile of a
// 128-row block publishes its stores (each wave's vmcnt drain, the block barrier,
// one agent-scope release) and takes an arrival ticket; the block that draws the
// last ticket acquires and normalises the 128 rows over all N columns
// (cdna_hip_programming.md §6 Guideline 16, counter form: correct for any
// placement of the column tiles over XCDs/CUs; no block waits on another). The
// row pass is k_normalize_rows_vec's arithmetic (k_data.hip: per-lane float4
// slots 4 lane + 256 j, sequential squares, xor-tree sum, sqrtf, true division),
// so C is bit-identical to the GEMM followed by normalize_rows(only_positive).
__device__ __forceinline__ void h2g_rownorm(const GemmArgs& g, int64_t tm, int64_t m0, unsigned char* lds) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    volatile int* flag = reinterpret_cast<volatile int*>(lds);  // k-loop stages are free here
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned t = __hip_atomic_fetch_add(g.row_tickets + tm, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = t == (unsigned)(g.tiles_n - 1);
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *flag = last;
    }
    __syncthreads();
    const int last = *flag;
    if (!last) return;  // the caller's next barrier precedes any reuse of the stages
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int r = wave; r < 128; r += 4) {
        const int64_t row = m0 + r;
        if (row >= g.M) break;
        float* x = g.C + row * g.ldc + 4 * lane;
        float4 v[4];
        float s = 0.0f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // slots past N add +0: the same sum as NV = ceil(N / 256) slots
            const bool on = 4 * lane + 256 * j < g.N;
            v[j] = on ? *reinterpret_cast<const float4*>(x + 256 * j) : make_float4(0.f, 0.f, 0.f, 0.f);
            s = __fadd_rn(s, __fmul_rn(v[j].x, v[j].x));
            s = __fadd_rn(s, __fmul_rn(v[j].y, v[j].y));
            s = __fadd_rn(s, __fmul_rn(v[j].z, v[j].z));
            s = __fadd_rn(s, __fmul_rn(v[j].w, v[j].w));
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        const float norm = sqrtf(s);
        if (!(norm > 0.0f)) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (4 * lane + 256 * j < g.N)
                *reinterpret_cast<float4*>(x + 256 * j) =
                    make_float4(v[j].x / norm, v[j].y / norm, v[j].z / norm, v[j].w / norm);
    }
}

template <bool DUAL>
__device__ __forceinline__ void h2g_tile(const GemmArgs& g, int epi, int64_t wgid) {
    constexpr int XA = 128 * 128;             // f32 A tile bytes per stage
    constexpr int STG = XA + 2 * XB_PLANE;    // 32 KB stage
    constexpr int NB = 4;                     // B DMA pieces per wave (2 planes x 8 pieces)
    extern __shared__ __attribute__((aligned(16))) unsigned char xsm[];

    const int64_t tm = wgid / g.tiles_n;
    const int tn = (int)(wgid % g.tiles_n);
    const int64_t m0 = tm * 128;
    const int n0 = tn * XBN;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 31, lh = lane >> 5;

    const int nk0 = g.K0 / 32;
    const int nk1 = DUAL ? g.K1 / 32 : 0;

    auto sw_a = [](int row) { return (row >> 1) & 7; };
    auto sw_b = [](int row) { return (row >> 2) & 3; };

    uint32_t a_off[2][4], b_off[2][NB];
    const char* a_base[2];
    const char* b_base[2];
#pragma unroll
    for (int ph = 0; ph < (DUAL ? 2 : 1); ++ph) {
        const float* A = ph ? g.A1 : g.A0;
        const _Float16* B = ph ? g.B1h : g.B0h;
        const int64_t lda = ph ? g.lda1 : g.lda0, ldb = ph ? g.ldb1 : g.ldb0, bpl = ph ? g.B1h_plane : g.B0h_plane;
        a_base[ph] = reinterpret_cast<const char*>(A + m0 * lda);
        b_base[ph] = reinterpret_cast<const char*>(B + (int64_t)n0 * ldb);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = 8 * (4 * wave + j) + (lane >> 3);
            const int chunk = (lane & 7) ^ sw_a(row);
            const int64_t rr = std::min<int64_t>(m0 + row, g.M - 1) - m0;
            a_off[ph][j] = (uint32_t)((rr * lda + 4 * chunk) * 4);
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const int piece = NB * wave + j;
            const int row = 16 * (piece & 7) + (lane >> 2);
            const int chunk = (lane & 3) ^ sw_b(row);
            const int64_t rr = std::min<int64_t>(n0 + row, (int64_t)g.N - 1) - n0;
            b_off[ph][j] = (uint32_t)(((piece >> 3) * bpl + rr * ldb + 8 * chunk) * 2);
        }
    }

    auto fill_ph = [&](int ph, int k0, unsigned char* base) {
        const char* ab = a_base[ph] + (int64_t)k0 * 4;
        const char* bb = b_base[ph] + (int64_t)k0 * 2;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            __builtin_amdgcn_global_load_lds((const void*)(ab + a_off[ph][j]),
                                             (__attribute__((address_space(3))) void*)(base + (4 * wave + j) * 1024),
                                             16, 0, 0);
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const int piece = NB * wave + j;
            __builtin_amdgcn_global_load_lds(
                (const void*)(bb + b_off[ph][j]),
                (__attribute__((address_space(3))) void*)(base + XA + (piece >> 3) * XB_PLANE + (piece & 7) * 1024),
                16, 0, 0);
        }
    };
    auto xa_sw = [&](int row, int chunk) { return row * 128 + ((chunk ^ sw_a(row)) << 4); };
    auto xb_sw = [&](int row, int chunk) { return row * 64 + ((chunk ^ sw_b(row)) << 4); };

    f32x16 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][e] = 0.0f;

    const int arow = wave * 32 + lr;
    const float a_sc0 = g.a_scale[std::min<int64_t>(m0 + arow, g.M - 1)];
    // phase 1 with a row multiplier m: v * (m * sc) == round(v * m) * sc bit for bit (sc is a
    // power of two), i.e. the split of the multiplied row at no extra k-loop work
    const float a_sc1 = g.a1_rowmul ? a_sc0 * g.a1_rowmul[std::min<int64_t>(m0 + arow, g.M - 1)] : a_sc0;
    int a_rd[2][2], b_rd[2][4];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        a_rd[s][0] = xa_sw(arow, 4 * s + 2 * lh);
        a_rd[s][1] = xa_sw(arow, 4 * s + 2 * lh + 1);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) b_rd[s][ni] = XA + xb_sw(ni * 32 + lr, 2 * s + lh);
    }

    auto tile = [&](const unsigned char* __restrict__ cur, unsigned char* __restrict__ nxt, int fph, int fk0,
                    float a_sc) {
        if (fph == 0) fill_ph(0, fk0, nxt);
        else if (DUAL && fph == 1) fill_ph(1, fk0, nxt);
        float4 alo[2], ahi[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            alo[s] = *reinterpret_cast<const float4*>(cur + a_rd[s][0]);
            ahi[s] = *reinterpret_cast<const float4*>(cur + a_rd[s][1]);
        }
        unsigned w[2][2][4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            split_h2_pair(f4_at(alo[0], ahi[0], 2 * j), f4_at(alo[0], ahi[0], 2 * j + 1), a_sc, w[0][0][j], w[0][1][j]);
        u32x4 bq[2][2];
#pragma unroll
        for (int p = 0; p < 2; ++p) bq[0][p] = *reinterpret_cast<const u32x4*>(cur + b_rd[0][0] + p * XB_PLANE);
#pragma unroll
        for (int gi = 0; gi < 8; ++gi) {
            const int s = gi >> 2, ni = gi & 3;
            if (gi + 1 < 8) {
#pragma unroll
                for (int p = 0; p < 2; ++p)
                    bq[(gi + 1) & 1][p] =
                        *reinterpret_cast<const u32x4*>(cur + b_rd[(gi + 1) >> 2][(gi + 1) & 3] + p * XB_PLANE);
            }
            f16x8 af[2], bf[2];
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                af[p] = __builtin_bit_cast(f16x8, u32x4{w[s][p][0], w[s][p][1], w[s][p][2], w[s][p][3]});
                bf[p] = __builtin_bit_cast(f16x8, bq[gi & 1][p]);
            }
            if (s == 0)
                split_h2_pair(f4_at(alo[1], ahi[1], 2 * ni), f4_at(alo[1], ahi[1], 2 * ni + 1), a_sc, w[1][0][ni],
                              w[1][1][ni]);
            acc[ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], bf[0], acc[ni], 0, 0, 0);
            acc[ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0], bf[1], acc[ni], 0, 0, 0);
            acc[ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0], bf[0], acc[ni], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    fill_ph(0, 0, xsm);
    __syncthreads();
    int stage = 0;
#pragma unroll
    for (int ph = 0; ph < (DUAL ? 2 : 1); ++ph) {
        const int nkp = ph ? nk1 : nk0;
        for (int kt = 0; kt < nkp; ++kt) {
            int fph = -1, fk0 = 0;
            if (kt + 1 < nkp) { fph = ph; fk0 = (kt + 1) * 32; }
            else if (DUAL && ph == 0 && nk1 > 0) fph = 1;
            tile(xsm + stage * STG, xsm + (stage ^ 1) * STG, fph, fk0, ph ? a_sc1 : a_sc0);
            __syncthreads();
            stage ^= 1;
        }
    }

    // epilogue: undo the row and column scales (powers of two: exact), then
    // alpha / bias / addend / activation as the other kernels; row-outer so the deferred
    // normalisation's per-row sum of squares needs one register
    float cinv[4], cb[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
        const int col = std::min(n0 + ni * 32 + lr, g.N - 1);
        cinv[ni] = g.b_inv[col];
        float b = 0.0f;
        if (g.bias0) b = g.bias0[col];
        if (g.bias1) b += g.bias1[col];
        cb[ni] = b;
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int64_t row = m0 + wave * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        const float rinv = 1.0f / g.a_scale[std::min<int64_t>(row, g.M - 1)];  // unconditional loads: no per-load wait
        float ssq = 0.0f;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
            const int col = n0 + ni * 32 + lr;
            if (col < g.N && row < g.M) {
                float v = (acc[ni][e] * rinv) * cinv[ni];
                if (g.alpha != 1.0f) v *= g.alpha;
                if (g.bias0 || g.bias1) v += cb[ni];
                if (g.addend) v += g.addend[row * g.ld_add + col];
                v = epi_apply(epi, v);
                g.C[row * g.ldc + col] = v;
                ssq = __fadd_rn(ssq, __fmul_rn(v, v));
            }
        }
        if (g.row_sumsq) {
            // this tile's 128 columns of the row: lanes lr of one half hold columns
            // ni * 32 + lr; a fixed xor tree over the 32 lanes of the half
#pragma unroll
            for (int off = 16; off > 0; off >>= 1) ssq += __shfl_xor(ssq, off);
            if (lr == 0 && row < g.M) g.row_sumsq[row * ROWSUMSQ_SLOTS + tn] = ssq;
        }
    }
    if (g.row_tickets) h2g_rownorm(g, tm, m0, xsm);
}

// Pre-split variant ("h2p") of the split-f16 GEMM: the producer (the SAGE
// gather, aggregate_rows with planes) already wrote A*a_scale as two f16
// planes with the same round-to-nearest split as split_h2_pair, so the k-loop
// is LDS-DMA fills and MFMAs only. A and B tiles share one layout (2 planes x
// rows x 64 B, 16-B chunks XOR-swizzled by (row>>2)&3). WM waves along M
// (32 rows each) x 128 columns; an NST-stage ring: step t waits only for its
// own DMAs (counted vmcnt), one raw barrier, then refills the stage step t-1
// read, so NST-1 steps of fills stay in flight across the MFMAs. Every output
// element sees the same MFMA chain as h2g: the results are bit-identical.
template <int V>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(V >= 0 && V < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((V & 15) | ((V >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

template <bool DUAL, int WM, int NST>
__global__ __launch_bounds__(64 * WM, WM == 4 && NST == 2 ? 2 : 1) void gemm_nt_h2p(GemmArgs g, int epi) {
    constexpr int BM = 32 * WM;
    constexpr int APL = BM * 64;               // one f16 A plane of a BM x 32 tile
    constexpr int BPL = XB_PLANE;              // one f16 B plane of a 128 x 32 tile
    constexpr int STG = 2 * APL + 2 * BPL;
    constexpr int NA = 4;                      // A DMA pieces per wave (2 planes x BM/16 rows / WM)
    constexpr int NBP = 16 / WM;               // B DMA pieces per wave
    constexpr int F = NA + NBP;                // DMAs per thread per step
    extern __shared__ __attribute__((aligned(16))) unsigned char xsm[];

    const int64_t nwg = g.nblocks;
    const int64_t bid = blockIdx.x;
    const int64_t xcd = bid % 8, q = nwg / 8, r = nwg % 8;
    const int64_t wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    const int64_t tm = wgid / g.tiles_n;
    const int tn = (int)(wgid % g.tiles_n);
    const int64_t m0 = tm * BM;
    const int n0 = tn * XBN;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 31, lh = lane >> 5;

    const int nk0 = g.K0 / 32;
    const int nsteps = nk0 + (DUAL ? g.K1 / 32 : 0);
    auto sw = [](int row) { return (row >> 2) & 3; };

    uint32_t a_off[2][NA], b_off[2][NBP];
    const char* a_base[2];
    const char* b_base[2];
#pragma unroll
    for (int ph = 0; ph < (DUAL ? 2 : 1); ++ph) {
        const _Float16* A = ph ? g.A1h : g.A0h;
        const _Float16* B = ph ? g.B1h : g.B0h;
        const int64_t lda = ph ? g.lda1 : g.lda0, ldb = ph ? g.ldb1 : g.ldb0, bpl = ph ? g.B1h_plane : g.B0h_plane;
        a_base[ph] = reinterpret_cast<const char*>(A + m0 * lda);
        b_base[ph] = reinterpret_cast<const char*>(B + (int64_t)n0 * ldb);
#pragma unroll
        for (int j = 0; j < NA; ++j) {  // piece: plane piece / (BM/16), rows 16 * (piece % (BM/16))
            const int piece = NA * wave + j;
            const int row = 16 * (piece % (BM / 16)) + (lane >> 2);
            const int chunk = (lane & 3) ^ sw(row);
            const int64_t ra = std::min<int64_t>(m0 + row, g.M - 1) - m0;
            a_off[ph][j] = (uint32_t)(((piece / (BM / 16)) * g.Ah_plane + ra * lda + 8 * chunk) * 2);
        }
#pragma unroll
        for (int j = 0; j < NBP; ++j) {
            const int piece = NBP * wave + j;
            const int row = 16 * (piece & 7) + (lane >> 2);
            const int chunk = (lane & 3) ^ sw(row);
            const int64_t rb = std::min<int64_t>(n0 + row, (int64_t)g.N - 1) - n0;
            b_off[ph][j] = (uint32_t)(((piece >> 3) * bpl + rb * ldb + 8 * chunk) * 2);
        }
    }

    auto fill = [&](int t, unsigned char* base) {
        const int ph = (DUAL && t >= nk0) ? 1 : 0;
        const int k0 = (t - (ph ? nk0 : 0)) * 32;
        const char* ab = a_base[ph] + (int64_t)k0 * 2;
        const char* bb = b_base[ph] + (int64_t)k0 * 2;
#pragma unroll
        for (int j = 0; j < NA; ++j) {
            const int piece = NA * wave + j;
            __builtin_amdgcn_global_load_lds(
                (const void*)(ab + a_off[ph][j]),
                (__attribute__((address_space(3))) void*)(base + (piece / (BM / 16)) * APL + (piece % (BM / 16)) * 1024),
                16, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < NBP; ++j) {
            const int piece = NBP * wave + j;
            __builtin_amdgcn_global_load_lds(
                (const void*)(bb + b_off[ph][j]),
                (__attribute__((address_space(3))) void*)(base + 2 * APL + (piece >> 3) * BPL + (piece & 7) * 1024),
                16, 0, 0);
        }
    };
    auto x_sw = [&](int row, int chunk) { return row * 64 + ((chunk ^ sw(row)) << 4); };

    f32x16 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][e] = 0.0f;

    int a_rd[2], b_rd[2][4];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        a_rd[s] = x_sw(wave * 32 + lr, 2 * s + lh);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) b_rd[s][ni] = 2 * APL + x_sw(ni * 32 + lr, 2 * s + lh);
    }

    auto compute = [&](const unsigned char* __restrict__ cur) {
        f16x8 af[2][2];
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int p = 0; p < 2; ++p) af[s][p] = *reinterpret_cast<const f16x8*>(cur + a_rd[s] + p * APL);
        u32x4 bq[2][2];
#pragma unroll
        for (int p = 0; p < 2; ++p) bq[0][p] = *reinterpret_cast<const u32x4*>(cur + b_rd[0][0] + p * BPL);
#pragma unroll
        for (int gi = 0; gi < 8; ++gi) {
            const int s = gi >> 2, ni = gi & 3;
            if (gi + 1 < 8) {
#pragma unroll
                for (int p = 0; p < 2; ++p)
                    bq[(gi + 1) & 1][p] =
                        *reinterpret_cast<const u32x4*>(cur + b_rd[(gi + 1) >> 2][(gi + 1) & 3] + p * BPL);
            }
            f16x8 bf[2];
#pragma unroll
            for (int p = 0; p < 2; ++p) bf[p] = __builtin_bit_cast(f16x8, bq[gi & 1][p]);
            acc[ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[s][1], bf[0], acc[ni], 0, 0, 0);
            acc[ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[s][0], bf[1], acc[ni], 0, 0, 0);
            acc[ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[s][0], bf[0], acc[ni], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    // ring: steps 0..NST-2 in flight before the loop
#pragma unroll
    for (int f = 0; f < NST - 1; ++f)
        if (f < nsteps) fill(f, xsm + f * STG);
    int st = 0, fst = NST - 1;
    for (int t = 0; t < nsteps; ++t) {
        const int later = min(NST - 2, nsteps - t - 1);  // steps after t already issued
        if (NST >= 4 && later >= 2) wait_vmcnt<(NST >= 4 ? 2 * F : 0)>();
        else if (NST >= 3 && later >= 1) wait_vmcnt<(NST >= 3 ? F : 0)>();
        else wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();  // every wave's share of step t landed; step t-1's stage is free
        asm volatile("" ::: "memory");
        if (t + NST - 1 < nsteps) fill(t + NST - 1, xsm + fst * STG);
        compute(xsm + st * STG);
        st = st == NST - 1 ? 0 : st + 1;
        fst = fst == NST - 1 ? 0 : fst + 1;
    }

    float rinv[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int64_t row = m0 + wave * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        rinv[e] = row < g.M ? 1.0f / g.a_scale[row] : 0.0f;
    }
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
        const int col = n0 + ni * 32 + lr;
        if (col >= g.N) continue;
        const float cinv = g.b_inv[col];
        float b = 0.0f;
        if (g.bias0) b = g.bias0[col];
        if (g.bias1) b += g.bias1[col];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int64_t row = m0 + wave * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
            if (row < g.M) {
                float v = (acc[ni][e] * rinv[e]) * cinv;
                if (g.alpha != 1.0f) v *= g.alpha;
                if (g.bias0 || g.bias1) v += b;
                if (g.addend) v += g.addend[row * g.ld_add + col];
                g.C[row * g.ldc + col] = epi_apply(epi, v);
            }
        }
    }
}

// One tile per block, or (grid capped below the tile count, RVX_GEMM_CAP) a
// persistent grid. Persistent blocks drain their XCD's tile range through a
// per-XCD atomic counter (g.queue, zeroed before the launch): tiles are taken
// in row-tile-major order as blocks free up, so the column tiles of one
// 128-row A tile start within a few tile-grabs of each other on one XCD and
// share the A rows through its L2 (a static stride lets the blocks drift
// apart and every column tile re-fetches A from HBM). Every block reaches the
// counter's end, so the grid always drains.
template <bool DUAL>
__global__ __launch_bounds__(256, 2) void gemm_nt_h2g(GemmArgs g, int epi) {
    if (g.queue) {
        __shared__ int64_t s_t;
        const int64_t xcd = blockIdx.x % 8;
        int64_t first = xcd_first(g.nblocks, xcd), cnt = xcd_count(g.nblocks, xcd);
        const int half = g.xsplit ? g.tiles_n / 2 : 0;
        if (half) {  // rows [first, first + cnt / half) of the pair's range, column tiles (xcd & 1) * half + [0, half)
            const int64_t tm_tot = g.nblocks / g.tiles_n;
            first = part_first(tm_tot, 4, xcd >> 1);
            cnt = part_count(tm_tot, 4, xcd >> 1) * half;
        }
        for (;;) {
            if (threadIdx.x == 0) s_t = (int64_t)atomicAdd(g.queue + 32 * xcd, 1u);
            __syncthreads();
            const int64_t t = s_t;
            if (t >= cnt) break;
            h2g_tile<DUAL>(g, epi, half ? (first + t / half) * g.tiles_n + (xcd & 1) * half + t % half : first + t);
            __syncthreads();  // LDS stages and s_t are reused by the next tile
        }
        return;
    }
    for (int64_t b = blockIdx.x; b < g.nblocks; b += gridDim.x) {
        h2g_tile<DUAL>(g, epi, xcd_first(g.nblocks, b % 8) + b / 8);
        if (b + gridDim.x < g.nblocks) __syncthreads();  // LDS stages are reused by the next tile
    }
}

// Wide split-f16 GEMM ("h2w"): gemm_nt_h2g's arithmetic — per-row power-of-two A scale,
// the in-register hi/lo split of A (split_h2_pair), three MFMA products per k16 in the
// same order (a_lo b_hi, a_hi b_lo, a_hi b_hi), k ascending — so every output is
// bit-identical to h2g, on a 256 x 256 x 32 tile: 8 waves (2 along M x 4 along N), 128 x 64
// outputs and 8 accumulators per wave, half the LDS bytes per MFMA of the 128 x 128 tile
// and one block (two 64 KB stages) per CU. Each K-tile opens with one vmcnt(0) + barrier
// (this stage landed everywhere, the other stage fully read), then runs four phases, one
// per 32-row block of the wave's rows: that block's A slice read and split in registers,
// 12 MFMAs against the wave's B fragments (read once per K-tile), and 2 of the 16 LDS-DMA
// pieces of the next K-tile issued between them, so the next stage's loads have a whole
// K-tile of MFMA work to land (cdna_hip_programming.md §5.5 T3/T4, without per-phase
// barriers). A and B stages keep h2g's layouts and source-side XOR swizzles.
#ifndef H2W_RING
#define H2W_RING 4
#endif
// K loop and epilogue of h2w_tile<..., M16 = true> (WN = 1: wave wm owns tile rows
// [32 wm, 32 wm + 32), all BN columns). Lane (lc, lg) = (lane & 15, lane >> 4): A fragment =
// row lc of a 16-row half, k 8 lg .. 8 lg + 7 (LDS chunks 2 lg, 2 lg + 1); B fragment = column lc
// of a 16-column subtile, k 8 lg .. 8 lg + 7 (chunk lg) of each f16 plane; accumulator element v
// = row 4 lg + v, column lc of the (half, subtile).
template <bool DUAL, int BN, int NW, bool AMX, class Issue>
__device__ __forceinline__ void h2w_m16_body(const GemmArgs& g, int epi, int64_t m0, int n0, int tn, int wm, int lane,
                                             int nk0, int nkt, const float* asc, const float* asc1, Issue& issue) {
    constexpr int XA = 32 * NW * 128, BPL = BN * 64, STG = XA + 2 * BPL;
    constexpr int NS = BN / 16;       // 16-column subtiles per wave
    constexpr int NBP = BN / (8 * NW);
    extern __shared__ __attribute__((aligned(16))) unsigned char xsm[];
    const int lc = lane & 15, lg = lane >> 4;
    const int arow = wm * 32 + lc;
    const int aswz = (arow & 7) ^ ((arow >> 3) & 1);  // rows arow and arow + 16 share it
    const int a_rd0 = arow * 128 + (((2 * lg) ^ aswz) << 4);
    const int a_rd1 = arow * 128 + (((2 * lg + 1) ^ aswz) << 4);
    const int b_rd = XA + lc * 64 + ((lg ^ ((4 - ((lc >> 2) & 3)) & 3)) << 4);  // + 1024 per subtile

    f32x4 acc[2][NS];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int ns = 0; ns < NS; ++ns) acc[h][ns] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

#pragma unroll
    for (int j = 0; j < 4 + NBP; ++j) issue(0, xsm, j);
    auto ktile = [&](const unsigned char* __restrict__ cur, unsigned char* __restrict__ nxt, int t) {
        if (t + 1 < nkt) {
#pragma unroll
            for (int j = 0; j < 4 + NBP; ++j) issue(t + 1, nxt, j);
        }
        const float sc = DUAL && t >= nk0 ? asc1[0] : asc[0];
        f16x8 af[2][2];  // [half][hi, lo]
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float4 alo = *reinterpret_cast<const float4*>(cur + a_rd0 + h * 2048);
            const float4 ahi = *reinterpret_cast<const float4*>(cur + a_rd1 + h * 2048);
            unsigned w[2][4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                split_h2_pair(f4_at(alo, ahi, 2 * j), f4_at(alo, ahi, 2 * j + 1), sc, w[0][j], w[1][j]);
#pragma unroll
            for (int p = 0; p < 2; ++p) af[h][p] = __builtin_bit_cast(f16x8, u32x4{w[p][0], w[p][1], w[p][2], w[p][3]});
        }
#pragma unroll
        for (int ns = 0; ns < NS; ++ns) {
            const f16x8 b0 = __builtin_bit_cast(f16x8, *reinterpret_cast<const u32x4*>(cur + b_rd + ns * 1024));
            const f16x8 b1 = __builtin_bit_cast(f16x8, *reinterpret_cast<const u32x4*>(cur + b_rd + ns * 1024 + BPL));
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                acc[h][ns] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[h][1], b0, acc[h][ns], 0, 0, 0);
                acc[h][ns] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[h][0], b1, acc[h][ns], 0, 0, 0);
                acc[h][ns] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[h][0], b0, acc[h][ns], 0, 0, 0);
            }
        }
    };
    for (int t = 0; t < nkt; ++t) {
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();  // stage t landed for every wave; stage t-1 fully read
        asm volatile("" ::: "memory");
        ktile(xsm + (t & 1) * STG, xsm + ((t + 1) & 1) * STG, t);
    }

    // epilogue: undo the row and column scales (powers of two: exact), then alpha / bias /
    // addend / activation; per row the tile's sum of squares (16-lane reduction)
    float cinv[NS], cb[NS];
#pragma unroll
    for (int ns = 0; ns < NS; ++ns) {
        const int col = std::min(n0 + ns * 16 + lc, g.N - 1);
        cinv[ns] = g.b_inv[col];
        float b = 0.0f;
        if (g.bias0) b = g.bias0[col];
        if (g.bias1) b += g.bias1[col];
        cb[ns] = b;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int64_t row = m0 + wm * 32 + h * 16 + 4 * lg + v;
            const float rinv = 1.0f / g.a_scale[std::min<int64_t>(row, g.M - 1)];
            float ssq = 0.0f, amx = 0.0f;
            float addv[NS];
            if (AMX && g.addend) {
                const int64_t arow2 = std::min<int64_t>(row, g.M - 1);
#pragma unroll
                for (int ns = 0; ns < NS; ++ns) addv[ns] = g.addend[arow2 * g.ld_add + std::min(n0 + ns * 16 + lc, g.N - 1)];
            }
#pragma unroll
            for (int ns = 0; ns < NS; ++ns) {
                const int col = n0 + ns * 16 + lc;
                if (col < g.N && row < g.M) {
                    float x = (acc[h][ns][v] * rinv) * cinv[ns];
                    if (g.alpha != 1.0f) x *= g.alpha;
                    if (g.bias0 || g.bias1) x += cb[ns];
                    if (g.addend) x += AMX ? addv[ns] : g.addend[row * g.ld_add + col];
                    x = epi_apply(epi, x);
                    g.C[row * g.ldc + col] = x;
                    ssq = __fadd_rn(ssq, __fmul_rn(x, x));
                    if constexpr (AMX) amx = fmaxf(amx, fabsf(x));
                }
            }
            if constexpr (AMX) {
#pragma unroll
                for (int off = 8; off > 0; off >>= 1) amx = fmaxf(amx, __shfl_xor(amx, off));
                if (lc == 0 && row < g.M) g.row_absmax[row * ROWSUMSQ_SLOTS + tn] = amx;
            }
            if (g.row_sumsq) {
#pragma unroll
                for (int off = 8; off > 0; off >>= 1) ssq += __shfl_xor(ssq, off);
                if (lc == 0 && row < g.M) g.row_sumsq[row * ROWSUMSQ_SLOTS + tn] = ssq;
            }
        }
}
// M16 (WN == 1, K loop without PIPE): the same tile on v_mfma_f32_16x16x32_f16 — a wave's 32
// rows as two 16-row halves, its columns as 16-column subtiles, one K = 32 MFMA step per
// (half, subtile) and product (a_lo b_hi, a_hi b_lo, a_hi b_hi); the chip holds a higher clock
// under the smaller shape (MI355X_MICROARCH.md DVFS, K10's +11%). The swizzles change so the
// 16x16x32 fragment reads stay bank-conflict free (enumerated for ds_read_b128's lane groups):
// A chunk c of row r at c ^ ((r & 7) ^ ((r >> 3) & 1)), B chunk c at c ^ ((4 - ((r >> 2) & 3)) & 3).
// One MFMA sums 32 products instead of two sums of 16, so the bits differ from h2g's (within
// the same error bound; tests hold M16 to the oracle, and M16 tilings to each other).
template <bool DUAL, int WN, int BN, int NW, bool PIPE = false, bool AMX = false, bool GATE = false, bool M16 = false>
__device__ __forceinline__ void h2w_tile(const GemmArgs& g, int epi, int64_t wgid) {
    static_assert(!M16 || (WN == 1 && !PIPE && !GATE), "16x16x32 form: waves own whole tile rows, plain K loop");
    constexpr int BM = 32 * NW;        // 256 rows with 8 waves, 128 with 4
    constexpr int WMW = NW / WN;                // waves along M
    constexpr int RB = BM / WMW / 32, NB = BN / WN / 32;  // 32-row / 32-column blocks per wave
    constexpr int NBP = BN / (8 * NW);  // B DMA pieces per wave (2 planes x BN / 16 pieces over NW waves)
    constexpr int XA = BM * 128;       // f32 A tile bytes per stage (BM rows x 32 k)
    constexpr int BPL = BN * 64;       // one f16 B plane tile (BN columns x 32 k)
    constexpr int STG = XA + 2 * BPL;  // 64 KB (BN 256) / 56 KB (BN 192)
    extern __shared__ __attribute__((aligned(16))) unsigned char xsm[];

    const int64_t tm = wgid / g.tiles_n;
    const int tn = (int)(wgid % g.tiles_n);
    const int64_t m0 = tm * BM;
    const int n0 = tn * BN;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int lr = lane & 31, lh = lane >> 5;
    const int nk0 = g.K0 / 32;
    const int nkt = nk0 + (DUAL ? g.K1 / 32 : 0);

    auto sw_a = [](int row) { return M16 ? ((row & 7) ^ ((row >> 3) & 1)) : ((row >> 1) & 7); };
    auto sw_b = [](int row) { return M16 ? ((4 - ((row >> 2) & 3)) & 3) : ((row >> 2) & 3); };

    // 64 DMA pieces of 1 KB per stage, 8 per wave: A pieces 4 wave + j (8 rows x 128 B),
    // B pieces 4 wave + j of 32 (plane piece / 16, 16 rows x 64 B each)
    // the host routes here only operands whose phase-1 strides equal phase 0's
    // (lda, ldb, B plane stride), so one set of lane offsets serves both phases
    uint32_t a_off[4], b_off[NBP];
    const char* a_base[2];
    const char* b_base[2];
    a_base[0] = reinterpret_cast<const char*>(g.A0 + m0 * g.lda0);
    b_base[0] = reinterpret_cast<const char*>(g.B0h + (int64_t)n0 * g.ldb0);
    a_base[1] = DUAL ? reinterpret_cast<const char*>(g.A1 + m0 * g.lda0) : a_base[0];
    b_base[1] = DUAL ? reinterpret_cast<const char*>(g.B1h + (int64_t)n0 * g.ldb0) : b_base[0];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int row = 8 * (4 * wave + j) + (lane >> 3);
        const int chunk = (lane & 7) ^ sw_a(row);
        const int64_t rr = std::min<int64_t>(m0 + row, g.M - 1) - m0;
        a_off[j] = (uint32_t)((rr * g.lda0 + 4 * chunk) * 4);
    }
#pragma unroll
    for (int j = 0; j < NBP; ++j) {
        const int piece = NBP * wave + j;
        const int brow = 16 * (piece % (BN / 16)) + (lane >> 2);
        const int bchunk = (lane & 3) ^ sw_b(brow);
        const int64_t rb = std::min<int64_t>(n0 + brow, (int64_t)g.N - 1) - n0;
        b_off[j] = (uint32_t)(((piece / (BN / 16)) * g.B0h_plane + rb * g.ldb0 + 8 * bchunk) * 2);
    }
    // piece j (0 .. 3 + NBP) of K-tile t's fill into stage `base`
    auto issue = [&](int t, unsigned char* base, int j) {
        const bool p1 = DUAL && t >= nk0;
        const int k0 = (t - (p1 ? nk0 : 0)) * 32;
        if (j < 4) {
            const char* src = (p1 ? a_base[1] : a_base[0]) + (int64_t)k0 * 4 + a_off[j];
            __builtin_amdgcn_global_load_lds((const void*)src,
                                             (__attribute__((address_space(3))) void*)(base + (4 * wave + j) * 1024),
                                             16, 0, 0);
        } else {
            const int jj = j - 4, piece = NBP * wave + jj;
            const char* src = (p1 ? b_base[1] : b_base[0]) + (int64_t)k0 * 2 + b_off[jj];
            __builtin_amdgcn_global_load_lds(
                (const void*)src,
                (__attribute__((address_space(3))) void*)(base + XA + (piece / (BN / 16)) * BPL +
                                                           (piece % (BN / 16)) * 1024),
                16, 0, 0);
        }
    };

    // read offsets (the swizzle depends on the row only mod 32: row blocks and column
    // blocks are immediate offsets 4096 / 2048)
    const int arow = wm * (32 * RB) + lr;
    const int bcol = wn * (32 * NB) + lr;
    int a_rd[2][2], b_rd[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        a_rd[s][0] = arow * 128 + (((4 * s + 2 * lh) ^ sw_a(arow)) << 4);
        a_rd[s][1] = arow * 128 + (((4 * s + 2 * lh + 1) ^ sw_a(arow)) << 4);
        b_rd[s] = XA + bcol * 64 + (((2 * s + lh) ^ sw_b(bcol)) << 4);
    }
    float asc[RB], asc1[RB];  // phase 1: s * m with the deferred normalisation's row multiplier (as h2g)
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
        const int64_t r = std::min<int64_t>(m0 + arow + 32 * rb, g.M - 1);
        asc[rb] = g.a_scale[r];
        asc1[rb] = g.a1_rowmul ? asc[rb] * g.a1_rowmul[r] : asc[rb];
    }

    if constexpr (M16) {
        h2w_m16_body<DUAL, BN, NW, AMX>(g, epi, m0, n0, tn, wm, lane, nk0, nkt, asc, asc1, issue);
        return;
    } else {
    f32x16 acc[RB][NB];
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

#pragma unroll
    for (int j = 0; j < 4 + NBP; ++j) issue(0, xsm, j);
    if constexpr (PIPE) {
        // Software-pipelined K loop. A wave owns 32 whole tile rows, so a K-tile is G = 2 NB
        // MFMA groups (k16 half s, column block nb), 3 MFMAs each. B fragments come from a
        // ring of R register pairs read L = R - 1 groups ahead of their MFMAs; the one barrier
        // per K-tile sits where the reads cross into the next stage (after group G - L: this
        // wave's reads of the stage are then all issued), and the DMA of tile t+2 into the
        // freed stage follows it. A(t, s1) is read and split during the s0 groups, A(t+1, s0)
        // during the s1 groups. Per accumulator the products keep h2w's order (s ascending;
        // a_lo b_hi, a_hi b_lo, a_hi b_hi), so every output is bit-identical.
        static_assert(WN == 1 && RB == 1, "pipelined form: a wave owns 32 whole tile rows");
        constexpr int G = 2 * NB, R = H2W_RING, L = R - 1, G0 = G - L;
        static_assert(G % R == 0 && G0 >= NB && G0 < G - 1, "ring slots are static per K-tile");
        u32x4 ring[R][2];
        float4 ra[2];
        u32x4 fx[2], fy[2];  // split A words [hi, lo] of the s0 / s1 half
        // pair j of the raw A slice into word j of af (one pair per MFMA group: the split's
        // VALU runs in the MFMA shadow instead of as one block ahead of a group)
        auto split_a = [&](float sc, u32x4 (&af)[2], int j) {
            unsigned w0, w1;
            split_h2_pair(f4_at(ra[0], ra[1], 2 * j), f4_at(ra[0], ra[1], 2 * j + 1), sc, w0, w1);
            af[0][j] = w0;
            af[1][j] = w1;
        };
        auto rd_a = [&](const unsigned char* st, int s) {
            ra[0] = *reinterpret_cast<const float4*>(st + a_rd[s][0]);
            ra[1] = *reinterpret_cast<const float4*>(st + a_rd[s][1]);
        };
        auto rd_b = [&](const unsigned char* st, int gg, u32x4 (&b)[2]) {
            const int s = gg / NB, nb = gg % NB;
            b[0] = *reinterpret_cast<const u32x4*>(st + b_rd[s] + nb * 2048);
            b[1] = *reinterpret_cast<const u32x4*>(st + b_rd[s] + nb * 2048 + BPL);
        };
        auto mm = [&](const u32x4 (&af)[2], const u32x4 (&b)[2], f32x16& c) {
            const f16x8 a0 = __builtin_bit_cast(f16x8, af[0]);
            const f16x8 a1 = __builtin_bit_cast(f16x8, af[1]);
            const f16x8 b0 = __builtin_bit_cast(f16x8, b[0]);
            const f16x8 b1 = __builtin_bit_cast(f16x8, b[1]);
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, c, 0, 0, 0);
        };
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (nkt > 1) {
#pragma unroll
            for (int j = 0; j < 4 + NBP; ++j) issue(1, xsm + STG, j);
        }
        rd_a(xsm, 0);
#pragma unroll
        for (int gg = 0; gg < L; ++gg) rd_b(xsm, gg, ring[gg]);
#pragma unroll
        for (int j = 0; j < 4; ++j) split_a(DUAL && nk0 == 0 ? asc1[0] : asc[0], fx, j);
        // tile t from `cur` (its stage), then the first reads of tile t+1 from `nxt`
        auto body = [&](unsigned char* __restrict__ cur, const unsigned char* __restrict__ nxt, int t) {
            const float sc = DUAL && t >= nk0 ? asc1[0] : asc[0];
            const float scn = DUAL && t + 1 >= nk0 ? asc1[0] : asc[0];
            const bool more = t + 1 < nkt;
#pragma unroll
            for (int gg = 0; gg < G; ++gg) {
                mm(gg < NB ? fx : fy, ring[gg % R], acc[0][gg % NB]);
                if (gg == 0) rd_a(cur, 1);
                if (gg >= 2 && gg < 6) split_a(sc, fy, gg - 2);  // A(t, s1), before group NB
                const int ng = gg + L;
                if (ng < G) {
                    rd_b(cur, ng, ring[ng % R]);
                } else if (more) {
                    if (ng == G) {
                        // this wave's reads of tile t are all issued: wait for them and for its
                        // DMA of tile t+1, then every wave's (barrier); tile t's stage is free
                        __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
                        __builtin_amdgcn_s_barrier();
                        asm volatile("" ::: "memory");
                        if (t + 2 < nkt) {
#pragma unroll
                            for (int j = 0; j < 4 + NBP; ++j) issue(t + 2, cur, j);
                        }
                        rd_a(nxt, 0);
                    }
                    rd_b(nxt, ng - G, ring[ng % R]);
                }
                if (gg > G0 && more) {  // A(t+1, s0): its pairs over the groups after the read
                    constexpr int NS = G - 1 - G0;
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (j * NS / 4 == gg - G0 - 1) split_a(scn, fx, j);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        for (int t = 0; t < nkt; ++t) body(xsm + (t & 1) * STG, xsm + ((t + 1) & 1) * STG, t);
    } else {
    // one K-tile; restrict parameters give the stage pointers distinct alias scopes, so
    // the ds_reads of `cur` do not wait for the LDS-DMA into `nxt` (vmcnt) in the phases
    auto ktile = [&](const unsigned char* __restrict__ cur, unsigned char* __restrict__ nxt, int t) {
        const bool more = t + 1 < nkt;
        const bool p1 = DUAL && t >= nk0;  // this K-tile reads the A1 / B1 operands
#ifndef RVX_H2W_SPREAD
        // all 16 KB of this wave's share of the next K-tile first: the loads get the whole
        // K-tile of MFMA work to land before the next tile's wait
        if (more) {
#pragma unroll
            for (int j = 0; j < 4 + NBP; ++j) issue(t + 1, nxt, j);
        }
#endif
        // B fragments [nb][s][plane]: held for the K-tile when the wave has 2 column blocks,
        // read per use when it has 8 (WN = 1)
        u32x4 bq[NB <= 2 ? NB : 1][2][2];
        if constexpr (NB <= 2) {
#pragma unroll
            for (int nb = 0; nb < NB; ++nb)
#pragma unroll
                for (int s = 0; s < 2; ++s)
#pragma unroll
                    for (int p = 0; p < 2; ++p)
                        bq[nb][s][p] = *reinterpret_cast<const u32x4*>(cur + b_rd[s] + nb * 2048 + p * BPL);
        }
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
#ifdef RVX_H2W_SPREAD
            if (more) {
                issue(t + 1, nxt, 2 * rb);
                issue(t + 1, nxt, 2 * rb + 1);
            }
#endif
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                // this k16 half of the row block's A slice, split in registers
                const float4 alo = *reinterpret_cast<const float4*>(cur + a_rd[s][0] + rb * 4096);
                const float4 ahi = *reinterpret_cast<const float4*>(cur + a_rd[s][1] + rb * 4096);
                unsigned w[2][4];  // [hi, lo][pair]
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    split_h2_pair(f4_at(alo, ahi, 2 * j), f4_at(alo, ahi, 2 * j + 1), p1 ? asc1[rb] : asc[rb],
                                  w[0][j], w[1][j]);
                f16x8 af[2];
#pragma unroll
                for (int p = 0; p < 2; ++p) af[p] = __builtin_bit_cast(f16x8, u32x4{w[p][0], w[p][1], w[p][2], w[p][3]});
#pragma unroll
                for (int nb = 0; nb < NB; ++nb) {
                    u32x4 q0, q1;
                    if constexpr (NB <= 2) {
                        q0 = bq[nb][s][0];
                        q1 = bq[nb][s][1];
                    } else {
                        q0 = *reinterpret_cast<const u32x4*>(cur + b_rd[s] + nb * 2048);
                        q1 = *reinterpret_cast<const u32x4*>(cur + b_rd[s] + nb * 2048 + BPL);
                    }
                    const f16x8 b0 = __builtin_bit_cast(f16x8, q0);
                    const f16x8 b1 = __builtin_bit_cast(f16x8, q1);
                    acc[rb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], b0, acc[rb][nb], 0, 0, 0);
                    acc[rb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0], b1, acc[rb][nb], 0, 0, 0);
                    acc[rb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0], b0, acc[rb][nb], 0, 0, 0);
                }
            }
        }
    };
    for (int t = 0; t < nkt; ++t) {
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();  // stage t landed for every wave; stage t-1 fully read
        asm volatile("" ::: "memory");
        ktile(xsm + (t & 1) * STG, xsm + ((t + 1) & 1) * STG, t);
    }
    }

    // epilogue as h2g: undo the row and column scales (powers of two: exact), then
    // alpha / bias / addend / activation; row-outer, and with WN = 1 (a wave holds whole
    // tile rows) the deferred normalisation's per-row sum of squares of this tile
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
        float cinv[NB], cb[NB];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
            const int col = std::min(n0 + wn * (32 * NB) + nb * 32 + lr, g.N - 1);
            cinv[nb] = g.b_inv[col];
            float b = 0.0f;
            if (g.bias0) b = g.bias0[col];
            if (g.bias1) b += g.bias1[col];
            cb[nb] = b;
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int64_t row = m0 + wm * (32 * RB) + rb * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
            const float rinv = 1.0f / g.a_scale[std::min<int64_t>(row, g.M - 1)];  // unconditional: no per-load wait
            float ssq = 0.0f, amx = 0.0f;
            // the row's addend values loaded (clamped, unconditional) before any store of the
            // row: the stores to C may alias them as far as the compiler knows, so loaded in
            // the store loop each waited alone (C4's out GEMM: 197 vs 133 ms for the same
            // GEMM without an addend per 10M step)
            // (AMX tiles only — C4's standalone GEMMs: the overlapped 256 x 192 tile keeps its
            // 163 VGPRs so a gather wave still fits beside it)
            float addv[NB];
            if (AMX && g.addend) {
                const int64_t arow = std::min<int64_t>(row, g.M - 1);
#pragma unroll
                for (int nb = 0; nb < NB; ++nb)
                    addv[nb] = g.addend[arow * g.ld_add + std::min(n0 + wn * (32 * NB) + nb * 32 + lr, g.N - 1)];
            } else if (GATE) {  // the gate's h values, same preload
                const int64_t arow = std::min<int64_t>(row, g.M - 1);
#pragma unroll
                for (int nb = 0; nb < NB; ++nb) {
                    const int cc = std::min(n0 + wn * (32 * NB) + nb * 32 + lr, g.N - 1);
                    addv[nb] = cc >= g.gate_col0 ? g.gate_h[arow * g.ld_gate_h + (cc - g.gate_col0)] : 0.0f;
                }
            }
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) {
                const int col = n0 + wn * (32 * NB) + nb * 32 + lr;
                if (col < g.N && row < g.M) {
                    float v = (acc[rb][nb][e] * rinv) * cinv[nb];
                    if (g.alpha != 1.0f) v *= g.alpha;
                    if (g.bias0 || g.bias1) v += cb[nb];
                    if (g.addend) v += AMX ? addv[nb] : g.addend[row * g.ld_add + col];
                    v = epi_apply(epi, v);
                    if (GATE && col >= g.gate_col0) {
                        const float o = v * addv[nb];
                        g.gate_out[row * g.ld_gate_out + (col - g.gate_col0)] = o;
                        amx = fmaxf(amx, fabsf(o));
                    } else {
                        g.C[row * g.ldc + col] = v;
                        ssq = __fadd_rn(ssq, __fmul_rn(v, v));
                        if constexpr (AMX && !GATE) amx = fmaxf(amx, fabsf(v));
                    }
                }
            }
            if constexpr (WN == 1) {
                if constexpr (AMX) row_absmax_store(g, row, tn, lr, amx);
                if (g.row_sumsq) {
#pragma unroll
                    for (int off = 16; off > 0; off >>= 1) ssq += __shfl_xor(ssq, off);
                    if (lr == 0 && row < g.M) g.row_sumsq[row * ROWSUMSQ_SLOTS + tn] = ssq;
                }
            }
        }
    }
    }  // !M16
}

// One tile per block (XCD-mapped tile order), or a persistent grid of one block per CU
// taking tiles from per-XCD counters in row-tile-major order (g.queue, as gemm_nt_h2g):
// beside the overlapped gather a persistent block keeps its LDS and registers.
// The tile ticket is passed through the first word of the (then idle) stage memory, so two
// 80 KB 4-wave blocks fit one CU's 160 KB.
// HELP: after the last tile every wave takes destination rows of the next chunk's gather
// (g.help, aggrow::agg_help_run) — the GEMM's CU slots would otherwise idle beside the gather's
// one block per CU until the chunk's gather ends.
#ifdef RVX_GEMM_CLOCK
// Diagnostic build only (scripts/exp/gemm_clock.sh): every block of gemm_nt_h2w adds its
// s_memtime and s_memrealtime deltas; the host prints the block-time-weighted clock per launch
// (MI355X_MICROARCH.md DVFS item 6: clock = d(s_memtime) / d(s_memrealtime) x 100 MHz).
__device__ unsigned long long g_gemm_clk[2];
struct GemmClockStamp {
    unsigned long long t0, r0;
    __device__ GemmClockStamp() : t0(__builtin_amdgcn_s_memtime()), r0(__builtin_amdgcn_s_memrealtime()) {}
    __device__ ~GemmClockStamp() {
        if (threadIdx.x == 0) {
            atomicAdd(&g_gemm_clk[0], __builtin_amdgcn_s_memtime() - t0);
            atomicAdd(&g_gemm_clk[1], __builtin_amdgcn_s_memrealtime() - r0);
        }
    }
};
#endif
template <bool DUAL, int WN, int BN, int NW = 8, bool PIPE = false, bool HELP = false, bool AMX = false,
          bool GATE = false, bool M16 = false>
__global__ __launch_bounds__(64 * NW, NW == 4 ? (PIPE ? 2 : 3) : 1) void gemm_nt_h2w(GemmArgs g, int epi) {
#ifdef RVX_GEMM_CLOCK
    GemmClockStamp clk_stamp;
#endif
    if (g.queue) {
        extern __shared__ __attribute__((aligned(16))) unsigned char xsm[];
        int64_t* s_t = reinterpret_cast<int64_t*>(xsm);
        const int64_t xcd = blockIdx.x % 8;
        const int64_t first = xcd_first(g.nblocks, xcd), cnt = xcd_count(g.nblocks, xcd);
        for (;;) {
            if (threadIdx.x == 0) *s_t = (int64_t)atomicAdd(g.queue + 32 * xcd, 1u);
            __syncthreads();
            const int64_t t = *s_t;
            __syncthreads();  // every wave holds t before the tile's DMA overwrites the word
            if (t >= cnt) break;
            h2w_tile<DUAL, WN, BN, NW, PIPE, AMX, GATE, M16>(g, epi, first + t);
            __syncthreads();  // LDS stages and s_t are reused by the next tile
        }
        // the loop ends after a barrier: the stage memory is free for the image windows
        if constexpr (HELP) aggrow::agg_help_run<true>(g.help, xsm);
        return;
    }
    const int64_t nwg = g.nblocks, bid = blockIdx.x;
    h2w_tile<DUAL, WN, BN, NW, PIPE, AMX, GATE, M16>(g, epi, xcd_first(nwg, bid % 8) + bid / 8);
    if constexpr (HELP) {
        extern __shared__ __attribute__((aligned(16))) unsigned char xsm_h[];
        __syncthreads();  // every wave is done with the tile's stages
        aggrow::agg_help_run<true>(g.help, xsm_h);
    }
}

// B rows n of one or two [N][K] matrices: common scale t_n, f16 planes of each
// (plane stride N*K), inv[n] = 1 / t_n. One wave per row.
__global__ __launch_bounds__(256) void k_split_h2_rows(const float* __restrict__ B0, const float* __restrict__ B1,
                                                       int N, int K, _Float16* __restrict__ P0,
                                                       _Float16* __restrict__ P1, float* __restrict__ inv) {
    const int lane = threadIdx.x & 63;
    const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (n >= N) return;
    float m = 0.0f;
    for (int k = lane; k < K; k += 64) {
        m = fmaxf(m, fabsf(B0[(int64_t)n * K + k]));
        if (B1) m = fmaxf(m, fabsf(B1[(int64_t)n * K + k]));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    const float t = h2_scale_dev(m);
    const int64_t plane = (int64_t)N * K;
    for (int k = lane; k < K; k += 64) {
        const int64_t i = (int64_t)n * K + k;
        const float x0 = B0[i] * t;
        const _Float16 h0 = (_Float16)x0;
        P0[i] = h0;
        P0[plane + i] = (_Float16)(x0 - (float)h0);
        if (B1) {
            const float x1 = B1[i] * t;
            const _Float16 h1 = (_Float16)x1;
            P1[i] = h1;
            P1[plane + i] = (_Float16)(x1 - (float)h1);
        }
    }
    if (lane == 0) inv[n] = 1.0f / t;
}

// Correctness path for shapes the tiled kernel cannot take (K % 4 != 0 or
// unaligned rows, e.g. the reference's 2-wide unit tests): one thread per
// output, k-sequential fma chain.
__global__ void gemm_nt_simple(GemmArgs g, int epi) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= g.M * (int64_t)g.N) return;
    const int64_t m = idx / g.N;
    const int n = (int)(idx % g.N);
    float acc = 0.0f;
    for (int k = 0; k < g.K0; ++k) acc = fmaf(g.A0[m * g.lda0 + k], g.B0[(int64_t)n * g.ldb0 + k], acc);
    if (g.A1)
        for (int k = 0; k < g.K1; ++k) acc = fmaf(g.A1[m * g.lda1 + k], g.B1[(int64_t)n * g.ldb1 + k], acc);
    if (g.alpha != 1.0f) acc *= g.alpha;
    if (g.bias0) acc += g.bias0[n] + (g.bias1 ? g.bias1[n] : 0.0f);
    else if (g.bias1) acc += g.bias1[n];
    if (g.addend) acc += g.addend[m * g.ld_add + n];
    g.C[m * g.ldc + n] = epi_apply(epi, acc);
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

void gemm_nt(int64_t M, int N, const GemmOperand& s0, const GemmOperand* s1, const GemmEpilogue& ep, float* C,
             int64_t ldc, const char* tag) {
    if (M <= 0 || N <= 0) return;
    const float* bias0 = ep.bias0;
    const float* bias1 = ep.bias1;
    const float alpha = ep.alpha;
    const int epi = ep.epi;
    GemmArgs g{};
    g.addend = ep.addend;
    g.ld_add = ep.ld_addend;
    g.A0 = s0.A; g.B0 = s0.B; g.lda0 = s0.lda; g.ldb0 = s0.ldb; g.K0 = s0.K;
    if (s1) { g.A1 = s1->A; g.B1 = s1->B; g.lda1 = s1->lda; g.ldb1 = s1->ldb; g.K1 = s1->K; }
    g.bias0 = bias0; g.bias1 = bias1; g.C = C; g.ldc = ldc; g.M = M; g.N = N; g.alpha = alpha;

    bool fast = (s0.K % 4 == 0) && (s0.lda % 4 == 0) && (s0.ldb % 4 == 0) && aligned16(s0.A) && aligned16(s0.B);
    if (s1) fast = fast && (s1->K % 4 == 0) && (s1->lda % 4 == 0) && (s1->ldb % 4 == 0) && aligned16(s1->A) &&
                   aligned16(s1->B);
    const char* t = tag ? tag : "gemm_nt";
    const int x3_mode = env_int("RVX_GEMM_X3", 1);  // read per call: bench times every GEMM path
    bool x3 = fast && x3_mode && s0.Bx3 && (s0.K % 8 == 0) && (s0.ldb % 8 == 0);
    if (s1) x3 = x3 && s1->Bx3 && (s1->K % 8 == 0) && (s1->ldb % 8 == 0);
    if (x3) {
        g.B0x3 = s0.Bx3; g.B0x3_plane = s0.Bx3_plane;
        if (s1) { g.B1x3 = s1->Bx3; g.B1x3_plane = s1->Bx3_plane; }
        const int use_dma = env_int("RVX_GEMM_DMA", 1);  // read per call: tests cover both tilings
        const int wm = env_int("RVX_GEMM_WM", 4) == 8 ? 8 : 4;  // 8: 256-row tile, one block / CU
        // the DMA kernel addresses each k-tile as scalar base + 32-bit lane offset
        const int bm = 32 * wm;
        auto offs_fit = [bm](const GemmOperand& o) {
            const int64_t lim = (int64_t)1 << 31;
            return (int64_t)bm * o.lda * 4 < lim && (2 * o.Bx3_plane + (int64_t)XBN * o.ldb) * 2 < lim;
        };
        const bool dma = use_dma && s0.K % 32 == 0 && offs_fit(s0) && (!s1 || (s1->K % 32 == 0 && offs_fit(*s1)));
        const int tile_m = dma ? bm : XBM;
        g.tiles_n = (N + XBN - 1) / XBN;
        const int64_t tiles_m = (M + tile_m - 1) / tile_m;
        g.nblocks = tiles_m * g.tiles_n;
        RVX_REQUIRE(g.nblocks < (int64_t)1 << 31, RVX_ERR_INVALID_SHAPE, "GEMM grid too large");
        const int lds_g = 2 * (bm * 128 + 3 * XB_PLANE);
        static bool attr = false;
        if (!attr) {
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_x3<true>, hipFuncAttributeMaxDynamicSharedMemorySize, X_LDS));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_x3<false>, hipFuncAttributeMaxDynamicSharedMemorySize, X_LDS));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_x3g<true, 4, false>, hipFuncAttributeMaxDynamicSharedMemorySize, X_LDS));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_x3g<false, 4, false>, hipFuncAttributeMaxDynamicSharedMemorySize, X_LDS));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_x3g<true, 4, true>, hipFuncAttributeMaxDynamicSharedMemorySize, X_LDS));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_x3g<false, 4, true>, hipFuncAttributeMaxDynamicSharedMemorySize, X_LDS));
            const int l8 = 2 * (256 * 128 + 3 * XB_PLANE);
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_x3g<true, 8, false>, hipFuncAttributeMaxDynamicSharedMemorySize, l8));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_x3g<false, 8, false>, hipFuncAttributeMaxDynamicSharedMemorySize, l8));
            attr = true;
        }
        const dim3 grid((unsigned)g.nblocks);
        if (dma) {
            const dim3 block(64 * wm);
            const int s16 = env_int("RVX_GEMM_MFMA16", 0);  // 16x16x32 MFMA form (128-row tile)
            if (s16 && s1) RVX_LAUNCH(t, (gemm_nt_x3g<true, 4, true>), grid, block, lds_g, g, epi);
            else if (s16) RVX_LAUNCH(t, (gemm_nt_x3g<false, 4, true>), grid, block, lds_g, g, epi);
            else if (wm == 8 && s1) RVX_LAUNCH(t, (gemm_nt_x3g<true, 8, false>), grid, block, lds_g, g, epi);
            else if (wm == 8) RVX_LAUNCH(t, (gemm_nt_x3g<false, 8, false>), grid, block, lds_g, g, epi);
            else if (s1) RVX_LAUNCH(t, (gemm_nt_x3g<true, 4, false>), grid, block, lds_g, g, epi);
            else RVX_LAUNCH(t, (gemm_nt_x3g<false, 4, false>), grid, block, lds_g, g, epi);
        } else if (s1) RVX_LAUNCH(t, gemm_nt_x3<true>, grid, dim3(256), X_LDS, g, epi);
        else RVX_LAUNCH(t, gemm_nt_x3<false>, grid, dim3(256), X_LDS, g, epi);
        return;
    }
    if (fast) {
        g.tiles_n = (N + BN - 1) / BN;
        const int64_t tiles_m = (M + BM - 1) / BM;
        g.nblocks = tiles_m * g.tiles_n;
        RVX_REQUIRE(g.nblocks < (int64_t)1 << 31, RVX_ERR_INVALID_SHAPE, "GEMM grid too large");
        static const int depth = env_int("RVX_GEMM_DEPTH", 1);
        const dim3 grid((unsigned)g.nblocks), block(256);
        if (s1 && depth >= 2) RVX_LAUNCH(t, (gemm_nt_mfma<true, 2>), grid, block, 0, g, epi);
        else if (s1) RVX_LAUNCH(t, (gemm_nt_mfma<true, 1>), grid, block, 0, g, epi);
        else if (depth >= 2) RVX_LAUNCH(t, (gemm_nt_mfma<false, 2>), grid, block, 0, g, epi);
        else RVX_LAUNCH(t, (gemm_nt_mfma<false, 1>), grid, block, 0, g, epi);
    } else {
        const int64_t total = M * (int64_t)N;
        RVX_LAUNCH(t, gemm_nt_simple, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, g, epi);
    }
}

bool gemm_h2_ok(int64_t M, int N, const GemmOperand& s0, const GemmOperand* s1) {
    if (!env_int("RVX_GEMM_H2", 1) || M <= 0 || N <= 0) return false;  // read per call: tests cover both GEMMs
    auto ok = [N](const GemmOperand& o) {
        const int64_t lim = (int64_t)1 << 31;
        const int64_t plane = o.Bh_plane ? o.Bh_plane : (int64_t)o.ldb * N;
        return o.K % 32 == 0 && o.lda % 4 == 0 && o.ldb % 8 == 0 && aligned16(o.A) && (int64_t)128 * o.lda * 4 < lim &&
               (plane + (int64_t)XBN * o.ldb) * 2 < lim;
    };
    return ok(s0) && (!s1 || ok(*s1));
}

// Opt-in (RVX_GEMM_ROWNORM=1, read per call; tests force both): bit-identical, but in the
// overlapped 10M x 768 layer the per-tile agent-scope release (an L2 write-back beside the
// gather's stores) costs more than the pass it removes: 491-526 vs 457-465 ms/step
// (scripts/exp_rownorm_ab.sh, profiles/r03_sage_rownorm_ab.txt).
bool gemm_h2_rownorm_ok(int N, const float* C, int64_t ldc) {
    return env_int("RVX_GEMM_ROWNORM", 0) && N % 4 == 0 && N <= 1024 && ldc % 4 == 0 && aligned16(C);
}

int gemm_nt_h2(int64_t M, int N, const GemmOperand& s0, const _Float16* B0h, const GemmOperand* s1,
               const _Float16* B1h, const float* a_scale, const float* b_inv, const GemmEpilogue& ep, float* C,
               int64_t ldc, const char* tag, int persist) {
    if (M <= 0 || N <= 0) return 0;
    GemmArgs g{};
    g.addend = ep.addend;
    g.ld_add = ep.ld_addend;
    g.A0 = s0.A; g.lda0 = s0.lda; g.ldb0 = s0.ldb; g.K0 = s0.K;
    g.B0h = B0h; g.B0h_plane = s0.Bh_plane ? s0.Bh_plane : (int64_t)N * s0.ldb;
    if (s1) {
        g.A1 = s1->A; g.lda1 = s1->lda; g.ldb1 = s1->ldb; g.K1 = s1->K; g.B1h = B1h;
        g.B1h_plane = s1->Bh_plane ? s1->Bh_plane : (int64_t)N * s1->ldb;
    }
    g.bias0 = ep.bias0; g.bias1 = ep.bias1; g.C = C; g.ldc = ldc; g.M = M; g.N = N; g.alpha = ep.alpha;
    g.a_scale = a_scale; g.b_inv = b_inv;
    g.row_sumsq = ep.row_sumsq; g.a1_rowmul = ep.a1_rowmul;
    RVX_REQUIRE(gemm_h2_ok(M, N, s0, s1), RVX_ERR_INVALID_SHAPE, "shape not supported by the split-f16 GEMM");
    RVX_REQUIRE(!ep.a1_rowmul || s1, RVX_ERR_INVALID_PARAMETER, "a1_rowmul needs a dual GEMM");
    g.tiles_n = (N + XBN - 1) / XBN;
    g.nblocks = ((M + 127) / 128) * g.tiles_n;
    RVX_REQUIRE(g.nblocks < (int64_t)1 << 31, RVX_ERR_INVALID_SHAPE, "GEMM grid too large");
    constexpr int lds = 2 * (128 * 128 + 2 * XB_PLANE);
    static bool attr = false;
    if (!attr) {
        RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2g<true>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2g<false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        attr = true;
    }
    const char* t = tag ? tag : "gemm_nt_h2";
    // Wide tiles (gemm_nt_h2w, bit-identical to h2g). Standalone launches: 256 x 256, 8 waves
    // along M (78.7-80.3 vs 87.2 ms for the 10M x 768 SAGE GEMM alone). The persistent GEMM
    // beside the gather (persist > 0): 256 x 192 (161 VGPRs, so two GEMM waves and a 152-VGPR
    // gather wave share each SIMD; the 256-wide tile's 193+ VGPRs do not fit and lost, 487 vs
    // 454 ms/step): 403-451 vs 455-470 ms/step for h2g (scripts/exp_wide3_pipe.sh).
    // RVX_GEMM_WIDE (read per call; tests cover all): 0 h2g, 1 waves 2 x 4, 2 waves 8 x 1,
    // 3 waves 8 x 1 on 256 x 192 tiles (32 x 192 per wave: 96 accumulator registers),
    // 4 the same rows on 4-wave 128 x 192 blocks, 5 / 6 / 7 the software-pipelined K loop on
    // 256 x 192 / 256 x 256 / 4-wave 128 x 192 (two blocks per CU, each its own barriers).
    // Standalone defaults: 7 for one operand (C4's K = 768 GEMMs: msg 26.9 vs 28.2 ms per 2M
    // step with 6), 6 for two (the dual zr / h GEMMs 95.5 / 46.7 vs 99.8 / 48.0 ms with 7, the
    // 10M GraphSAGE GEMM 72.8 vs 77.2 ms; scripts/exp_gemm_pipe.sh, profiles/r03_gemm_pipe_ab.txt).
    const int wide_mode = env_int("RVX_GEMM_WIDE", persist > 0 ? 3 : (s1 && !ep.gate_out ? 6 : 7));  // gate: 7 (registers)
    const bool same_strides = !s1 || (g.lda1 == g.lda0 && g.ldb1 == g.ldb0 && g.B1h_plane == g.B0h_plane);
    const bool wide = !ep.normalize_rows && (wide_mode >= 2 || (!ep.row_sumsq && !ep.a1_rowmul)) && wide_mode &&
                      same_strides && (int64_t)256 * g.lda0 * 4 < ((int64_t)1 << 31) &&
                      (!s1 || (int64_t)256 * g.lda1 * 4 < ((int64_t)1 << 31)) &&
                      (g.B0h_plane + (int64_t)256 * g.ldb0) * 2 < ((int64_t)1 << 31) &&
                      (!s1 || (g.B1h_plane + (int64_t)256 * g.ldb1) * 2 < ((int64_t)1 << 31));
    if (wide) {
        const int wbn = wide_mode == 3 || wide_mode == 4 || wide_mode == 5 || wide_mode == 7 ? 192 : 256;  // 5 / 6: 256 x 192 / 256 x 256, software-pipelined K loop
        const int wbm = wide_mode == 4 || wide_mode == 7 ? 128 : 256;  // 4: 4-wave blocks (one GEMM wave per SIMD)
        const int wlds = 2 * (wbm * 128 + 2 * wbn * 64);
        static bool wattr = false;
        if (!wattr) {
            constexpr int l256 = 2 * (256 * 128 + 2 * 256 * 64), l192 = 2 * (256 * 128 + 2 * 192 * 64);
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<true, 4, 256>, hipFuncAttributeMaxDynamicSharedMemorySize, l256));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<false, 4, 256>, hipFuncAttributeMaxDynamicSharedMemorySize, l256));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<true, 1, 256>, hipFuncAttributeMaxDynamicSharedMemorySize, l256));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<false, 1, 256>, hipFuncAttributeMaxDynamicSharedMemorySize, l256));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<true, 1, 192>, hipFuncAttributeMaxDynamicSharedMemorySize, l192));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<false, 1, 192>, hipFuncAttributeMaxDynamicSharedMemorySize, l192));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<true, 1, 256, 8, true, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l256));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<false, 1, 256, 8, true, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l256));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<true, 1, 192, 8, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l192));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<false, 1, 192, 8, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l192));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<true, 1, 192, 8, false, true, false, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l192));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<false, 1, 192, 8, false, true, false, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l192));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<true, 1, 192, 8, false, false, false, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l192));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<false, 1, 192, 8, false, false, false, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l192));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<true, 1, 256, 8, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l256));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<false, 1, 256, 8, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l256));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<true, 1, 192, 8, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l192));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<false, 1, 192, 8, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l192));
            constexpr int l4 = 2 * (128 * 128 + 2 * 192 * 64);
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<true, 1, 192, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, l4));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<false, 1, 192, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, l4));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<true, 1, 192, 4, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l4));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<false, 1, 192, 4, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l4));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<true, 1, 192, 4, true, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l4));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<true, 1, 192, 4, true, false, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l4));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<false, 1, 192, 4, true, false, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l4));
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2w<false, 1, 192, 4, true, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l4));
            wattr = true;
        }
        g.tiles_n = (N + wbn - 1) / wbn;
        g.nblocks = ((M + wbm - 1) / wbm) * g.tiles_n;
        RVX_REQUIRE(!ep.row_sumsq || g.tiles_n <= ROWSUMSQ_SLOTS, RVX_ERR_INVALID_SHAPE, "row sums: N too large");
        RVX_REQUIRE(g.nblocks < (int64_t)1 << 31, RVX_ERR_INVALID_SHAPE, "GEMM grid too large");
        // persistent (one block per CU, per-XCD tile queue) when asked for, as h2g
        const int wcap = persist >= 0 ? persist : env_int("RVX_GEMM_CAP", 0);
        int64_t wgrid = g.nblocks;
        if (wcap > 0) wgrid = std::min<int64_t>(wgrid, ((int64_t)(wbm == 128 ? 2 : 1) * active_cus() + 7) / 8 * 8);  // 4-wave blocks: two per CU
        if (wgrid < g.nblocks && wgrid % 8 == 0) {
            g.queue = (unsigned*)scratch_bytes("gemm_h2_queue", 8 * 32 * 4);
            RVX_HIP(hipMemsetAsync(g.queue, 0, 8 * 32 * 4, stream()));
        } else {
            wgrid = g.nblocks;
        }
        // row maxima from the epilogue on the standalone defaults (6, 7); other tiles: a pass
        g.row_absmax = (ep.row_absmax && (wide_mode == 6 || wide_mode == 7) && g.tiles_n <= ROWSUMSQ_SLOTS)
                           ? ep.row_absmax : nullptr;
        const bool amx = g.row_absmax != nullptr;
        const bool gate = amx && ep.gate_out && wide_mode == 7;  // the 4-wave tile has the registers for it
        if (gate) {
            g.gate_h = ep.gate_h; g.ld_gate_h = ep.ld_gate_h; g.gate_out = ep.gate_out;
            g.ld_gate_out = ep.ld_gate_out; g.gate_col0 = ep.gate_col0;
        }
        const dim3 wg((unsigned)wgrid), wb(wide_mode == 4 || wide_mode == 7 ? 256 : 512);
        // the 256 x 192 tile on 16x16x32 MFMAs (RVX_GEMM_M16, read per call; tests cover both)
        const bool m16 = env_int("RVX_GEMM_M16", 0) != 0;
        // RVX_GEMM_WIDE=1: waves 2 (M) x 4 (N), 128 x 64 each; 2: waves 8 x 1, 32 x 256 each
        // (A converted once per row instead of by four waves)
        if (gate) {
            if (s1) RVX_LAUNCH(t, (gemm_nt_h2w<true, 1, 192, 4, true, false, true, true>), wg, wb, wlds, g, ep.epi);
            else RVX_LAUNCH(t, (gemm_nt_h2w<false, 1, 192, 4, true, false, true, true>), wg, wb, wlds, g, ep.epi);
        } else if (wide_mode == 7 && amx) {
            if (s1) RVX_LAUNCH(t, (gemm_nt_h2w<true, 1, 192, 4, true, false, true>), wg, wb, wlds, g, ep.epi);
            else RVX_LAUNCH(t, (gemm_nt_h2w<false, 1, 192, 4, true, false, true>), wg, wb, wlds, g, ep.epi);
        } else if (wide_mode == 6 && amx) {
            if (s1) RVX_LAUNCH(t, (gemm_nt_h2w<true, 1, 256, 8, true, false, true>), wg, wb, wlds, g, ep.epi);
            else RVX_LAUNCH(t, (gemm_nt_h2w<false, 1, 256, 8, true, false, true>), wg, wb, wlds, g, ep.epi);
        } else if (wide_mode == 7) {
            if (s1) RVX_LAUNCH(t, (gemm_nt_h2w<true, 1, 192, 4, true>), wg, wb, wlds, g, ep.epi);
            else RVX_LAUNCH(t, (gemm_nt_h2w<false, 1, 192, 4, true>), wg, wb, wlds, g, ep.epi);
        } else if (wide_mode == 6) {
            if (s1) RVX_LAUNCH(t, (gemm_nt_h2w<true, 1, 256, 8, true>), wg, wb, wlds, g, ep.epi);
            else RVX_LAUNCH(t, (gemm_nt_h2w<false, 1, 256, 8, true>), wg, wb, wlds, g, ep.epi);
        } else if (wide_mode == 5) {
            if (s1) RVX_LAUNCH(t, (gemm_nt_h2w<true, 1, 192, 8, true>), wg, wb, wlds, g, ep.epi);
            else RVX_LAUNCH(t, (gemm_nt_h2w<false, 1, 192, 8, true>), wg, wb, wlds, g, ep.epi);
        } else if (wide_mode == 4) {
            if (s1) RVX_LAUNCH(t, (gemm_nt_h2w<true, 1, 192, 4>), wg, wb, wlds, g, ep.epi);
            else RVX_LAUNCH(t, (gemm_nt_h2w<false, 1, 192, 4>), wg, wb, wlds, g, ep.epi);
        } else if (wide_mode == 3 && m16 && ep.help && ep.help->n > 0) {
            g.help = *ep.help;
            if (s1) RVX_LAUNCH(t, (gemm_nt_h2w<true, 1, 192, 8, false, true, false, false, true>), wg, wb, wlds, g, ep.epi);
            else RVX_LAUNCH(t, (gemm_nt_h2w<false, 1, 192, 8, false, true, false, false, true>), wg, wb, wlds, g, ep.epi);
        } else if (wide_mode == 3 && m16) {
            if (s1) RVX_LAUNCH(t, (gemm_nt_h2w<true, 1, 192, 8, false, false, false, false, true>), wg, wb, wlds, g, ep.epi);
            else RVX_LAUNCH(t, (gemm_nt_h2w<false, 1, 192, 8, false, false, false, false, true>), wg, wb, wlds, g, ep.epi);
        } else if (wide_mode == 3 && ep.help && ep.help->n > 0) {
            g.help = *ep.help;
            if (s1) RVX_LAUNCH(t, (gemm_nt_h2w<true, 1, 192, 8, false, true>), wg, wb, wlds, g, ep.epi);
            else RVX_LAUNCH(t, (gemm_nt_h2w<false, 1, 192, 8, false, true>), wg, wb, wlds, g, ep.epi);
        } else if (wide_mode == 3) {
            if (s1) RVX_LAUNCH(t, (gemm_nt_h2w<true, 1, 192>), wg, wb, wlds, g, ep.epi);
            else RVX_LAUNCH(t, (gemm_nt_h2w<false, 1, 192>), wg, wb, wlds, g, ep.epi);
        } else if (wide_mode == 2) {
            if (s1) RVX_LAUNCH(t, (gemm_nt_h2w<true, 1, 256>), wg, wb, wlds, g, ep.epi);
            else RVX_LAUNCH(t, (gemm_nt_h2w<false, 1, 256>), wg, wb, wlds, g, ep.epi);
        } else {
            if (s1) RVX_LAUNCH(t, (gemm_nt_h2w<true, 4, 256>), wg, wb, wlds, g, ep.epi);
            else RVX_LAUNCH(t, (gemm_nt_h2w<false, 4, 256>), wg, wb, wlds, g, ep.epi);
        }
#ifdef RVX_GEMM_CLOCK
        {
            static unsigned long long prev[2] = {0, 0};
            unsigned long long h[2];
            sync();
            RVX_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_gemm_clk), sizeof h));
            const double dt = (double)(h[0] - prev[0]), dr = (double)(h[1] - prev[1]);
            if (dr > 0)
                std::fprintf(stderr, "[gemm clock] %s: %.3f GHz (block-time weighted, %.1f block-ms)\n", t,
                             dt / dr * 0.1, dr * 1e-5);
            prev[0] = h[0]; prev[1] = h[1];
        }
#endif
        if (ep.gate_out && !g.gate_out)
            mul_rows(C + ep.gate_col0, ldc, ep.gate_h, ep.gate_out, M, N - ep.gate_col0, ep.row_absmax);
        else if (ep.row_absmax && !g.row_absmax)
            row_absmax_pass(C, ldc, M, N, ep.row_absmax);
        return g.tiles_n;
    }
    // persistent grid of `cap` blocks per CU (a multiple of 8 blocks, so a block
    // keeps its XCD across the tiles it strides over). The overlapped GraphSAGE
    // GEMM asks for 2 (every resident slot, no block turnover beside the gather:
    // +2% per step, scripts/exp_gemm_cap.sh); standalone GEMMs are 6-13% faster
    // with one block per tile (C4 layer GEMMs), so that stays the default.
    const int cap = persist >= 0 ? persist : env_int("RVX_GEMM_CAP", 0);
    int64_t grid = g.nblocks;
    if (cap > 0) grid = std::min<int64_t>(grid, ((int64_t)cap * active_cus() + 7) / 8 * 8);
    if (grid < g.nblocks && grid % 8 == 0 && env_int("RVX_GEMM_QUEUE", 1)) {
        g.queue = (unsigned*)scratch_bytes("gemm_h2_queue", 8 * 32 * 4);
        RVX_HIP(hipMemsetAsync(g.queue, 0, 8 * 32 * 4, stream()));
        // XCD pairs split the column tiles: each L2 holds half of W's f16 planes
        // (10M x 768 layer: GEMM fetch 10.5 -> 7.7 GB per launch, step time
        // unchanged within noise, scripts/exp_xsplit.sh); RVX_GEMM_XSPLIT=0 restores
        g.xsplit = (g.tiles_n % 2 == 0 && g.nblocks % g.tiles_n == 0) ? env_int("RVX_GEMM_XSPLIT", 1) : 0;
    }
    if (ep.normalize_rows) {
        RVX_REQUIRE(gemm_h2_rownorm_ok(N, C, ldc), RVX_ERR_INVALID_SHAPE, "row normalisation needs N % 4 == 0, N <= 1024");
        const int64_t tiles_m = (M + 127) / 128;
        g.row_tickets = (unsigned*)scratch_bytes("gemm_h2_row_tickets", tiles_m * 4);
        RVX_HIP(hipMemsetAsync(g.row_tickets, 0, (size_t)tiles_m * 4, stream()));
    }
    g.row_absmax = nullptr;  // h2g: row maxima by a pass over C
    if (s1) RVX_LAUNCH(t, gemm_nt_h2g<true>, dim3((unsigned)grid), dim3(256), lds, g, ep.epi);
    else RVX_LAUNCH(t, gemm_nt_h2g<false>, dim3((unsigned)grid), dim3(256), lds, g, ep.epi);
    if (ep.gate_out)
        mul_rows(C + ep.gate_col0, ldc, ep.gate_h, ep.gate_out, M, N - ep.gate_col0, ep.row_absmax);
    else if (ep.row_absmax && !g.row_absmax)
        row_absmax_pass(C, ldc, M, N, ep.row_absmax);
    return g.tiles_n;
}

bool gemm_h2p_ok(int64_t M, int N, int64_t lda, int64_t a_plane, const GemmOperand& s0, const GemmOperand* s1) {
    // read per call so tests cover every path; RVX_GEMM_H2=0 turns off both split-f16 kernels
    // (opt-in: no faster than h2g in the 10M x 768 layer, which runs power-capped at ~1.9 GHz in every
    // tiling tried, scripts/exp_h2p.sh)
    if (!env_int("RVX_GEMM_H2P", 0) || !env_int("RVX_GEMM_H2", 1) || M <= 0 || N <= 0) return false;
    const int64_t lim = (int64_t)1 << 31;
    auto ok = [&](const GemmOperand& o) {
        const int64_t plane = o.Bh_plane ? o.Bh_plane : (int64_t)o.ldb * N;
        return o.K % 32 == 0 && o.ldb % 8 == 0 && (plane + (int64_t)XBN * o.ldb) * 2 < lim;
    };
    return lda % 8 == 0 && (a_plane + 256 * lda) * 2 < lim && ok(s0) && (!s1 || ok(*s1));
}

void gemm_nt_h2p(int64_t M, int N, const _Float16* Ah, int64_t lda, int64_t a_plane, const GemmOperand& s0,
                 const _Float16* B0h, const GemmOperand* s1, const _Float16* B1h, const float* a_scale,
                 const float* b_inv, const GemmEpilogue& ep, float* C, int64_t ldc, const char* tag) {
    if (M <= 0 || N <= 0) return;
    RVX_REQUIRE(gemm_h2p_ok(M, N, lda, a_plane, s0, s1) && aligned16(Ah), RVX_ERR_INVALID_SHAPE,
                "shape not supported by the pre-split f16 GEMM");
    GemmArgs g{};
    g.addend = ep.addend;
    g.ld_add = ep.ld_addend;
    g.A0h = Ah; g.lda0 = lda; g.ldb0 = s0.ldb; g.K0 = s0.K; g.Ah_plane = a_plane;
    g.B0h = B0h; g.B0h_plane = s0.Bh_plane ? s0.Bh_plane : (int64_t)N * s0.ldb;
    if (s1) {
        g.A1h = Ah + s0.K; g.lda1 = lda; g.ldb1 = s1->ldb; g.K1 = s1->K; g.B1h = B1h;
        g.B1h_plane = s1->Bh_plane ? s1->Bh_plane : (int64_t)N * s1->ldb;
    }
    g.bias0 = ep.bias0; g.bias1 = ep.bias1; g.C = C; g.ldc = ldc; g.M = M; g.N = N; g.alpha = ep.alpha;
    g.a_scale = a_scale; g.b_inv = b_inv;
    // RVX_GEMM_H2P_CFG: 0 = 128x128, 2 stages, 2 blocks/CU; 1 = 256x128, 3 stages; 2 = 128x128, 3 stages;
    // 3 = 256x128, 2 stages (one block of 8 or 4 waves per CU for 1-3)
    const int cfg = env_int("RVX_GEMM_H2P_CFG", 0);
    const int bm = (cfg == 1 || cfg == 3) ? 256 : 128;
    g.tiles_n = (N + XBN - 1) / XBN;
    g.nblocks = ((M + bm - 1) / bm) * g.tiles_n;
    RVX_REQUIRE(g.nblocks < (int64_t)1 << 31, RVX_ERR_INVALID_SHAPE, "GEMM grid too large");
    const char* t = tag ? tag : "gemm_nt_h2p";
#define RVX_H2P(WM, NST)                                                                                           \
    do {                                                                                                           \
        constexpr int lds = NST * (2 * 32 * WM * 64 + 2 * XB_PLANE);                                               \
        static bool attr = false;                                                                                  \
        if (!attr) {                                                                                               \
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2p<true, WM, NST>,                                   \
                                        hipFuncAttributeMaxDynamicSharedMemorySize, lds));                         \
            RVX_HIP(hipFuncSetAttribute((const void*)gemm_nt_h2p<false, WM, NST>,                                  \
                                        hipFuncAttributeMaxDynamicSharedMemorySize, lds));                         \
            attr = true;                                                                                           \
        }                                                                                                          \
        if (s1) RVX_LAUNCH(t, (gemm_nt_h2p<true, WM, NST>), dim3((unsigned)g.nblocks), dim3(64 * WM), lds, g, ep.epi); \
        else RVX_LAUNCH(t, (gemm_nt_h2p<false, WM, NST>), dim3((unsigned)g.nblocks), dim3(64 * WM), lds, g, ep.epi); \
    } while (0)
    if (cfg == 1) RVX_H2P(8, 3);
    else if (cfg == 2) RVX_H2P(4, 3);
    else if (cfg == 3) RVX_H2P(8, 2);
    else RVX_H2P(4, 2);
#undef RVX_H2P
}

namespace {
// One wave per row: max |a| over A0's and A1's row -> h2_scale_dev.
__global__ __launch_bounds__(256) void k_row_scale_h2(const float* __restrict__ A0, int64_t lda0, int K0,
                                                     const float* __restrict__ A1, int64_t lda1, int K1, int64_t M,
                                                     float* __restrict__ scale) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    float m = 0.0f;
    const float* a0 = A0 + row * lda0;
    for (int k = 4 * lane; k < K0; k += 256) {
        const float4 v = *reinterpret_cast<const float4*>(a0 + k);
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    if (A1) {
        const float* a1 = A1 + row * lda1;
        for (int k = 4 * lane; k < K1; k += 256) {
            const float4 v = *reinterpret_cast<const float4*>(a1 + k);
            m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane == 0) scale[row] = h2_scale_dev(m);
}
}  // namespace

namespace {
// Row scales from the producers' per-row partial maxima (GemmOperand::amax): one thread
// per row, max over both operands' ROWSUMSQ_SLOTS slots -> h2_scale_dev, the value
// k_row_scale_h2 computes from the rows themselves.
__global__ __launch_bounds__(256) void k_row_scale_amax(const float* __restrict__ a0, const float* __restrict__ a1,
                                                       int64_t M, float* __restrict__ scale) {
    const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (row >= M) return;
    static_assert(ROWSUMSQ_SLOTS == 8, "two float4 per row");
    const float4* p = reinterpret_cast<const float4*>(a0 + row * ROWSUMSQ_SLOTS);
    float4 u = p[0], v = p[1];
    float m = fmaxf(fmaxf(fmaxf(u.x, u.y), fmaxf(u.z, u.w)), fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
    if (a1) {
        p = reinterpret_cast<const float4*>(a1 + row * ROWSUMSQ_SLOTS);
        u = p[0]; v = p[1];
        m = fmaxf(m, fmaxf(fmaxf(fmaxf(u.x, u.y), fmaxf(u.z, u.w)), fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w))));
    }
    scale[row] = h2_scale_dev(fmaxf(m, 0.0f));
}

// Fallback for GEMM paths without the epilogue form: one wave per row of C, max |v| into
// slot 0, the other slots 0.
__global__ __launch_bounds__(256) void k_row_absmax(const float* __restrict__ C, int64_t ldc, int64_t M, int N,
                                                   float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    float m = 0.0f;
    for (int k = lane; k < N; k += 64) m = fmaxf(m, fabsf(C[row * ldc + k]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane < ROWSUMSQ_SLOTS) out[row * ROWSUMSQ_SLOTS + lane] = lane == 0 ? m : 0.0f;
}
}  // namespace

void row_absmax_pass(const float* C, int64_t ldc, int64_t M, int N, float* out) {
    if (M <= 0) return;
    RVX_LAUNCH("gemm_row_absmax", k_row_absmax, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, C, ldc, M, N, out);
}

void row_scale_h2(const float* A0, int64_t lda0, int K0, const float* A1, int64_t lda1, int K1, int64_t M,
                  float* scale) {
    if (M <= 0) return;
    RVX_LAUNCH("gemm_row_scale", k_row_scale_h2, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, A0, lda0, K0, A1, lda1,
               K1, M, scale);
}

void gemm_auto(int64_t M, int N, const GemmOperand& s0, const GemmOperand* s1, const GemmEpilogue& ep, float* C,
               int64_t ldc, const char* tag) {
    const bool planes = s0.Bh && s0.b_inv && (!s1 || (s1->Bh && s1->b_inv == s0.b_inv));
    if (planes && env_int("RVX_GNN_H2", 1) && gemm_h2_ok(M, N, s0, s1)) {  // read per call: tests cover both
        float* scale = scratch_f32("gemm_auto_scale", M);
        if (s0.amax && (!s1 || s1->amax) && env_int("RVX_GEMM_AMAX", 1))  // read per call: tests cover both
            RVX_LAUNCH("gemm_row_scale_amax", k_row_scale_amax, dim3((unsigned)((M + 255) / 256)), dim3(256), 0,
                       s0.amax, s1 ? s1->amax : nullptr, M, scale);
        else
            row_scale_h2(s0.A, s0.lda, s0.K, s1 ? s1->A : nullptr, s1 ? s1->lda : 0, s1 ? s1->K : 0, M, scale);
        gemm_nt_h2(M, N, s0, s0.Bh, s1, s1 ? s1->Bh : nullptr, scale, s0.b_inv, ep, C, ldc, tag);
        return;
    }
    gemm_nt(M, N, s0, s1, ep, C, ldc, tag);
    if (ep.gate_out)
        mul_rows(C + ep.gate_col0, ldc, ep.gate_h, ep.gate_out, M, N - ep.gate_col0, ep.row_absmax);
    else if (ep.row_absmax)
        row_absmax_pass(C, ldc, M, N, ep.row_absmax);
}

void split_h2_rows(const float* B0, const float* B1, int N, int K, _Float16* P0, _Float16* P1, float* inv) {
    if (N <= 0) return;
    RVX_LAUNCH("split_h2", k_split_h2_rows, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, B0, B1, N, K, P0, P1, inv);
}

}  // namespace rvx

namespace rvx {
void split_x3(const float* src, int64_t n, uint16_t* dst) {
    if (n <= 0) return;
    RVX_LAUNCH("split_x3", k_split_x3, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, src, n, dst);
}
}  // namespace rvx
