// k_sage_gemm.hip — the GraphSAGE layer's dual GEMM with the ReLU and the row L2
// normalisation fused, one block per 64 output rows x ALL output columns
// (crates/ruvector-postgres/src/gnn/graphsage.rs:151-184: relu(x̄ W_n + x W_s), then
// output / ||output|| when normalize).
//
// Why a full-width tile. The layer is HBM-bound: per row chunk the gather streams
// ~42 GB of random neighbour rows while the GEMM beside it moved 8.9 GB (the A operand
// [aggregate | self] fetched ~3x, once per XCD pair and again when the column tiles of
// a row tile drift apart) and the separate normalise pass another 2.56 GB. Here a
// block owns 64 rows and every output column: A is read from HBM exactly once, the
// output row is complete inside the block, so ReLU + normalisation happen in the
// epilogue and y is written once (coalesced 16-B row stores). The price is that every
// block streams all of W (2 x 768 x 1536 f16 planes = 4.7 MB) from L2 / Infinity
// Cache: 64 rows per 4.7 MB, the same W bytes per MFMA as the 128x128 tile of h2g.
//
// Bits. The split-f16 arithmetic is h2g's (gemm_f32.hip): A rows scaled by the
// gather's per-row power of two and split round-to-nearest into two f16 planes, the
// pre-split f16 planes of W, per 16-deep k step the three MFMAs a2b1, a1b2, a1b1 in
// that order, phase 0 (aggregate x W_n) then phase 1 (self x W_s), the epilogue
// (acc * 1/scale_row) * 1/scale_col then ReLU. The normalisation reproduces
// normalize_rows_vec<N/256> (k_data.hip): lane l sums the squares of columns
// 4l + 256j (j ascending, x y z w), a butterfly over the wave, sqrtf, true
// division, rows with norm 0 left as they are. So y is bit-identical to
// gemm_nt_h2 + normalize_rows — the tests compare bits.
//
// Tiling (CDNA4): 512 threads = 8 waves; wave w owns all 64 rows x columns
// [32 TN w, 32 TN (w+1)) as 2 x TN accumulators of v_mfma_f32_32x32x16_f16
// (TN = N / 256). Per 16-deep k step the stage holds A (64 rows x 16 f32, 4 KB) and
// both W planes (N x 16 f16 each, 48 KB at N = 768), filled by LDS-DMA
// (global_load_lds_dwordx4) with the 16-B chunk XOR swizzle applied to the source
// address: A chunk c of row r at position c ^ ((r >> 2) & 3), W chunk c of column n at
// c ^ ((n >> 3) & 1) — the ds_read_b128 fragment reads are bank-conflict free. Two
// stages (104 KB); the epilogue reuses them for a 32-row f32 image of the output.
#include "common.hpp"
#include "kernels.hpp"

namespace rvx {
namespace {

typedef _Float16 f16x8s __attribute__((ext_vector_type(8)));
typedef float f32x16s __attribute__((ext_vector_type(16)));
typedef unsigned u32x4s __attribute__((ext_vector_type(4)));

struct SageGemmArgs {
    const float* A0; int64_t lda0; int K0;   // aggregate rows [M][lda0]
    const float* A1; int64_t lda1; int K1;   // self rows [M][lda1]
    const _Float16* B0h; const _Float16* B1h; int64_t ldb0, ldb1, plane0, plane1;  // W planes [2][N][K]
    const float* a_scale;                    // [M] power-of-two row scale (gather)
    const float* b_inv;                      // [N] 1 / column scale
    float* C; int64_t ldc;                   // [M][ldc]
    int64_t M; int N; int normalize;
};

__device__ __forceinline__ void split_pair_h2(float a0, float a1, float sc, unsigned& w1, unsigned& w2) {
    const float x0 = a0 * sc, x1 = a1 * sc;
    const _Float16 h0 = (_Float16)x0, h1 = (_Float16)x1;
    const _Float16 l0 = (_Float16)(x0 - (float)h0), l1 = (_Float16)(x1 - (float)h1);
    w1 = (unsigned)__builtin_bit_cast(unsigned short, h0) | ((unsigned)__builtin_bit_cast(unsigned short, h1) << 16);
    w2 = (unsigned)__builtin_bit_cast(unsigned short, l0) | ((unsigned)__builtin_bit_cast(unsigned short, l1) << 16);
}

__device__ __forceinline__ float f8_at(const float4& lo, const float4& hi, int i) {
    switch (i) {
        case 0: return lo.x; case 1: return lo.y; case 2: return lo.z; case 3: return lo.w;
        case 4: return hi.x; case 5: return hi.y; case 6: return hi.z; default: return hi.w;
    }
}

constexpr int SG_ROWS = 64;
constexpr int SG_A = SG_ROWS * 64;  // A stage bytes: 64 rows x 16 f32
constexpr int SG_YSTRIDE_PAD = 8;   // output image row stride N + 8 floats (rows r, r+4 on opposite bank halves)

template <int TN>
struct SgCfg {
    static constexpr int N = 256 * TN;
    static constexpr int BPL = N * 32;               // one W plane per stage: N columns x 32 B
    static constexpr int STAGE = SG_A + 2 * BPL;
    static constexpr int LDS = 2 * STAGE;
    static constexpr int BPIECES = 2 * BPL / 1024;   // 1-KiB DMA pieces of W per stage
    static_assert(32 * (N + SG_YSTRIDE_PAD) * 4 <= LDS, "output image fits the stages");
    static_assert(BPIECES % 8 == 0, "W pieces split evenly over the 8 waves");
};

template <int TN>
__global__ __launch_bounds__(512) void k_sage_gemm_fused(SageGemmArgs g) {
    using Cf = SgCfg<TN>;
    extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 31, lh = lane >> 5;
    const int64_t m0 = (int64_t)blockIdx.x * SG_ROWS;
    const int c0w = wave * 32 * TN;  // this wave's first column

    // ---- DMA sources: wave-uniform base + per-lane 32-bit offsets
    // A piece j (waves 0..3): rows 16j + lane/4, position lane%4 -> chunk (lane%4) ^ sw(row)
    uint32_t a_off[2] = {0, 0};
    const int a_row = 16 * wave + (lane >> 2);
    if (wave < 4) {
        const int64_t rr = min<int64_t>(m0 + a_row, g.M - 1) - m0;
        const int chunk = (lane & 3) ^ ((a_row >> 2) & 3);
        a_off[0] = (uint32_t)((rr * g.lda0 + 4 * chunk) * 4);
        a_off[1] = (uint32_t)((rr * g.lda1 + 4 * chunk) * 4);
    }
    // W pieces: piece p (of BPIECES) = plane p / (BPL/1024), columns 32 (p % per_plane) + lane/2,
    // position lane%2 -> chunk (lane%2) ^ ((col >> 3) & 1)
    constexpr int PER_PLANE = Cf::BPL / 1024;
    constexpr int WPW = Cf::BPIECES / 8;  // pieces per wave
    uint32_t b_off[2][WPW];
#pragma unroll
    for (int j = 0; j < WPW; ++j) {
        const int p = wave * WPW + j;
        const int plane = p / PER_PLANE;
        const int col = 32 * (p % PER_PLANE) + (lane >> 1);
        const int chunk = (lane & 1) ^ ((col >> 3) & 1);
        b_off[0][j] = (uint32_t)(((int64_t)plane * g.plane0 + (int64_t)col * g.ldb0 + 8 * chunk) * 2);
        b_off[1][j] = (uint32_t)(((int64_t)plane * g.plane1 + (int64_t)col * g.ldb1 + 8 * chunk) * 2);
    }
    const char* a_base0 = reinterpret_cast<const char*>(g.A0 + m0 * g.lda0);
    const char* a_base1 = reinterpret_cast<const char*>(g.A1 + m0 * g.lda1);
    const char* b_base0 = reinterpret_cast<const char*>(g.B0h);
    const char* b_base1 = reinterpret_cast<const char*>(g.B1h);

    auto fill = [&](int ph, int k0, unsigned char* st) {
        if (wave < 4)
            __builtin_amdgcn_global_load_lds((const void*)((ph ? a_base1 : a_base0) + (int64_t)k0 * 4 + a_off[ph]),
                                             (__attribute__((address_space(3))) void*)(st + wave * 1024), 16, 0, 0);
#pragma unroll
        for (int j = 0; j < WPW; ++j) {
            const int p = wave * WPW + j;
            __builtin_amdgcn_global_load_lds((const void*)((ph ? b_base1 : b_base0) + (int64_t)k0 * 2 + b_off[ph][j]),
                                             (__attribute__((address_space(3))) void*)(st + SG_A + p * 1024), 16, 0, 0);
        }
    };

    // ---- fragment read offsets (bytes within a stage)
    // A: row r = 32 grp + lr, chunks 2 lh and 2 lh + 1 (k 8 lh .. 8 lh + 7)
    int a_rd[2][2];
#pragma unroll
    for (int grp = 0; grp < 2; ++grp) {
        const int r = 32 * grp + lr;
#pragma unroll
        for (int h = 0; h < 2; ++h) a_rd[grp][h] = r * 64 + (((2 * lh + h) ^ ((r >> 2) & 3)) << 4);
    }
    // W: column n = c0w + 32 t + lr, chunk lh; plane 1 is BPL further
    int b_rd[TN];
#pragma unroll
    for (int t = 0; t < TN; ++t) {
        const int n = c0w + 32 * t + lr;
        b_rd[t] = SG_A + n * 32 + ((lh ^ ((n >> 3) & 1)) << 4);
    }
    float a_sc[2];
#pragma unroll
    for (int grp = 0; grp < 2; ++grp) a_sc[grp] = g.a_scale[min<int64_t>(m0 + 32 * grp + lr, g.M - 1)];

    f32x16s acc[2][TN];
#pragma unroll
    for (int grp = 0; grp < 2; ++grp)
#pragma unroll
        for (int t = 0; t < TN; ++t)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[grp][t][e] = 0.0f;

    auto step = [&](const unsigned char* __restrict__ cur) {
        unsigned w[2][2][4];  // [grp][plane][pair]
#pragma unroll
        for (int grp = 0; grp < 2; ++grp) {
            const float4 lo = *reinterpret_cast<const float4*>(cur + a_rd[grp][0]);
            const float4 hi = *reinterpret_cast<const float4*>(cur + a_rd[grp][1]);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                split_pair_h2(f8_at(lo, hi, 2 * j), f8_at(lo, hi, 2 * j + 1), a_sc[grp], w[grp][0][j], w[grp][1][j]);
        }
        f16x8s af[2][2];
#pragma unroll
        for (int grp = 0; grp < 2; ++grp)
#pragma unroll
            for (int p = 0; p < 2; ++p)
                af[grp][p] = __builtin_bit_cast(f16x8s, u32x4s{w[grp][p][0], w[grp][p][1], w[grp][p][2], w[grp][p][3]});
#pragma unroll
        for (int t = 0; t < TN; ++t) {
            const f16x8s b1 = __builtin_bit_cast(f16x8s, *reinterpret_cast<const u32x4s*>(cur + b_rd[t]));
            const f16x8s b2 = __builtin_bit_cast(f16x8s, *reinterpret_cast<const u32x4s*>(cur + b_rd[t] + Cf::BPL));
#pragma unroll
            for (int grp = 0; grp < 2; ++grp) {  // h2g's order per fragment pair: a2b1, a1b2, a1b1
                acc[grp][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[grp][1], b1, acc[grp][t], 0, 0, 0);
                acc[grp][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[grp][0], b2, acc[grp][t], 0, 0, 0);
                acc[grp][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[grp][0], b1, acc[grp][t], 0, 0, 0);
            }
        }
    };

    const int n0k = g.K0 / 16, n1k = g.K1 / 16, nk = n0k + n1k;
    fill(0, 0, sm);
    __syncthreads();
    for (int it = 0; it < nk; ++it) {
        unsigned char* cur = sm + (it & 1) * Cf::STAGE;
        unsigned char* nxt = sm + ((it + 1) & 1) * Cf::STAGE;
        if (it + 1 < nk) {
            const int nit = it + 1;
            if (nit < n0k) fill(0, nit * 16, nxt);
            else fill(1, (nit - n0k) * 16, nxt);
        }
        step(cur);
        __syncthreads();  // next stage landed (vmcnt drained), current stage free
    }

    // ---- epilogue: undo the scales, ReLU, then normalise rows as normalize_rows_vec
    float cinv[TN];
#pragma unroll
    for (int t = 0; t < TN; ++t) cinv[t] = g.b_inv[c0w + 32 * t + lr];
    float* img = reinterpret_cast<float*>(sm);
    constexpr int YS = Cf::N + SG_YSTRIDE_PAD;
#pragma unroll
    for (int grp = 0; grp < 2; ++grp) {
        // accumulator layout (32x32x16): element e of lane (lh, lr) is row (e&3) + 8(e>>2) + 4 lh, column lr
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int rl = (e & 3) + 8 * (e >> 2) + 4 * lh;
            const int64_t row = m0 + 32 * grp + rl;
            const float rinv = row < g.M ? 1.0f / g.a_scale[row] : 0.0f;
#pragma unroll
            for (int t = 0; t < TN; ++t) {
                const float v = (acc[grp][t][e] * rinv) * cinv[t];
                img[rl * YS + c0w + 32 * t + lr] = fmaxf(v, 0.0f);
            }
        }
        __syncthreads();
        // 32 rows, 4 per wave, one wave per row: lane l holds columns 4l + 256 j
#pragma unroll 1
        for (int i = 0; i < 4; ++i) {
            const int rl = wave * 4 + i;
            const int64_t row = m0 + 32 * grp + rl;
            if (row >= g.M) continue;  // wave-uniform
            const float* src = img + rl * YS + 4 * lane;
            float4 v[TN];
            float s = 0.0f;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                v[j] = *reinterpret_cast<const float4*>(src + 256 * j);
                s = __fadd_rn(s, __fmul_rn(v[j].x, v[j].x));
                s = __fadd_rn(s, __fmul_rn(v[j].y, v[j].y));
                s = __fadd_rn(s, __fmul_rn(v[j].z, v[j].z));
                s = __fadd_rn(s, __fmul_rn(v[j].w, v[j].w));
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
            const float norm = sqrtf(s);
            const bool scale = g.normalize && norm > 0.0f;
            float* dst = g.C + row * g.ldc + 4 * lane;
#pragma unroll
            for (int j = 0; j < TN; ++j)
                *reinterpret_cast<float4*>(dst + 256 * j) =
                    scale ? make_float4(v[j].x / norm, v[j].y / norm, v[j].z / norm, v[j].w / norm) : v[j];
        }
        __syncthreads();  // image rows reused by the next group
    }
}

}  // namespace

bool sage_gemm_fused_ok(int64_t M, int N, int K0, int K1, int64_t lda0, int64_t lda1, int64_t ldb0, int64_t ldb1,
                        int64_t plane0, int64_t plane1, int64_t ldc, const void* A0, const void* A1, const void* C) {
    // opt-in (read per call, tests cover both): in the overlapped 10M x 768 pipeline it
    // measured 1.16G vs 1.39G edges/s for gemm_nt_h2 + normalize_rows (every block streams
    // all 4.7 MB of W from L2 / Infinity Cache beside the gather, one 8-wave block per CU
    // waits at every 16-deep k step; profiles/r03_sage_fused_ab.txt)
    if (!env_int("RVX_SAGE_FUSED", 0) || M <= 0) return false;
    if (N != 256 && N != 512 && N != 768 && N != 1024) return false;
    if (K0 % 16 || K1 % 16 || lda0 % 4 || lda1 % 4 || ldb0 % 8 || ldb1 % 8 || ldc % 4) return false;
    if ((((uintptr_t)A0 | (uintptr_t)A1 | (uintptr_t)C) & 15) != 0) return false;
    const int64_t lim = (int64_t)1 << 31;
    return (int64_t)SG_ROWS * std::max(lda0, lda1) * 4 < lim && (plane0 + (int64_t)N * ldb0) * 2 < lim &&
           (plane1 + (int64_t)N * ldb1) * 2 < lim;
}

void sage_gemm_fused(int64_t M, int N, const float* A0, int64_t lda0, int K0, const float* A1, int64_t lda1, int K1,
                     const _Float16* B0h, int64_t ldb0, int64_t plane0, const _Float16* B1h, int64_t ldb1,
                     int64_t plane1, const float* a_scale, const float* b_inv, float* C, int64_t ldc, bool normalize,
                     const char* tag) {
    if (M <= 0) return;
    SageGemmArgs g{A0, lda0, K0, A1, lda1, K1, B0h, B1h, ldb0, ldb1, plane0, plane1, a_scale, b_inv, C, ldc, M, N,
                   normalize ? 1 : 0};
    const dim3 grid((unsigned)((M + SG_ROWS - 1) / SG_ROWS)), block(512);
    static bool attr = false;
    if (!attr) {
        RVX_HIP(hipFuncSetAttribute((const void*)k_sage_gemm_fused<1>, hipFuncAttributeMaxDynamicSharedMemorySize, SgCfg<1>::LDS));
        RVX_HIP(hipFuncSetAttribute((const void*)k_sage_gemm_fused<2>, hipFuncAttributeMaxDynamicSharedMemorySize, SgCfg<2>::LDS));
        RVX_HIP(hipFuncSetAttribute((const void*)k_sage_gemm_fused<3>, hipFuncAttributeMaxDynamicSharedMemorySize, SgCfg<3>::LDS));
        RVX_HIP(hipFuncSetAttribute((const void*)k_sage_gemm_fused<4>, hipFuncAttributeMaxDynamicSharedMemorySize, SgCfg<4>::LDS));
        attr = true;
    }
    switch (N) {
        case 256: RVX_LAUNCH(tag, k_sage_gemm_fused<1>, grid, block, SgCfg<1>::LDS, g); break;
        case 512: RVX_LAUNCH(tag, k_sage_gemm_fused<2>, grid, block, SgCfg<2>::LDS, g); break;
        case 768: RVX_LAUNCH(tag, k_sage_gemm_fused<3>, grid, block, SgCfg<3>::LDS, g); break;
        default: RVX_LAUNCH(tag, k_sage_gemm_fused<4>, grid, block, SgCfg<4>::LDS, g); break;
    }
}

}  // namespace rvx
