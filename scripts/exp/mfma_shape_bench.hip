// Micro-benchmark (round 4): f16 MFMA shapes fed from LDS, 8 waves per block (2 per SIMD),
// one block per CU, random operands: v_mfma_f32_32x32x16_f16 (16 per K=32 step, 128x64
// wave tile) vs v_mfma_f32_16x16x32_f16 (32 per step, same tile and bytes). Timing only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int SHAPE>
__global__ __launch_bounds__(512, 1) void k(const _Float16* src, float* out, int iters) {
    __shared__ __attribute__((aligned(16))) _Float16 lds[2][256 * 32 + 256 * 32];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < 2 * 512 * 32; i += 512) (&lds[0][0])[i] = src[(blockIdx.x * 977 + i) & 65535];
    __syncthreads();
    const int wm = wave & 1, wn = wave >> 1;
    if constexpr (SHAPE == 32) {
        f32x16 acc[4][2] = {};
        const int lr = lane & 31, lh = lane >> 5;
        for (int it = 0; it < iters; ++it) {
            const _Float16* cur = lds[it & 1];
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                h16x8 a[4], b[2];
#pragma unroll
                for (int f = 0; f < 4; ++f) a[f] = *reinterpret_cast<const h16x8*>(cur + (wm * 128 + f * 32 + lr) * 32 + (2 * ks + lh) * 8);
#pragma unroll
                for (int f = 0; f < 2; ++f) b[f] = *reinterpret_cast<const h16x8*>(cur + 256 * 32 + (wn * 64 + f * 32 + lr) * 32 + (2 * ks + lh) * 8);
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int n = 0; n < 2; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[m], b[n], acc[m][n], 0, 0, 0);
            }
        }
        float s = 0;
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
                for (int e = 0; e < 16; ++e) s += acc[m][n][e];
        out[blockIdx.x * 512 + tid] = s;
    } else {
        f32x4 acc[8][4] = {};
        const int lc = lane & 15, lg = lane >> 4;
        for (int it = 0; it < iters; ++it) {
            const _Float16* cur = lds[it & 1];
            h16x8 a[8], b[4];
#pragma unroll
            for (int f = 0; f < 8; ++f) a[f] = *reinterpret_cast<const h16x8*>(cur + (wm * 128 + f * 16 + lc) * 32 + lg * 8);
#pragma unroll
            for (int f = 0; f < 4; ++f) b[f] = *reinterpret_cast<const h16x8*>(cur + 256 * 32 + (wn * 64 + f * 16 + lc) * 32 + lg * 8);
#pragma unroll
            for (int m = 0; m < 8; ++m)
#pragma unroll
                for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[m], b[n], acc[m][n], 0, 0, 0);
        }
        float s = 0;
#pragma unroll
        for (int m = 0; m < 8; ++m)
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int e = 0; e < 4; ++e) s += acc[m][n][e];
        out[blockIdx.x * 512 + tid] = s;
    }
}

int main() {
    int ncu = 256;
    std::vector<_Float16> h(65536);
    unsigned s = 12345;
    for (auto& v : h) { s = s * 1664525u + 1013904223u; v = (_Float16)(((s >> 9) & 0xFFFF) / 32768.0f - 1.0f); }
    _Float16* d; float* o;
    hipMalloc(&d, h.size() * 2); hipMalloc(&o, ncu * 512 * 4 * 4);
    hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const int iters = 20000;
    const double flops = 2.0 * 256 * 256 * 32 * (double)iters * ncu * 4;  // 4 blocks/CU-equivalents below
    for (int rep = 0; rep < 3; ++rep) {
        for (int shape : {32, 16}) {
            hipEventRecord(e0);
            for (int r = 0; r < 4; ++r) {
                if (shape == 32) k<32><<<ncu, 512>>>(d, o + r * ncu * 512, iters);
                else k<16><<<ncu, 512>>>(d, o + r * ncu * 512, iters);
            }
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            printf("shape %dx%d: %.1f ms, %.1f TFLOP/s\n", shape, shape, ms, flops / ms / 1e9);
        }
    }
    return 0;
}
