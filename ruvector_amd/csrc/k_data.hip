// k_data.hip — synthetic corpora and small layout kernels.
//
// The counter-based stream h(seed, i) = splitmix64(splitmix64(seed) + i) is the
// same one oracle/oracle.cpp implements, so CPU baselines and GPU runs see the
// same integers; uniform floats are exact (24-bit mantissa draws) and therefore
// bit-identical on both sides. Normal draws go through libm (Box–Muller) and are
// generated once on the device and downloaded when the CPU needs them.
#include "common.hpp"
#include "kernels.hpp"

namespace rvx {
namespace {

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void k_fill_uniform(float* p, int64_t n, uint64_t s0, float lo, float span) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t h = splitmix64(s0 + (uint64_t)i);
        const float u = (float)(uint32_t)(h >> 40) * 5.9604644775390625e-08f;  // 2^-24
        p[i] = __fadd_rn(__fmul_rn(u, span), lo);
    }
}

__global__ void k_fill_normal(float* p, int64_t n, uint64_t s0) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t h1 = splitmix64(s0 + 2 * (uint64_t)i);
        const uint64_t h2 = splitmix64(s0 + 2 * (uint64_t)i + 1);
        const float u1 = (float)((uint32_t)(h1 >> 40) + 1u) * 5.9604644775390625e-08f;  // (0,1]
        const float u2 = (float)(uint32_t)(h2 >> 40) * 5.9604644775390625e-08f;
        p[i] = sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
    }
}

// C5 points: row r of the global corpus = direction ~ N(0,1)^dim
// normalised, times radius rmax * U[0,1): the normals are elements [r*dim, (r+1)*dim)
// of the fill_normal(seed) stream and the radius element r of the
// fill_uniform(seed + 1) stream, so a node-range shard generates exactly its rows of
// the single-GPU corpus. One wave per row; the norm is a wave reduction.
__global__ __launch_bounds__(256) void k_fill_ball_rows(float* p, int64_t rows, int dim, uint64_t s_dir,
                                                        uint64_t s_rad, int64_t first_row, float rmax) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int64_t g = first_row + r;
    float* row = p + r * dim;
    float ss = 0.0f;
    for (int j = lane; j < dim; j += 64) {
        const uint64_t i = (uint64_t)(g * dim + j);
        const uint64_t h1 = splitmix64(s_dir + 2 * i);
        const uint64_t h2 = splitmix64(s_dir + 2 * i + 1);
        const float u1 = (float)((uint32_t)(h1 >> 40) + 1u) * 5.9604644775390625e-08f;
        const float u2 = (float)(uint32_t)(h2 >> 40) * 5.9604644775390625e-08f;
        const float v = sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
        row[j] = v;
        ss += v * v;
    }
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
    const uint64_t hr = splitmix64(s_rad + (uint64_t)g);
    const float rad = rmax * ((float)(uint32_t)(hr >> 40) * 5.9604644775390625e-08f);
    const float scale = ss > 0.0f ? rad / sqrtf(ss) : 0.0f;
    for (int j = lane; j < dim; j += 64) row[j] *= scale;
}

// One wave per row: norm = sqrt(sum x^2); x /= norm (true division, as
// normalize_vector in crates/ruvector-core/tests/hnsw_integration_test.rs:21-28
// and the GraphSAGE output normalisation, graphsage.rs:177-182).
__global__ void k_normalize_rows(float* p, int64_t rows, int dim, int only_positive) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (row >= rows) return;
    float* x = p + row * dim;
    float s = 0.0f;
    for (int c = lane; c < dim; c += 64) s = __fadd_rn(s, __fmul_rn(x[c], x[c]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    const float norm = sqrtf(s);
    if (only_positive && !(norm > 0.0f)) return;
    for (int c = lane; c < dim; c += 64) x[c] = x[c] / norm;
}

// Vector form for dim % 4 == 0, dim <= 256*NV: the row stays in registers
// (one 1-KiB wave load per 256 columns), one read and one write per element.
template <int NV>
__global__ __launch_bounds__(256) void k_normalize_rows_vec(float* __restrict__ p, int64_t rows, int dim,
                                                            int only_positive) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    float* x = p + row * dim + 4 * lane;
    float4 v[NV];
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const bool on = 4 * lane + 256 * j < dim;
        v[j] = on ? *reinterpret_cast<const float4*>(x + 256 * j) : make_float4(0.f, 0.f, 0.f, 0.f);
        s = __fadd_rn(s, __fmul_rn(v[j].x, v[j].x));
        s = __fadd_rn(s, __fmul_rn(v[j].y, v[j].y));
        s = __fadd_rn(s, __fmul_rn(v[j].z, v[j].z));
        s = __fadd_rn(s, __fmul_rn(v[j].w, v[j].w));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    const float norm = sqrtf(s);
    if (only_positive && !(norm > 0.0f)) return;
#pragma unroll
    for (int j = 0; j < NV; ++j)
        if (4 * lane + 256 * j < dim)
            *reinterpret_cast<float4*>(x + 256 * j) =
                make_float4(v[j].x / norm, v[j].y / norm, v[j].z / norm, v[j].w / norm);
}

// rows [row_begin, row_begin + n_rows) of an n_total-node graph; the edge id
// stream is global so every shard reproduces its slice of the same graph.
__global__ void k_random_csr(int64_t n_total, int64_t row_begin, int64_t n_rows, int deg, uint64_t s0,
                             int64_t* row_ptr, int32_t* col) {
    const int64_t total = n_rows * deg;
    const uint64_t e0 = (uint64_t)(row_begin * deg);
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        col[e] = (int32_t)(splitmix64(s0 + e0 + (uint64_t)e) % (uint64_t)n_total);
    }
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n_rows; i += (int64_t)gridDim.x * blockDim.x)
        row_ptr[i] = i * deg;
}

__global__ void k_transpose(const float* in, int64_t rows, int64_t cols, float* out) {
    __shared__ float tile[32][33];
    const int64_t c0 = (int64_t)blockIdx.x * 32, r0 = (int64_t)blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
    for (int j = ty; j < 32; j += 8) {
        const int64_t r = r0 + j, c = c0 + tx;
        if (r < rows && c < cols) tile[j][tx] = in[r * cols + c];
    }
    __syncthreads();
    for (int j = ty; j < 32; j += 8) {
        const int64_t c = c0 + j, r = r0 + tx;
        if (r < rows && c < cols) out[c * rows + r] = tile[tx][j];
    }
}

// sum over 8-byte words i of mix64(w_i + (i + 1) * golden) mod 2^64: order-free integer
// arithmetic, so the result does not depend on the launch, and a permutation or a
// single flipped bit changes it (rvx_buffer_checksum; cross-rank table agreement)
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__global__ __launch_bounds__(256) void k_checksum(const uint64_t* w, int64_t words, const uint8_t* tail, int tail_bytes,
                                                  unsigned long long* out) {
    uint64_t acc = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride)
        acc += mix64(__builtin_nontemporal_load(w + i) + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull);
    if (blockIdx.x == 0 && threadIdx.x == 0 && tail_bytes > 0) {
        uint64_t t = 0;
        for (int b = 0; b < tail_bytes; ++b) t |= (uint64_t)tail[b] << (8 * b);
        acc += mix64(t + (uint64_t)(words + 1) * 0x9E3779B97F4A7C15ull);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)acc);
}

unsigned grid_for(int64_t n, int block) {
    int64_t g = (n + block - 1) / block;
    if (g > 65536) g = 65536;
    if (g < 1) g = 1;
    return (unsigned)g;
}

}  // namespace

void checksum(const void* p, int64_t bytes, uint64_t* out_dev) {
    RVX_HIP(hipMemsetAsync(out_dev, 0, 8, stream()));
    if (bytes <= 0) return;
    const int64_t words = bytes / 8;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(2048, (words + 255) / 256));
    RVX_LAUNCH("checksum", k_checksum, dim3(grid), dim3(256), 0, (const uint64_t*)p, words,
               (const uint8_t*)p + words * 8, (int)(bytes - words * 8), (unsigned long long*)out_dev);
}

void fill_uniform(float* p, int64_t n, uint64_t seed, float lo, float hi) {
    ProfScope ps("fill_uniform");
    hipLaunchKernelGGL(k_fill_uniform, dim3(grid_for(n, 256)), dim3(256), 0, stream(), p, n, splitmix64(seed), lo,
                       hi - lo);
    RVX_HIP(hipGetLastError());
}
void fill_uniform_at(float* p, int64_t n, uint64_t seed, int64_t first, float lo, float hi) {
    ProfScope ps("fill_uniform");
    hipLaunchKernelGGL(k_fill_uniform, dim3(grid_for(n, 256)), dim3(256), 0, stream(), p, n,
                       splitmix64(seed) + (uint64_t)first, lo, hi - lo);
    RVX_HIP(hipGetLastError());
}
void fill_ball_rows(float* p, int64_t rows, int dim, uint64_t seed, int64_t first_row, float rmax) {
    if (rows <= 0) return;
    ProfScope ps("fill_ball");
    hipLaunchKernelGGL(k_fill_ball_rows, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream(), p, rows, dim,
                       splitmix64(seed), splitmix64(seed + 1), first_row, rmax);
    RVX_HIP(hipGetLastError());
}

void fill_normal(float* p, int64_t n, uint64_t seed) {
    ProfScope ps("fill_normal");
    hipLaunchKernelGGL(k_fill_normal, dim3(grid_for(n, 256)), dim3(256), 0, stream(), p, n, splitmix64(seed));
    RVX_HIP(hipGetLastError());
}
void normalize_rows(float* p, int64_t rows, int dim, bool only_positive, const char* tag) {
    if (rows <= 0) return;
    const char* t = tag ? tag : "normalize_rows";
    const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
    const int op = only_positive ? 1 : 0;
    const bool vec = dim % 4 == 0 && ((uintptr_t)p & 15) == 0;
    if (vec && dim <= 256) RVX_LAUNCH(t, k_normalize_rows_vec<1>, grid, block, 0, p, rows, dim, op);
    else if (vec && dim <= 512) RVX_LAUNCH(t, k_normalize_rows_vec<2>, grid, block, 0, p, rows, dim, op);
    else if (vec && dim <= 768) RVX_LAUNCH(t, k_normalize_rows_vec<3>, grid, block, 0, p, rows, dim, op);
    else if (vec && dim <= 1024) RVX_LAUNCH(t, k_normalize_rows_vec<4>, grid, block, 0, p, rows, dim, op);
    else RVX_LAUNCH(t, k_normalize_rows, grid, block, 0, p, rows, dim, op);
}
void random_csr(int64_t n, int deg, uint64_t seed, int64_t* row_ptr, int32_t* col) {
    random_csr_shard(n, 0, n, deg, seed, row_ptr, col);
}
void random_csr_shard(int64_t n_total, int64_t row_begin, int64_t n_rows, int deg, uint64_t seed, int64_t* row_ptr,
                      int32_t* col) {
    ProfScope ps("random_csr");
    hipLaunchKernelGGL(k_random_csr, dim3(grid_for(std::max<int64_t>(n_rows * deg, n_rows + 1), 256)), dim3(256), 0,
                       stream(), n_total, row_begin, n_rows, deg, splitmix64(seed), row_ptr, col);
    RVX_HIP(hipGetLastError());
}
void transpose(const float* in, int64_t rows, int64_t cols, float* out) {
    if (rows <= 0 || cols <= 0) return;
    dim3 grid((unsigned)((cols + 31) / 32), (unsigned)((rows + 31) / 32));
    hipLaunchKernelGGL(k_transpose, grid, dim3(256), 0, stream(), in, rows, cols, out);
    RVX_HIP(hipGetLastError());
}

}  // namespace rvx

using namespace rvx;

extern "C" {
rvx_status rvx_fill_uniform(rvx_buffer* buf, int64_t n, uint64_t seed, float lo, float hi) {
    return guard([&] {
        RVX_REQUIRE(buf && n >= 0 && n * 4 <= buf->mem.bytes, RVX_ERR_INVALID_PARAMETER, "buffer too small");
        fill_uniform(buf->mem.as<float>(), n, seed, lo, hi);
    });
}
rvx_status rvx_fill_uniform_at(rvx_buffer* buf, int64_t n, uint64_t seed, int64_t first, float lo, float hi) {
    return guard([&] {
        RVX_REQUIRE(buf && n >= 0 && first >= 0 && n * 4 <= buf->mem.bytes, RVX_ERR_INVALID_PARAMETER,
                    "buffer too small");
        fill_uniform_at(buf->mem.as<float>(), n, seed, first, lo, hi);
    });
}
rvx_status rvx_fill_normal(rvx_buffer* buf, int64_t n, uint64_t seed) {
    return guard([&] {
        RVX_REQUIRE(buf && n >= 0 && n * 4 <= buf->mem.bytes, RVX_ERR_INVALID_PARAMETER, "buffer too small");
        fill_normal(buf->mem.as<float>(), n, seed);
    });
}
rvx_status rvx_fill_ball_rows(rvx_buffer* buf, int64_t rows, int32_t dim, uint64_t seed, int64_t first_row,
                              float rmax) {
    return guard([&] {
        RVX_REQUIRE(buf && rows >= 0 && dim > 0 && first_row >= 0 && rows * dim * 4 <= buf->mem.bytes,
                    RVX_ERR_INVALID_PARAMETER, "buffer too small");
        fill_ball_rows(buf->mem.as<float>(), rows, dim, seed, first_row, rmax);
    });
}
rvx_status rvx_normalize_rows(rvx_buffer* buf, int64_t rows, int32_t dim) {
    return guard([&] {
        RVX_REQUIRE(buf && rows >= 0 && dim > 0 && rows * dim * 4 <= buf->mem.bytes, RVX_ERR_INVALID_PARAMETER,
                    "buffer too small");
        normalize_rows(buf->mem.as<float>(), rows, dim, true, "normalize_rows");
    });
}
rvx_status rvx_random_csr(int64_t n, int32_t deg, uint64_t seed, rvx_buffer* row_ptr, rvx_buffer* col) {
    return guard([&] {
        RVX_REQUIRE(n > 0 && n < (int64_t)1 << 31 && deg >= 0, RVX_ERR_INVALID_PARAMETER, "bad graph size");
        RVX_REQUIRE(row_ptr && row_ptr->mem.bytes >= (n + 1) * 8, RVX_ERR_INVALID_PARAMETER, "row_ptr too small");
        RVX_REQUIRE(col && col->mem.bytes >= n * deg * 4, RVX_ERR_INVALID_PARAMETER, "col too small");
        random_csr(n, deg, seed, row_ptr->mem.as<int64_t>(), col->mem.as<int32_t>());
    });
}
rvx_status rvx_random_csr_shard(int64_t n_total, int64_t row_begin, int64_t n_rows, int32_t deg, uint64_t seed,
                                rvx_buffer* row_ptr, rvx_buffer* col) {
    return guard([&] {
        RVX_REQUIRE(n_total > 0 && n_total < (int64_t)1 << 31 && deg >= 0 && row_begin >= 0 && n_rows >= 0 &&
                        row_begin + n_rows <= n_total,
                    RVX_ERR_INVALID_PARAMETER, "bad shard range");
        RVX_REQUIRE(row_ptr && row_ptr->mem.bytes >= (n_rows + 1) * 8, RVX_ERR_INVALID_PARAMETER, "row_ptr too small");
        RVX_REQUIRE(col && col->mem.bytes >= n_rows * deg * 4, RVX_ERR_INVALID_PARAMETER, "col too small");
        random_csr_shard(n_total, row_begin, n_rows, deg, seed, row_ptr->mem.as<int64_t>(), col->mem.as<int32_t>());
    });
}
}
