// common.hpp — shared host-side plumbing of librvx: status/error handling,
// the per-device stream, device buffers and the event-based kernel profiler.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "rvx/rvx.h"

namespace rvx {

// An exception carrying an rvx_status; every extern "C" entry point catches it
// and turns it into (status, thread-local message).
struct Error : std::runtime_error {
    rvx_status code;
    Error(rvx_status c, const std::string& m) : std::runtime_error(m), code(c) {}
};

[[noreturn]] void fail(rvx_status code, const std::string& msg);
void set_last_error(const std::string& msg);

#define RVX_HIP(expr)                                                                            \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            ::rvx::fail(e_ == hipErrorOutOfMemory ? RVX_ERR_OUT_OF_MEMORY : RVX_ERR_DEVICE,      \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                      \
    } while (0)

#define RVX_REQUIRE(cond, code, msg)                                                             \
    do {                                                                                         \
        if (!(cond)) ::rvx::fail((code), (msg));                                                 \
    } while (0)

// Wrap an API body: maps exceptions to status codes.
template <class F>
rvx_status guard(F&& f) {
    try {
        f();
        return RVX_OK;
    } catch (const Error& e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc&) {
        set_last_error("host allocation failed");
        return RVX_ERR_OUT_OF_MEMORY;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return RVX_ERR_INVALID_PARAMETER;
    }
}

// ---------------------------------------------------------------- device
struct Device {
    int id = 0;
    hipStream_t stream = nullptr;  // every kernel of this device runs here ...
    hipStream_t aux = nullptr;     // ... except pipelined stages overlapped on this one
    hipStream_t xfer = nullptr;    // RCCL halo exchange overlapped with compute
    hipStream_t aux2 = nullptr;    // a third pipeline stage (GraphSAGE row normalisation)
    std::vector<hipEvent_t> pipe_events;  // timing-free events for stream hand-offs
    // CU-partitioned stream pair (cu_split_streams): [0] the MFMA side, [1] the gather side
    hipStream_t cu_split[2] = {nullptr, nullptr};
    int cu_split_mode = 0, cu_split_count[2] = {0, 0};
    int num_cus = 0;
    int64_t hbm_bytes = 0;
    std::string arch;
};
Device& device();          // current thread's device (lazily initialised)
hipStream_t stream();      // the stream launches go to (device().stream unless a StreamScope is active)
void sync();               // hipStreamSynchronize(device().stream)
// At least `count` reusable hand-off events of the current device (callers
// hold the device's ComputeLock).
hipEvent_t* pipeline_events(int count);

// Integer tuning knob from the environment (read once by the caller).
inline int env_int(const char* name, int dflt) {
    const char* v = std::getenv(name);
    return (v && *v) ? std::atoi(v) : dflt;
}

// Two streams whose queues own complementary CU sets (hipExtStreamCreateWithCUMask),
// for overlapping an MFMA-bound and an HBM-bound stage without sharing CUs.
// mode 1: mask bit i to the MFMA side iff (i >> 3) & 1 == 0; mode 2: iff i & 1 == 0
// (both give each side half the CUs; which half of an XCD depends on how the
// queue maps mask bits to XCDs). Created once per mode; counts[] = CUs per side.
void cu_split_streams(int mode, hipStream_t out[2], int counts[2]);
// CUs the current launches may occupy: num_cus, or a CuScope's count.
int active_cus();
struct CuScope {
    int prev;
    explicit CuScope(int cus);
    ~CuScope();
};

// Route this thread's launches to `s` for the scope's lifetime (pipelining).
struct StreamScope {
    hipStream_t prev;
    explicit StreamScope(hipStream_t s);
    ~StreamScope();
};

// RAII device allocation (256-B aligned by hipMalloc).
struct DevMem {
    void* p = nullptr;
    int64_t bytes = 0;
    int dev = 0;
    DevMem() = default;
    explicit DevMem(int64_t b);
    ~DevMem();
    DevMem(const DevMem&) = delete;
    DevMem& operator=(const DevMem&) = delete;
    DevMem(DevMem&& o) noexcept { *this = std::move(o); }
    DevMem& operator=(DevMem&& o) noexcept;
    void reset(int64_t b);
    template <class T> T* as() const { return static_cast<T*>(p); }
    void upload(const void* src, int64_t n, int64_t off = 0);
    void download(void* dst, int64_t n, int64_t off = 0) const;
};

// ---------------------------------------------------------------- profiler
// Records a start/stop hipEvent pair on the library stream around one launch
// when profiling is on; rvx_profile_query sums the pairs per tag.
struct ProfScope {
    const char* name;
    hipEvent_t a = nullptr, b = nullptr;
    explicit ProfScope(const char* n);
    ~ProfScope();
};

// Event pair stamped by the dispatch packet itself (hipExtLaunchKernelGGL), so
// the measured interval is exactly the kernel's execution; null when profiling
// is off.
struct KernelTimer {
    const char* name;
    hipEvent_t a = nullptr, b = nullptr;
    explicit KernelTimer(const char* n);
    ~KernelTimer();
};

// Power-of-two scale putting a row maximum m in [2^14, 2^15) (1 for zero or
// non-finite rows): the split-f16 GEMM's operand scaling (gemm_f32.hip), also
// produced by the gather kernel (k_aggregate.hip).
__device__ __forceinline__ float h2_scale_dev(float m) {
    if (!(m > 0.0f) || !__builtin_isfinite(m)) return 1.0f;
    const int e = ilogbf(m);
    return ldexpf(1.0f, min(127, max(-126, 14 - e)));
}

}  // namespace rvx

// Launch on the library stream, timed per kernel when profiling is enabled.
#define RVX_LAUNCH(TAG, KERNEL, GRID, BLOCK, SHMEM, ...)                                                  \
    do {                                                                                                   \
        ::rvx::KernelTimer kt_(TAG);                                                                       \
        hipExtLaunchKernelGGL(KERNEL, GRID, BLOCK, SHMEM, ::rvx::stream(), kt_.a, kt_.b, 0, __VA_ARGS__); \
        RVX_HIP(hipGetLastError());                                                                        \
    } while (0)

struct rvx_buffer {
    rvx::DevMem mem;
};
