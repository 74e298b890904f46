// runtime.cpp — device selection, the library stream, buffers, profiler and
// the small C-ABI surface that is pure plumbing (no reference analogue).
#include <map>
#include <mutex>
#include <unordered_map>

#include <vector>

#include "common.hpp"
#include "graph.hpp"
#include "kernels.hpp"

namespace rvx {

static thread_local std::string g_last_error;
static thread_local int g_thread_device = -1;

void set_last_error(const std::string& msg) { g_last_error = msg; }
[[noreturn]] void fail(rvx_status code, const std::string& msg) { throw Error(code, msg); }

static std::mutex g_dev_mu;
static std::map<int, std::unique_ptr<Device>> g_devices;

static Device& device_for(int id) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    auto it = g_devices.find(id);
    if (it != g_devices.end()) return *it->second;
    int n = 0;
    RVX_HIP(hipGetDeviceCount(&n));
    RVX_REQUIRE(id >= 0 && id < n, RVX_ERR_DEVICE, "no HIP device " + std::to_string(id));
    RVX_HIP(hipSetDevice(id));
    auto d = std::make_unique<Device>();
    d->id = id;
    RVX_HIP(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
    RVX_HIP(hipStreamCreateWithFlags(&d->aux, hipStreamNonBlocking));
    RVX_HIP(hipStreamCreateWithFlags(&d->xfer, hipStreamNonBlocking));
    RVX_HIP(hipStreamCreateWithFlags(&d->aux2, hipStreamNonBlocking));
    hipDeviceProp_t prop;
    RVX_HIP(hipGetDeviceProperties(&prop, id));
    d->num_cus = prop.multiProcessorCount;
    d->hbm_bytes = (int64_t)prop.totalGlobalMem;
    d->arch = prop.gcnArchName;
    Device& ref = *d;
    g_devices[id] = std::move(d);
    return ref;
}

Device& device() {
    if (g_thread_device < 0) g_thread_device = 0;
    Device& d = device_for(g_thread_device);
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != d.id) RVX_HIP(hipSetDevice(d.id));
    return d;
}
static thread_local hipStream_t g_stream_override = nullptr;
hipStream_t stream() {
    Device& d = device();
    return g_stream_override ? g_stream_override : d.stream;
}
void sync() { RVX_HIP(hipStreamSynchronize(device().stream)); }
hipEvent_t* pipeline_events(int count) {
    Device& d = device();
    while ((int)d.pipe_events.size() < count) {
        hipEvent_t e;
        RVX_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        d.pipe_events.push_back(e);
    }
    return d.pipe_events.data();
}
static thread_local int g_cu_override = 0;
int active_cus() { return g_cu_override > 0 ? g_cu_override : device().num_cus; }
CuScope::CuScope(int cus) : prev(g_cu_override) { g_cu_override = cus; }
CuScope::~CuScope() { g_cu_override = prev; }

void cu_split_streams(int mode, hipStream_t out[2], int counts[2]) {
    Device& d = device();
    if (d.cu_split_mode != mode) {
        for (auto& st : d.cu_split)
            if (st) { RVX_HIP(hipStreamSynchronize(st)); RVX_HIP(hipStreamDestroy(st)); st = nullptr; }
        const int n = d.num_cus;
        std::vector<uint32_t> m[2];
        for (auto& v : m) v.assign((size_t)(n + 31) / 32, 0u);
        int cnt[2] = {0, 0};
        for (int i = 0; i < n; ++i) {
            const int side = mode == 2 ? (i & 1) : ((i >> 3) & 1);
            m[side][(size_t)i / 32] |= 1u << (i % 32);
            ++cnt[side];
        }
        for (int k = 0; k < 2; ++k) {
            RVX_HIP(hipExtStreamCreateWithCUMask(&d.cu_split[k], (uint32_t)m[k].size(), m[k].data()));
            d.cu_split_count[k] = cnt[k];
        }
        d.cu_split_mode = mode;
    }
    for (int k = 0; k < 2; ++k) { out[k] = d.cu_split[k]; counts[k] = d.cu_split_count[k]; }
}

StreamScope::StreamScope(hipStream_t s) : prev(g_stream_override) { g_stream_override = s; }
StreamScope::~StreamScope() { g_stream_override = prev; }

DevMem::DevMem(int64_t b) { reset(b); }
DevMem::~DevMem() {
    if (p) {
        int cur = -1;
        hipGetDevice(&cur);
        if (cur != dev) hipSetDevice(dev);
        hipFree(p);
        if (cur != dev && cur >= 0) hipSetDevice(cur);
    }
}
DevMem& DevMem::operator=(DevMem&& o) noexcept {
    if (this != &o) {
        if (p) hipFree(p);
        p = o.p; bytes = o.bytes; dev = o.dev;
        o.p = nullptr; o.bytes = 0;
    }
    return *this;
}
void DevMem::reset(int64_t b) {
    if (p) { hipFree(p); p = nullptr; bytes = 0; }
    RVX_REQUIRE(b >= 0, RVX_ERR_INVALID_PARAMETER, "negative allocation");
    dev = device().id;
    if (b > 0) {
        // Large tables are read at random (HNSW rows, gathered features): a
        // physically contiguous allocation lets the VM map large fragments, so
        // the per-CU translation cache covers far more of the table.
        static const int64_t contig_min = (int64_t)env_int("RVX_CONTIG_MIN_MB", 256) << 20;
        if (contig_min > 0 && b >= contig_min) {
            if (hipExtMallocWithFlags(&p, (size_t)b, hipDeviceMallocContiguous) != hipSuccess) {
                (void)hipGetLastError();
                p = nullptr;
            }
        }
        if (!p) RVX_HIP(hipMalloc(&p, (size_t)b));
        bytes = b;
    }
}
void DevMem::upload(const void* src, int64_t n, int64_t off) {
    RVX_REQUIRE(off >= 0 && n >= 0 && off + n <= bytes, RVX_ERR_INVALID_PARAMETER, "upload out of range");
    if (n == 0) return;
    RVX_HIP(hipMemcpyAsync((char*)p + off, src, (size_t)n, hipMemcpyHostToDevice, stream()));
    sync();
}
void DevMem::download(void* dst, int64_t n, int64_t off) const {
    RVX_REQUIRE(off >= 0 && n >= 0 && off + n <= bytes, RVX_ERR_INVALID_PARAMETER, "download out of range");
    if (n == 0) return;
    RVX_HIP(hipMemcpyAsync(dst, (const char*)p + off, (size_t)n, hipMemcpyDeviceToHost, stream()));
    sync();
}

// ---------------------------------------------------------------- profiler
struct ProfState {
    std::mutex mu;
    bool on = false;
    struct Rec { std::string name; hipEvent_t a, b; };
    std::vector<Rec> pending;
    std::unordered_map<std::string, std::pair<double, int64_t>> totals;
    std::vector<std::string> order;
    void drain() {  // caller holds mu
        for (auto& r : pending) {
            float ms = 0.f;
            if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
                auto it = totals.find(r.name);
                if (it == totals.end()) { totals[r.name] = {0.0, 0}; order.push_back(r.name); }
                totals[r.name].first += ms;
                totals[r.name].second += 1;
            }
            hipEventDestroy(r.a);
            hipEventDestroy(r.b);
        }
        pending.clear();
    }
};
static ProfState g_prof;

ProfScope::ProfScope(const char* n) : name(n) {
    if (!g_prof.on) return;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) { a = b = nullptr; return; }
    hipEventRecord(a, stream());
}
ProfScope::~ProfScope() {
    if (!a) return;
    hipEventRecord(b, stream());
    std::lock_guard<std::mutex> lk(g_prof.mu);
    g_prof.pending.push_back({name, a, b});
    if (g_prof.pending.size() > 4096) g_prof.drain();
}

KernelTimer::KernelTimer(const char* n) : name(n) {
    if (!g_prof.on) return;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) a = b = nullptr;
}
KernelTimer::~KernelTimer() {
    if (!a) return;
    std::lock_guard<std::mutex> lk(g_prof.mu);
    g_prof.pending.push_back({name, a, b});
    if (g_prof.pending.size() > 4096) g_prof.drain();
}

}  // namespace rvx

using namespace rvx;

extern "C" {

int32_t rvx_last_error(char* buf, size_t len) {
    const std::string& m = g_last_error;
    if (buf && len) {
        size_t n = std::min(len - 1, m.size());
        std::memcpy(buf, m.data(), n);
        buf[n] = 0;
    }
    return (int32_t)m.size();
}

#ifndef RVX_SRC_HASH
#define RVX_SRC_HASH "unknown"
#endif
// "rvx <version> (gfx950) src <hash>": the hash is sha256 over the library's
// sources (Makefile SRC_HASH), checked against the shipped tree on import.
const char* rvx_version(void) { return "rvx 0.2.0 (gfx950) src " RVX_SRC_HASH; }

rvx_status rvx_device_count(int32_t* count) {
    return guard([&] {
        int n = 0;
        hipError_t e = hipGetDeviceCount(&n);
        *count = (e == hipSuccess) ? n : 0;
    });
}

rvx_status rvx_set_device(int32_t dev) {
    return guard([&] {
        int n = 0;
        RVX_HIP(hipGetDeviceCount(&n));
        RVX_REQUIRE(dev >= 0 && dev < n, RVX_ERR_DEVICE, "device index out of range");
        g_thread_device = dev;
        device();
    });
}

rvx_status rvx_get_device(int32_t* dev) {
    return guard([&] { *dev = device().id; });
}

rvx_status rvx_synchronize(void) {
    return guard([&] { sync(); });
}

rvx_status rvx_device_info(int32_t* num_cus, int64_t* hbm_bytes, char* arch, size_t arch_len) {
    return guard([&] {
        Device& d = device();
        if (num_cus) *num_cus = d.num_cus;
        if (hbm_bytes) *hbm_bytes = d.hbm_bytes;
        if (arch && arch_len) {
            size_t n = std::min(arch_len - 1, d.arch.size());
            std::memcpy(arch, d.arch.data(), n);
            arch[n] = 0;
        }
    });
}

rvx_status rvx_buffer_alloc(int64_t bytes, rvx_buffer** out) {
    return guard([&] {
        RVX_REQUIRE(out, RVX_ERR_INVALID_PARAMETER, "null out");
        auto b = std::make_unique<rvx_buffer>();
        b->mem.reset(bytes);
        *out = b.release();
    });
}
rvx_status rvx_buffer_free(rvx_buffer* buf) {
    return guard([&] { delete buf; });
}
int64_t rvx_buffer_bytes(const rvx_buffer* buf) { return buf ? buf->mem.bytes : 0; }
void* rvx_buffer_device_ptr(rvx_buffer* buf) { return buf ? buf->mem.p : nullptr; }
rvx_status rvx_buffer_upload(rvx_buffer* buf, const void* src, int64_t bytes, int64_t offset) {
    return guard([&] { buf->mem.upload(src, bytes, offset); });
}
rvx_status rvx_buffer_download(const rvx_buffer* buf, void* dst, int64_t bytes, int64_t offset) {
    return guard([&] { buf->mem.download(dst, bytes, offset); });
}
rvx_status rvx_buffer_zero(rvx_buffer* buf) {
    return guard([&] {
        if (buf->mem.bytes) RVX_HIP(hipMemsetAsync(buf->mem.p, 0, (size_t)buf->mem.bytes, stream()));
    });
}

rvx_status rvx_buffer_checksum(const rvx_buffer* buf, int64_t offset, int64_t bytes, uint64_t* out) {
    return guard([&] {
        RVX_REQUIRE(buf && out && offset >= 0 && bytes >= 0 && offset <= buf->mem.bytes &&
                        bytes <= buf->mem.bytes - offset,
                    RVX_ERR_INVALID_PARAMETER, "checksum range outside the buffer");
        RVX_REQUIRE(offset % 8 == 0, RVX_ERR_INVALID_PARAMETER, "checksum offset must be a multiple of 8 bytes");
        ComputeLock cl;  // the scratch slot is only valid under the device's compute lock
        auto* d = (uint64_t*)scratch_bytes("checksum", 8);
        checksum((const uint8_t*)buf->mem.p + offset, bytes, d);
        RVX_HIP(hipMemcpyAsync(out, d, 8, hipMemcpyDeviceToHost, stream()));
        sync();
    });
}

rvx_status rvx_profile_enable(int32_t on) {
    return guard([&] {
        std::lock_guard<std::mutex> lk(g_prof.mu);
        g_prof.on = on != 0;
    });
}
rvx_status rvx_profile_reset(void) {
    return guard([&] {
        std::lock_guard<std::mutex> lk(g_prof.mu);
        g_prof.drain();
        g_prof.totals.clear();
        g_prof.order.clear();
    });
}
rvx_status rvx_profile_query(const char* name, double* total_ms, int64_t* launches) {
    return guard([&] {
        std::lock_guard<std::mutex> lk(g_prof.mu);
        g_prof.drain();
        auto it = g_prof.totals.find(name);
        *total_ms = it == g_prof.totals.end() ? 0.0 : it->second.first;
        *launches = it == g_prof.totals.end() ? 0 : it->second.second;
    });
}
rvx_status rvx_profile_names(char* buf, size_t len) {
    return guard([&] {
        std::lock_guard<std::mutex> lk(g_prof.mu);
        g_prof.drain();
        std::string s;
        for (auto& n : g_prof.order) { if (!s.empty()) s += ","; s += n; }
        RVX_REQUIRE(buf && len > s.size(), RVX_ERR_INVALID_PARAMETER, "profile name buffer too small");
        std::memcpy(buf, s.c_str(), s.size() + 1);
    });
}

}  // extern "C"
