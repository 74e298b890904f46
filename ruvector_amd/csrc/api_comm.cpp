// api_comm.cpp — RCCL communicator for node-range sharding over xGMI.
// One process per GPU; the unique id travels over the host launcher's store.
// The only data-path collective of the path is the per-layer all-gather of
// node tables (GNN halo); HNSW shards merge per-shard top-k.
#include <rccl/rccl.h>

#include "comm.hpp"
#include "graph.hpp"

using namespace rvx;

struct rvx_comm {
    ncclComm_t comm = nullptr;  // RCCL transport
    int nranks = 0, rank = 0;
    rvx_host_exchange_fn host_fn = nullptr;  // host-staged transport (rvx_comm_init_host)
    void* host_user = nullptr;
    int64_t sent = 0, recv = 0;  // payload bytes this rank handed to / took from the transport (rvx_comm_traffic)
    int64_t check_rows = 0;      // RVX_COMM_SELF_P2P record check: rows compared (host count) ...
    rvx::DevMem check_words;     // ... and mismatched 32-bit words (device counter)
};

#define RVX_NCCL(expr)                                                                         \
    do {                                                                                       \
        ncclResult_t r_ = (expr);                                                              \
        if (r_ != ncclSuccess) ::rvx::fail(RVX_ERR_COMM, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

static_assert(sizeof(ncclUniqueId) == RVX_COMM_ID_BYTES, "ncclUniqueId size");

namespace rvx {

int comm_rank(const rvx_comm* c) { return c ? c->rank : 0; }
int comm_size(const rvx_comm* c) { return c ? c->nranks : 1; }

// RVX_COMM_SELF_P2P=1 (read per call; tests and `bench.py --force-comm`): an RCCL
// communicator of one rank still runs every collective of the exchange and search paths —
// the grouped ncclSend/ncclRecv of comm_exchange_rows to its own rank, ncclBroadcast,
// ncclAllGather — so the RCCL code runs on a one-GPU box with the results checked
// bit-identical to the path that skips them.
bool comm_self_p2p(const rvx_comm* c) {
    return c && c->comm && c->nranks == 1 && env_int("RVX_COMM_SELF_P2P", 0) != 0;
}

namespace {
__global__ void k_count_mismatch(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b, int64_t words,
                                 unsigned long long* __restrict__ bad) {
    unsigned long long c = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x)
        c += a[i] != b[i] ? 1ull : 0ull;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(bad, c);
}
}  // namespace

void comm_selfcheck_rows(rvx_comm* c, const float* shadow, const float* rows, int64_t nrows, int dim, hipStream_t s) {
    if (!c || nrows <= 0) return;
    if (!c->check_words.p) {
        c->check_words.reset(8);
        RVX_HIP(hipMemsetAsync(c->check_words.p, 0, 8, s));
    }
    const int64_t words = nrows * dim;
    const unsigned blocks = (unsigned)std::min<int64_t>(2048, (words + 255) / 256);
    hipLaunchKernelGGL(k_count_mismatch, dim3(blocks), dim3(256), 0, s, reinterpret_cast<const uint32_t*>(shadow),
                       reinterpret_cast<const uint32_t*>(rows), words, c->check_words.as<unsigned long long>());
    RVX_HIP(hipGetLastError());
    c->check_rows += nrows;
}

namespace {
// Host-staged round: wait for the rows on `s`, copy this rank's block to host,
// let the host transport move every block, copy the peers' blocks back.
void host_exchange_rows(rvx_comm* c, float* table, int64_t row_elems, const int64_t* r0, const int64_t* rows,
                        hipStream_t s) {
    const int me = c->rank, w = c->nranks;
    RVX_HIP(hipStreamSynchronize(s));
    std::vector<float> send((size_t)std::max<int64_t>(rows[me] * row_elems, 1));
    if (rows[me] > 0)
        RVX_HIP(hipMemcpy(send.data(), table + r0[me] * row_elems, (size_t)(rows[me] * row_elems * 4),
                          hipMemcpyDeviceToHost));
    std::vector<std::vector<float>> recv(w);
    std::vector<void*> rptr(w, nullptr);
    std::vector<int64_t> rbytes(w, 0);
    for (int p = 0; p < w; ++p) {
        if (p == me) continue;
        rbytes[p] = rows[p] * row_elems * 4;
        recv[p].resize((size_t)std::max<int64_t>(rows[p] * row_elems, 1));
        rptr[p] = recv[p].data();
    }
    const int32_t rc = c->host_fn(c->host_user, send.data(), rows[me] * row_elems * 4, rptr.data(), rbytes.data());
    RVX_REQUIRE(rc == 0, RVX_ERR_COMM, "host transport failed with status " + std::to_string(rc));
    for (int p = 0; p < w; ++p)
        if (p != me && rows[p] > 0)
            RVX_HIP(hipMemcpyAsync(table + r0[p] * row_elems, recv[p].data(), (size_t)rbytes[p],
                                   hipMemcpyHostToDevice, s));
    RVX_HIP(hipStreamSynchronize(s));  // recv blocks are host temporaries
}
}  // namespace

void comm_exchange_rows(rvx_comm* c, float* table, int64_t row_elems, const int64_t* r0, const int64_t* rows,
                        hipStream_t s) {
    if (comm_self_p2p(c)) {
        // one rank: its block goes out and comes back through RCCL's p2p path (a grouped
        // send/recv pair to itself), lands in a staging buffer and is copied over the rows
        const int64_t cnt = rows[0] * row_elems;
        if (cnt <= 0) return;
        c->sent += cnt * 4;
        c->recv += cnt * 4;
        DevMem stage(cnt * 4);
        RVX_NCCL(ncclGroupStart());
        RVX_NCCL(ncclSend(table + r0[0] * row_elems, (size_t)cnt, ncclFloat32, 0, c->comm, s));
        RVX_NCCL(ncclRecv(stage.p, (size_t)cnt, ncclFloat32, 0, c->comm, s));
        RVX_NCCL(ncclGroupEnd());
        RVX_HIP(hipMemcpyAsync(table + r0[0] * row_elems, stage.p, (size_t)cnt * 4, hipMemcpyDeviceToDevice, s));
        RVX_HIP(hipStreamSynchronize(s));  // the staging buffer is freed on return
        return;
    }
    if (!c || c->nranks <= 1) return;
    for (int p = 0; p < c->nranks; ++p) {
        if (p == c->rank) c->sent += rows[p] * row_elems * 4 * (c->nranks - 1);
        else c->recv += rows[p] * row_elems * 4;
    }
    if (c->host_fn) {
        host_exchange_rows(c, table, row_elems, r0, rows, s);
        return;
    }
    const int me = c->rank;
    RVX_NCCL(ncclGroupStart());
    for (int k = 1; k < c->nranks; ++k) {
        // peers in rotated order so every rank starts on a different link
        const int p = (me + k) % c->nranks;
        if (rows[me] > 0)
            RVX_NCCL(ncclSend(table + r0[me] * row_elems, (size_t)(rows[me] * row_elems), ncclFloat32, p, c->comm, s));
        if (rows[p] > 0)
            RVX_NCCL(ncclRecv(table + r0[p] * row_elems, (size_t)(rows[p] * row_elems), ncclFloat32, p, c->comm, s));
    }
    RVX_NCCL(ncclGroupEnd());
}

void comm_broadcast_bytes(rvx_comm* c, void* buf, int64_t bytes, int root, hipStream_t s) {
    if (bytes > 0 && comm_self_p2p(c) && root == 0) {
        RVX_NCCL(ncclBroadcast(buf, buf, (size_t)bytes, ncclUint8, 0, c->comm, s));
        return;
    }
    if (!c || c->nranks <= 1 || bytes <= 0) return;
    RVX_REQUIRE(root >= 0 && root < c->nranks, RVX_ERR_INVALID_PARAMETER, "bad broadcast root");
    if (c->rank == root) c->sent += bytes * (c->nranks - 1);
    else c->recv += bytes;
    if (!c->host_fn) {
        RVX_NCCL(ncclBroadcast(buf, buf, (size_t)bytes, ncclUint8, root, c->comm, s));
        return;
    }
    // host transport: the root ships its block to every peer, the others receive from the root only
    const int me = c->rank, w = c->nranks;
    RVX_HIP(hipStreamSynchronize(s));
    std::vector<uint8_t> host((size_t)bytes);
    std::vector<void*> rptr(w, nullptr);
    std::vector<int64_t> rbytes(w, 0);
    if (me == root) {
        RVX_HIP(hipMemcpy(host.data(), buf, (size_t)bytes, hipMemcpyDeviceToHost));
    } else {
        rptr[root] = host.data();
        rbytes[root] = bytes;
    }
    const int32_t rc = c->host_fn(c->host_user, host.data(), me == root ? bytes : 0, rptr.data(), rbytes.data());
    RVX_REQUIRE(rc == 0, RVX_ERR_COMM, "host transport failed with status " + std::to_string(rc));
    if (me != root) RVX_HIP(hipMemcpy(buf, host.data(), (size_t)bytes, hipMemcpyHostToDevice));
}

void comm_allgather_bytes(rvx_comm* c, const void* send, void* recv, int64_t bytes, hipStream_t s) {
    const int w = comm_size(c), me = comm_rank(c);
    if (bytes <= 0) return;
    if (comm_self_p2p(c)) {
        RVX_NCCL(ncclAllGather(send, recv, (size_t)bytes, ncclUint8, c->comm, s));
        return;
    }
    if (w <= 1) {
        if (recv != send) RVX_HIP(hipMemcpyAsync(recv, send, (size_t)bytes, hipMemcpyDeviceToDevice, s));
        return;
    }
    c->sent += bytes * (w - 1);
    c->recv += bytes * (w - 1);
    if (!c->host_fn) {
        RVX_NCCL(ncclAllGather(send, recv, (size_t)bytes, ncclUint8, c->comm, s));
        return;
    }
    RVX_HIP(hipStreamSynchronize(s));
    std::vector<uint8_t> mine((size_t)bytes);
    RVX_HIP(hipMemcpy(mine.data(), send, (size_t)bytes, hipMemcpyDeviceToHost));
    std::vector<std::vector<uint8_t>> blk(w);
    std::vector<void*> rptr(w, nullptr);
    std::vector<int64_t> rbytes(w, 0);
    for (int p = 0; p < w; ++p) {
        if (p == me) continue;
        blk[p].resize((size_t)bytes);
        rptr[p] = blk[p].data();
        rbytes[p] = bytes;
    }
    const int32_t rc = c->host_fn(c->host_user, mine.data(), bytes, rptr.data(), rbytes.data());
    RVX_REQUIRE(rc == 0, RVX_ERR_COMM, "host transport failed with status " + std::to_string(rc));
    auto* out = static_cast<uint8_t*>(recv);
    for (int p = 0; p < w; ++p)
        RVX_HIP(hipMemcpy(out + (size_t)p * (size_t)bytes, p == me ? mine.data() : blk[p].data(), (size_t)bytes,
                          hipMemcpyHostToDevice));
}

}  // namespace rvx

extern "C" {

rvx_status rvx_comm_traffic(const rvx_comm* c, int64_t* sent, int64_t* recv) {
    return guard([&] {
        RVX_REQUIRE(c && sent && recv, RVX_ERR_INVALID_PARAMETER, "null argument");
        *sent = c->sent;
        *recv = c->recv;
    });
}

rvx_status rvx_comm_selfcheck(rvx_comm* c, int64_t* rows, int64_t* mismatched_words) {
    return guard([&] {
        RVX_REQUIRE(c && rows && mismatched_words, RVX_ERR_INVALID_PARAMETER, "null argument");
        unsigned long long bad = 0;
        if (c->check_words.p) {
            ComputeLock cl;
            RVX_HIP(hipDeviceSynchronize());  // the checks run on the transfer stream
            RVX_HIP(hipMemcpy(&bad, c->check_words.p, 8, hipMemcpyDeviceToHost));
        }
        *rows = c->check_rows;
        *mismatched_words = (int64_t)bad;
    });
}

rvx_status rvx_comm_unique_id(uint8_t id[RVX_COMM_ID_BYTES]) {
    return guard([&] {
        RVX_REQUIRE(id, RVX_ERR_INVALID_PARAMETER, "null id");
        ncclUniqueId u;
        RVX_NCCL(ncclGetUniqueId(&u));
        std::memcpy(id, &u, sizeof u);
    });
}

rvx_status rvx_comm_init(const uint8_t id[RVX_COMM_ID_BYTES], int32_t nranks, int32_t rank, rvx_comm** out) {
    return guard([&] {
        RVX_REQUIRE(id && out && nranks > 0 && rank >= 0 && rank < nranks, RVX_ERR_INVALID_PARAMETER, "bad comm args");
        device();  // bind the calling thread's device first
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof u);
        auto c = std::make_unique<rvx_comm>();
        RVX_NCCL(ncclCommInitRank(&c->comm, nranks, u, rank));
        c->nranks = nranks;
        c->rank = rank;
        *out = c.release();
    });
}

rvx_status rvx_comm_init_host(int32_t nranks, int32_t rank, rvx_host_exchange_fn fn, void* user, rvx_comm** out) {
    return guard([&] {
        RVX_REQUIRE(fn && out && nranks > 0 && rank >= 0 && rank < nranks, RVX_ERR_INVALID_PARAMETER,
                    "bad host comm args");
        auto c = std::make_unique<rvx_comm>();
        c->nranks = nranks;
        c->rank = rank;
        c->host_fn = fn;
        c->host_user = user;
        *out = c.release();
    });
}

rvx_status rvx_comm_destroy(rvx_comm* c) {
    return guard([&] {
        if (c && c->comm) ncclCommDestroy(c->comm);
        delete c;
    });
}

rvx_status rvx_comm_allgather_f32(rvx_comm* c, const rvx_buffer* send, int64_t count, rvx_buffer* recv) {
    return guard([&] {
        RVX_REQUIRE(c && send && recv && count >= 0, RVX_ERR_INVALID_PARAMETER, "bad all-gather args");
        RVX_REQUIRE(c->comm, RVX_ERR_UNSUPPORTED, "all-gather needs the RCCL transport");
        RVX_REQUIRE(send->mem.bytes >= count * 4 && recv->mem.bytes >= count * 4 * c->nranks, RVX_ERR_INVALID_PARAMETER,
                    "all-gather buffers too small");
        ProfScope ps("rccl_allgather");
        RVX_NCCL(ncclAllGather(send->mem.p, recv->mem.p, (size_t)count, ncclFloat32, c->comm, stream()));
    });
}

rvx_status rvx_comm_allreduce_max_f64(rvx_comm* c, double* value) {
    return guard([&] {
        RVX_REQUIRE(c && value, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(c->comm, RVX_ERR_UNSUPPORTED, "all-reduce needs the RCCL transport");
        double* d = (double*)scratch_bytes("comm_scalar", 8);
        RVX_HIP(hipMemcpyAsync(d, value, 8, hipMemcpyHostToDevice, stream()));
        RVX_NCCL(ncclAllReduce(d, d, 1, ncclFloat64, ncclMax, c->comm, stream()));
        RVX_HIP(hipMemcpyAsync(value, d, 8, hipMemcpyDeviceToHost, stream()));
        sync();
    });
}

rvx_status rvx_comm_allreduce_f64(rvx_comm* c, double* values, int32_t count, int32_t op) {
    return guard([&] {
        RVX_REQUIRE(c && values && count >= 0, RVX_ERR_INVALID_PARAMETER, "bad all-reduce args");
        RVX_REQUIRE(op >= RVX_REDUCE_SUM && op <= RVX_REDUCE_MIN, RVX_ERR_INVALID_PARAMETER, "unknown reduce op");
        RVX_REQUIRE(c->comm, RVX_ERR_UNSUPPORTED, "all-reduce needs the RCCL transport");
        if (count == 0) return;
        const ncclRedOp_t rop = op == RVX_REDUCE_SUM ? ncclSum : op == RVX_REDUCE_MAX ? ncclMax : ncclMin;
        double* d = (double*)scratch_bytes("comm_scalars", (int64_t)count * 8);
        RVX_HIP(hipMemcpyAsync(d, values, (size_t)count * 8, hipMemcpyHostToDevice, stream()));
        RVX_NCCL(ncclAllReduce(d, d, (size_t)count, ncclFloat64, rop, c->comm, stream()));
        RVX_HIP(hipMemcpyAsync(values, d, (size_t)count * 8, hipMemcpyDeviceToHost, stream()));
        sync();
    });
}

}  // extern "C"
