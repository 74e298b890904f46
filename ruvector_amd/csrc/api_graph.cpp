// api_graph.cpp — graph handles, scratch pool and the message-passing layers
// of crates/ruvector-postgres/src/gnn (GraphSAGE, GCN, aggregators).
#include <algorithm>
#include <cmath>

#include <functional>

#include "comm.hpp"
#include "graph.hpp"
#include "kernels.hpp"

namespace rvx {

namespace {
std::mutex g_scratch_mu;
std::map<std::pair<int, std::string>, std::unique_ptr<DevMem>> g_scratch;
std::map<int, std::unique_ptr<std::recursive_mutex>> g_compute_mu;
}  // namespace

void* scratch_bytes(const std::string& slot, int64_t bytes) {
    const int dev = device().id;
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    auto& m = g_scratch[{dev, slot}];
    if (!m) m = std::make_unique<DevMem>();
    if (m->bytes < bytes) m->reset(std::max<int64_t>(bytes, 256));
    return m->p;
}
float* scratch_f32(const std::string& slot, int64_t count) { return (float*)scratch_bytes(slot, count * 4); }
void scratch_release_all() {
    const int dev = device().id;
    RVX_HIP(hipDeviceSynchronize());
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    for (auto it = g_scratch.begin(); it != g_scratch.end();) {
        if (it->first.first == dev) it = g_scratch.erase(it);
        else ++it;
    }
}
int64_t scratch_held(const std::string& slot) {
    const int dev = device().id;
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    auto it = g_scratch.find({dev, slot});
    return it == g_scratch.end() || !it->second ? 0 : it->second->bytes;
}

ComputeLock::ComputeLock() {
    const int dev = device().id;
    std::recursive_mutex* mu;
    {
        std::lock_guard<std::mutex> lk(g_scratch_mu);
        auto& p = g_compute_mu[dev];
        if (!p) p = std::make_unique<std::recursive_mutex>();
        mu = p.get();
    }
    lk = std::unique_lock<std::recursive_mutex>(*mu);
}

void check_graph(const rvx_graph* g) {
    RVX_REQUIRE(g && g->row_ptr && (g->e == 0 || g->col), RVX_ERR_INVALID_PARAMETER, "null graph");
}

// hand-off events sage_forward_dev uses (callers that add their own take them after these)
#define SAGE_PIPE_EVENTS(chunks) (2 * (chunks) + 3)

// Row chunking of the layer pipeline (same on every rank for a given chunk count).
int sage_chunks_for(int64_t n) {
    // 24 chunks with the gather capped at one block per CU (k_aggregate.hip):
    // 1.46G vs 1.37G edges/s for 16 uncapped at 10M x 768 (scripts/exp_sweep3.sh); 48 once
    // the GEMM helps the gather (smaller lone first gather / last GEMM per layer): 399.7 /
    // 425.8 / 401.2 / 406.0 vs 433.7 / 427.5 / 419.9 / 427.9 ms/step for 24
    // (scripts/exp_help_chunks.sh, profiles/r03_help_chunks.txt)
    const int pipe_chunks = std::max(1, env_int("RVX_SAGE_CHUNKS", 48));
    return n >= (int64_t)pipe_chunks * 16384 ? pipe_chunks : 1;
}
int64_t chunk_step(int64_t n, int chunks) { return ((n + chunks - 1) / chunks + 127) / 128 * 128; }

std::vector<ExchangeRound> exchange_plan(int kind, const int64_t* offsets, int world) {
    std::vector<ExchangeRound> plan;
    if (kind == PLAN_WHOLE) {
        ExchangeRound r;
        for (int p = 0; p < world; ++p) {
            r.r0.push_back(offsets[p]);
            r.rows.push_back(offsets[p + 1] - offsets[p]);
        }
        plan.push_back(r);
        return plan;
    }
    // every rank uses the chunk count of the largest shard, so the p2p rounds
    // pair up (a shard with fewer real chunks sends empty ones)
    int64_t maxn = 0;
    for (int p = 0; p < world; ++p) maxn = std::max(maxn, offsets[p + 1] - offsets[p]);
    const int chunks = sage_chunks_for(maxn);
    for (int c = 0; c < chunks; ++c) {
        ExchangeRound r;
        for (int p = 0; p < world; ++p) {
            const int64_t np = offsets[p + 1] - offsets[p];
            const int64_t st = chunk_step(np, chunks);
            const int64_t b = std::min(np, (int64_t)c * st);
            r.r0.push_back(offsets[p] + b);
            r.rows.push_back(std::min(st, np - b));
        }
        plan.push_back(r);
    }
    return plan;
}

void produce_and_exchange(rvx_comm* comm, const int64_t* offsets, const std::vector<TableRef>& tables,
                          const std::function<void(int64_t r0, int64_t rows)>& produce) {
    const int world = comm_size(comm), me = comm_rank(comm);
    if (world <= 1 && !comm_self_p2p(comm)) {
        produce(offsets[me], offsets[me + 1] - offsets[me]);
        return;
    }
    const std::vector<ExchangeRound> plan = exchange_plan(PLAN_SAGE, offsets, world);
    const int rounds = (int)plan.size();
    Device& d = device();
    hipEvent_t* ev = pipeline_events(rounds + 1);
    RVX_HIP(hipEventRecord(ev[rounds], d.stream));  // the transfer stream may not write rows still being read
    RVX_HIP(hipStreamWaitEvent(d.xfer, ev[rounds], 0));
    for (int c = 0; c < rounds; ++c) {
        if (plan[c].rows[me] > 0) produce(plan[c].r0[me], plan[c].rows[me]);
        RVX_HIP(hipEventRecord(ev[c], d.stream));
        RVX_HIP(hipStreamWaitEvent(d.xfer, ev[c], 0));
        StreamScope on_xfer(d.xfer);
        ProfScope ps("halo_exchange");
        for (const TableRef& t : tables) comm_exchange_rows(comm, t.first, t.second, plan[c].r0.data(), plan[c].rows.data(), d.xfer);
    }
    RVX_HIP(hipEventRecord(ev[rounds], d.xfer));
    ProfScope ps("exchange_wait");  // the exchange tail the compute stream waits for
    RVX_HIP(hipStreamWaitEvent(d.stream, ev[rounds], 0));
}

namespace {

// Finish a graph once row_ptr/col are on the device and a host row_ptr is known.
void finish_graph(rvx_graph* g, const std::vector<int64_t>& rp) {
    std::vector<int32_t> iso;
    int64_t maxd = 0;
    for (int64_t i = 0; i < g->n; ++i) {
        const int64_t d = rp[i + 1] - rp[i];
        RVX_REQUIRE(d >= 0, RVX_ERR_INVALID_PARAMETER, "row_ptr must be non-decreasing");
        maxd = std::max(maxd, d);
        if (d == 0) iso.push_back((int32_t)i);
    }
    RVX_REQUIRE(maxd < ((int64_t)1 << 31), RVX_ERR_INVALID_SHAPE, "degree too large");
    g->max_deg = (int32_t)maxd;
    g->n_isolated = (int64_t)iso.size();
    if (!iso.empty()) {
        g->isolated_mem.reset((int64_t)iso.size() * 4);
        g->isolated_mem.upload(iso.data(), (int64_t)iso.size() * 4);
        g->isolated = g->isolated_mem.as<int32_t>();
    }
}

void upload_csr(rvx_graph* g, const std::vector<int64_t>& rp, const int32_t* col, const float* w) {
    g->row_ptr_mem.reset((g->n + 1) * 8);
    g->row_ptr_mem.upload(rp.data(), (g->n + 1) * 8);
    g->row_ptr = g->row_ptr_mem.as<int64_t>();
    g->col_mem.reset(std::max<int64_t>(g->e, 1) * 4);
    g->col_mem.upload(col, g->e * 4);
    g->col = g->col_mem.as<int32_t>();
    if (w) {
        g->w_mem.reset(std::max<int64_t>(g->e, 1) * 4);
        g->w_mem.upload(w, g->e * 4);
        g->w = g->w_mem.as<float>();
        g->host_w.assign(w, w + g->e);
    }
    finish_graph(g, rp);
}

// GraphSAGELayer::with_aggregator deterministic init (graphsage.rs:56-78) and
// GCNLayer::new_with_normalize (gcn.rs:32-41): W[i][j] = (((i*out+j+off) as f32 * 0.01) % 1.0 - 0.5) * scale.
std::vector<float> det_init(int in, int out, int offset) {
    const float scale = std::sqrt(2.0f / (float)(in + out));
    std::vector<float> w((size_t)in * out);
    for (int64_t i = 0; i < in; ++i)
        for (int64_t j = 0; j < out; ++j) {
            const float val = std::fmod((float)(uint64_t)(i * out + j + offset) * 0.01f, 1.0f);
            w[(size_t)(i * out + j)] = (val - 0.5f) * scale;
        }
    return w;
}

// Upload an [in][out] matrix as its transpose [out][in] (the GEMM's K-contiguous B).
void upload_transposed(DevMem& dst, const std::vector<float>& w_in_out, int in, int out) {
    std::vector<float> t((size_t)in * out);
    for (int64_t i = 0; i < in; ++i)
        for (int64_t j = 0; j < out; ++j) t[(size_t)(j * in + i)] = w_in_out[(size_t)(i * out + j)];
    dst.reset((int64_t)t.size() * 4);
    dst.upload(t.data(), (int64_t)t.size() * 4);
}

}  // namespace
}  // namespace rvx

using namespace rvx;

struct rvx_sage_layer {
    int in = 0, out = 0, num_samples = 0, aggregator = 0, normalize = 1;
    std::vector<float> wn, ws;  // host [in][out]
    DevMem wn_t, ws_t;          // device [out][in]
    DevMem wn_x3, ws_x3;        // exact 3-way bf16 splits of wn_t / ws_t (split-bf16 MFMA GEMM)
    DevMem wn_h2, ws_h2, w_inv; // f16 [hi][lo] planes of wn_t / ws_t scaled per output feature (split-f16 GEMM)
};

struct rvx_gcn_layer {
    int in = 0, out = 0, normalize = 1;
    std::vector<float> w, b;
    DevMem w_t, bias;
};

namespace {


// Called on the host after chunk c's launches are queued (rows [r0, r0+rows)
// of y, possibly empty); the chunk's output is complete at that point of the
// library stream.
using ChunkHook = std::function<void(int c, int64_t r0, int64_t rows)>;

// The layer runs the in-register split-f16 dual GEMM (gemm_nt_h2, h2g) — the path that
// can take a deferred normalisation (below) — rather than h2p, the fused kernel or the
// split-bf16 / fp32 GEMMs. Same conditions as sage_forward_dev's choice.
bool sage_defer_path(const rvx_sage_layer* l, int64_t n, const float* x, const float* y, int64_t row_offset) {
    const GemmOperand w0{nullptr, 2 * l->in, nullptr, l->in, l->in, nullptr, 0, l->wn_h2.as<_Float16>(), 0, nullptr};
    const int64_t a_plane = std::max<int64_t>(n, 1) * 2 * l->in;
    const bool h2p = l->wn_h2.p && l->in <= 1024 && l->in % 4 == 0 && ((uintptr_t)x & 15) == 0 &&
                     gemm_h2p_ok(std::max<int64_t>(n, 1), l->out, 2 * l->in, a_plane, w0, &w0);
    if (h2p || !l->wn_h2.p || l->in > 1024 || l->out > 1024 || ((uintptr_t)x & 15) != 0 || l->in % 4 != 0)
        return false;
    // the aggregate scratch is hipMalloc'd (aligned): x stands in for its alignment check
    if (!gemm_h2_ok(std::max<int64_t>(n, 1), l->out, GemmOperand{x, l->in, nullptr, l->in, l->in}, nullptr)) return false;
    const int64_t wplane = (int64_t)l->in * l->out;
    return !sage_gemm_fused_ok(std::max<int64_t>(n, 1), l->out, l->in, l->in, l->in, l->in, l->in, l->in, wplane,
                               wplane, l->out, x, x + row_offset * l->in, y);
}

__global__ void k_rows_inv_norm(const float* __restrict__ ssq, int stride, int tiles, int64_t rows,
                                float* __restrict__ inv) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    float s = 0.0f;
    for (int t = 0; t < tiles; ++t) s = __fadd_rn(s, ssq[r * stride + t]);
    const float norm = sqrtf(s);
    inv[r] = norm > 0.0f ? 1.0f / norm : 1.0f;  // rows with norm 0 / NaN stay as they are (normalize_rows)
}

__global__ void k_fill_value(float* __restrict__ p, int64_t n, float v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}
void fill_value(float* p, int64_t n, float v) {
    if (n > 0) RVX_LAUNCH("fill_value", k_fill_value, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, p, n, v);
}

__global__ void k_scale_rows(float* __restrict__ x, int64_t rows, int dim, const float* __restrict__ mul) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows * dim) return;
    x[i] *= mul[i / dim];
}

// x: node table indexed by the CSR columns; rows [row_offset, row_offset+g->n)
// of it are this graph's destination (self) rows.
// Deferred normalisation (h2g path only, sage_defer_path): x_mul (nullable) holds a
// multiplier for every row of x (the previous layer's 1/|y|, applied as rows are gathered
// and in the GEMM's self-operand split); y_inv (nullable) makes the layer leave its output
// rows unnormalised and write 1/|y| per row instead (from the GEMM epilogue's per-tile
// sums of squares) — the pass that re-reads and re-writes y is not run.
// Row images (RowImage, kernels.hpp; both optional): x_img, an image of every row of x (global
// row ids), lets the overlapped gather read ReLU-sparse neighbour rows from it; y_img (indexed
// like y, i.e. this graph's rows) receives the image of each output row chunk as it completes.
void sage_forward_dev(const rvx_sage_layer* l, const rvx_graph* g, const float* x, float* y, int64_t row_offset = 0,
                      int chunks = 0, const ChunkHook& hook = nullptr, const float* x_mul = nullptr,
                      float* y_inv = nullptr, RowImage x_img = RowImage(), RowImage y_img = RowImage()) {
    // rows with more than num_samples neighbours aggregate the reference's
    // sample_neighbors subset (graphsage.rs:92-102, k_sample.hip)
    g = sampled_graph(g, l->num_samples);
    const int64_t n = g->n;
    const int a = (l->aggregator == RVX_SAGE_MAXPOOL) ? AGG_MAX : AGG_MEAN;
    // split-f16 dual GEMM when the shapes allow it: the gather also emits the
    // per-row operand scale over the aggregate and self rows, and (h2p) the
    // scaled [aggregate | self] operand itself as two f16 planes, so the GEMM
    // k-loop does no conversion work
    const int64_t plane = (int64_t)l->in * l->out;
    const GemmOperand w0{nullptr, 2 * l->in, nullptr, l->in, l->in, nullptr, 0, l->wn_h2.as<_Float16>(), 0, nullptr};
    const int64_t a_plane = std::max<int64_t>(n, 1) * 2 * l->in;
    const bool h2p = l->wn_h2.p && l->in <= 1024 && l->in % 4 == 0 && ((uintptr_t)x & 15) == 0 &&
                     gemm_h2p_ok(std::max<int64_t>(n, 1), l->out, 2 * l->in, a_plane, w0, &w0);
    float* agg = h2p ? nullptr : scratch_f32("sage_agg", n * (int64_t)l->in);
    _Float16* aplanes = h2p ? (_Float16*)scratch_bytes("sage_aplanes", a_plane * 2 * 2) : nullptr;
    const bool h2 = h2p || (l->wn_h2.p && l->in <= 1024 && ((uintptr_t)x & 15) == 0 &&
                            gemm_h2_ok(std::max<int64_t>(n, 1), l->out,
                                       GemmOperand{agg, l->in, nullptr, l->in, l->in}, nullptr) &&
                            gemm_h2_ok(std::max<int64_t>(n, 1), l->out, GemmOperand{x, l->in, nullptr, l->in, l->in},
                                       nullptr));
    float* scale = h2 ? scratch_f32("sage_scale", std::max<int64_t>(n, 1)) : nullptr;
    // the dual GEMM with ReLU + normalisation fused, one block per 64 rows x all columns:
    // A read once, no normalise pass (k_sage_gemm.hip); same bits as gemm_nt_h2 + normalize_rows
    const int64_t wplane = (int64_t)l->in * l->out;
    const bool fused = h2 && !h2p &&
                       sage_gemm_fused_ok(std::max<int64_t>(n, 1), l->out, l->in, l->in, l->in, l->in, l->in, l->in,
                                          wplane, wplane, l->out, agg, x + row_offset * l->in, y);
    GemmEpilogue ep;
    ep.epi = GEMM_EPI_RELU;
    RVX_REQUIRE((!x_mul && !y_inv) || (h2 && !h2p && !fused), RVX_ERR_UNSUPPORTED,
                "deferred normalisation needs the split-f16 GEMM path");
    const int ntiles = ROWSUMSQ_SLOTS;
    float* ssq = y_inv ? scratch_f32("sage_sumsq", std::max<int64_t>(n, 1) * ntiles) : nullptr;
    // Rows are independent, so the layer runs as a two-stage pipeline over
    // row chunks: the HBM-bound gather of chunk c+1 (aux stream) overlaps the
    // MFMA-bound GEMM + normalisation of chunk c (library stream). Every row
    // sees the same arithmetic as the unchunked layer.
    if (chunks <= 0) chunks = sage_chunks_for(n);
    const int64_t step = chunk_step(n, chunks);
    Device& d = device();
    hipEvent_t* ev = pipeline_events(SAGE_PIPE_EVENTS(chunks));
    hipEvent_t* evg = ev + chunks + 2;  // GEMM of chunk c done (normalise stream hand-off)
    // Opt-in (RVX_SAGE_NORM_STREAM=1, read per call): the row normalisation of chunk c on a
    // third stream beside the GEMM of chunk c+1 instead of between the GEMMs. Three kernels
    // at once slow the gather and the GEMM more than the pass costs in line: 488 vs
    // 435-466 ms/step at 10M x 768 (scripts/exp_norm_stream.sh).
    const bool norm_side = chunks > 1 && l->normalize && env_int("RVX_SAGE_NORM_STREAM", 0);
    // RVX_SAGE_CU_SPLIT (experiment, read per call): the GEMM and the gather on
    // two streams owning disjoint CU halves instead of sharing every CU
    const int split = chunks > 1 ? env_int("RVX_SAGE_CU_SPLIT", 0) : 0;
    hipStream_t main_s = d.stream, gath_s = d.aux;
    int main_cus = 0, gath_cus = 0;
    if (split > 0) {
        hipStream_t ss[2];
        int cc[2];
        cu_split_streams(split, ss, cc);
        main_s = ss[0]; gath_s = ss[1]; main_cus = cc[0]; gath_cus = cc[1];
    }
    if (chunks > 1) {
        RVX_HIP(hipEventRecord(ev[chunks], d.stream));  // aux may not overwrite agg before earlier work is done
        RVX_HIP(hipStreamWaitEvent(gath_s, ev[chunks], 0));
        if (main_s != d.stream) RVX_HIP(hipStreamWaitEvent(main_s, ev[chunks], 0));
        if (norm_side) RVX_HIP(hipStreamWaitEvent(d.aux2, ev[chunks], 0));
    }
    // RVX_SAGE_NORM_AUX (opt-in, read per call; no hooks or images): the row normalisation
    // of chunk c runs on the gather stream after the gather of chunk c+1 (and after the GEMM
    // of chunk c), before the gather of chunk c+2, instead of between the GEMMs of chunks c and
    // c+1 — the GEMM of chunk c+1 no longer waits for it, and at most two kernels share the
    // chip at any time (the third-stream form above had three). Same kernel, same bits.
    const bool norm_aux = chunks > 1 && l->normalize && !hook && !y_img && !norm_side && split == 0 &&
                          env_int("RVX_SAGE_NORM_AUX", 0);
    struct PendingNorm { bool on = false; int cc = 0; int64_t rr0 = 0, rrows = 0; } pend;
    auto flush_norm = [&]() {  // on the gather stream, behind the gather just queued there
        if (!pend.on) return;
        RVX_HIP(hipStreamWaitEvent(gath_s, evg[pend.cc], 0));
        StreamScope on_gather(gath_s);
        normalize_rows(y + pend.rr0 * l->out, pend.rrows, l->out, true, "sage_normalize");
        pend.on = false;
    };
    // chunk c's output finished by the GEMM: normalise it (third stream or in line), then
    // the caller's hook on the stream that completed the rows
    auto finish_chunk = [&](int cc, int64_t rr0, int64_t rrows, bool norm) {
        if (norm && norm_aux) {
            RVX_HIP(hipEventRecord(evg[cc], main_s));  // the GEMM of chunk cc is done
            pend.on = true; pend.cc = cc; pend.rr0 = rr0; pend.rrows = rrows;
            return;
        }
        if (norm && norm_side) {
            RVX_HIP(hipEventRecord(evg[cc], main_s));
            RVX_HIP(hipStreamWaitEvent(d.aux2, evg[cc], 0));
            StreamScope on_norm(d.aux2);
            normalize_rows(y + rr0 * l->out, rrows, l->out, true, "sage_normalize");
            if (y_img) rows_image_pack(y, rr0, rrows, l->out, y_img);
            if (hook) hook(cc, rr0, rrows);
            return;
        }
        if (norm) normalize_rows(y + rr0 * l->out, rrows, l->out, true, "sage_normalize");
        if (y_img) rows_image_pack(y, rr0, rrows, l->out, y_img);
        if (hook) {
            if (norm_side) {  // keep the hooks in chunk order on the normalise stream
                RVX_HIP(hipEventRecord(evg[cc], main_s));
                RVX_HIP(hipStreamWaitEvent(d.aux2, evg[cc], 0));
                StreamScope on_norm(d.aux2);
                hook(cc, rr0, rrows);
            } else {
                hook(cc, rr0, rrows);
            }
        }
    };
    // Dynamic gather (RVX_SAGE_HELP, default on; read per call, tests cover both): chunk c's
    // gather takes its rows from a counter, and the persistent GEMM of chunk c-1 joins it once
    // its tiles are done — without it the GEMM's CU slots idle for the last ~third of every
    // chunk while the gather runs on one block per CU. Same rows, same arithmetic, same bits.
    const bool help = chunks > 1 && h2 && !h2p && !fused && split == 0 &&
                      env_int("RVX_SAGE_GEMM_CAP", 2) > 0 && env_int("RVX_GEMM_WIDE", 3) == 3 &&
                      agg_help_ok(l->in, x, agg, x + row_offset * l->in);
    unsigned* counters = nullptr;
    if (help) {
        counters = (unsigned*)scratch_bytes("sage_help_counters", (int64_t)chunks * 64);
        RVX_HIP(hipMemsetAsync(counters, 0, (size_t)chunks * 64, d.stream));
        // (recorded into ev[chunks] below, before the gather stream's first launch)
        RVX_HIP(hipEventRecord(ev[chunks], d.stream));
        RVX_HIP(hipStreamWaitEvent(gath_s, ev[chunks], 0));
    }
    // imaged rows expanded in registers (1, default) or through LDS windows (0); read per call
    const int img_reg = env_int("RVX_IMG_REG", 1) != 0 ? 1 : 0;
    auto help_of = [&](int64_t rr0) {
        AggHelp h{};
        h.rp = g->row_ptr + rr0; h.col = g->col; h.n = std::min(step, n - rr0);
        h.x = x; h.dim = l->in; h.agg = a;
        h.out = agg + rr0 * l->in; h.self_x = x + (row_offset + rr0) * l->in; h.row_scale = scale + rr0;
        h.row_mul = x_mul; h.self_mul = x_mul ? x_mul + row_offset + rr0 : nullptr;
        h.counter = counters + (rr0 / step) * 16;
        if (x_img && row_image_ok(l->in) && a != AGG_MAX) {
            h.img_slots = x_img.slots;
            h.img_nnz = x_img.nnz;
            h.img_reg = img_reg;
        }
        return h;
    };
    StreamScope on_main(main_s);
    CuScope main_cu(main_cus);
    int c = 0;
    for (int64_t r0 = 0; r0 < n; r0 += step, ++c) {
        const int64_t rows = std::min(step, n - r0);
        if (chunks > 1 && help) {
            StreamScope on_aux(gath_s);
            // the layer's first chunk has no GEMM beside it: a wider grid (RVX_AGG_FIRST_CAP
            // blocks per CU, read per call; same rows, same bits)
            const AggHelp hc = help_of(r0);
            aggregate_rows_help(hc, hc.img_slots ? "sage_aggregate_img" : "sage_aggregate",
                                c == 0 ? env_int("RVX_AGG_FIRST_CAP", 4) : 0);
            RVX_HIP(hipEventRecord(ev[c], gath_s));
            RVX_HIP(hipStreamWaitEvent(main_s, ev[c], 0));
            flush_norm();  // chunk c-1's normalisation, behind gather c
        } else if (chunks > 1) {
            StreamScope on_aux(gath_s);
            CuScope aux_cu(gath_cus);
            aggregate_rows(g->row_ptr + r0, g->col, nullptr, rows, x, l->in, a, /*empty_fill zeros*/ 0, 0,
                           h2p ? nullptr : agg + r0 * l->in, "sage_aggregate", /*overlapped*/ true,
                           x + (row_offset + r0) * l->in, h2 ? scale + r0 : nullptr,
                           h2p ? aplanes + r0 * 2 * l->in : nullptr, a_plane, x_mul,
                           x_mul ? x_mul + row_offset + r0 : nullptr);
            RVX_HIP(hipEventRecord(ev[c], gath_s));
            RVX_HIP(hipStreamWaitEvent(main_s, ev[c], 0));
            flush_norm();
        } else {
            aggregate_rows(g->row_ptr, g->col, nullptr, n, x, l->in, a, 0, 0, agg, "sage_aggregate", false,
                           x + row_offset * l->in, scale, aplanes, a_plane, x_mul, x_mul ? x_mul + row_offset : nullptr);
        }
        if (h2p) {
            GemmOperand s0{nullptr, 2 * l->in, nullptr, l->in, l->in};
            gemm_nt_h2p(rows, l->out, aplanes + r0 * 2 * l->in, 2 * l->in, a_plane, s0, l->wn_h2.as<_Float16>(), &s0,
                        l->ws_h2.as<_Float16>(), scale + r0, l->w_inv.as<float>(), ep, y + r0 * l->out, l->out,
                        "sage_gemm");
            finish_chunk(c, r0, rows, l->normalize != 0);
            continue;
        }
        if (fused) {
            sage_gemm_fused(rows, l->out, agg + r0 * l->in, l->in, l->in, x + (row_offset + r0) * l->in, l->in, l->in,
                            l->wn_h2.as<_Float16>(), l->in, wplane, l->ws_h2.as<_Float16>(), l->in, wplane, scale + r0,
                            l->w_inv.as<float>(), y + r0 * l->out, l->out, l->normalize != 0, "sage_gemm");
            finish_chunk(c, r0, rows, false);
            continue;
        }
        GemmOperand s0{agg + r0 * l->in, l->in, l->wn_t.as<float>(), l->in, l->in, l->wn_x3.as<uint16_t>(), plane};
        GemmOperand s1{x + (row_offset + r0) * l->in, l->in, l->ws_t.as<float>(), l->in, l->in,
                       l->ws_x3.as<uint16_t>(), plane};
        // opt-in: the h2g GEMM normalises its own rows (last column tile of each 128-row
        // block, same bits as normalize_rows) instead of a separate pass over y
        GemmEpilogue epn = ep;
        epn.normalize_rows = h2 && l->normalize && !y_inv && gemm_h2_rownorm_ok(l->out, y, l->out);
        epn.a1_rowmul = x_mul ? x_mul + row_offset + r0 : nullptr;
        epn.row_sumsq = y_inv ? ssq + r0 * ntiles : nullptr;
        AggHelp next{};
        if (help && r0 + step < n && env_int("RVX_SAGE_HELP", 1) != 2) {  // 2: dynamic gather alone
            next = help_of(r0 + step);
            epn.help = &next;
        }
        int coltiles = 0;
        if (h2)
            coltiles = gemm_nt_h2(rows, l->out, s0, l->wn_h2.as<_Float16>(), &s1, l->ws_h2.as<_Float16>(), scale + r0,
                                  l->w_inv.as<float>(), epn, y + r0 * l->out, l->out, "sage_gemm",
                                  chunks > 1 ? env_int("RVX_SAGE_GEMM_CAP", 2) : -1);
        else
            gemm_nt(rows, l->out, s0, &s1, ep, y + r0 * l->out, l->out, "sage_gemm");
        if (y_inv && rows > 0) {
            if (l->normalize) {
                RVX_LAUNCH("sage_inv_norm", k_rows_inv_norm, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0,
                           ssq + r0 * ntiles, ntiles, coltiles, rows, y_inv + r0);
            } else {
                fill_value(y_inv + r0, rows, 1.0f);
            }
        }
#ifndef RVX_AB_NO_NORMALIZE  // timing-only ablation build (scripts/exp_sage_ablate.sh): results wrong
        finish_chunk(c, r0, rows, l->normalize && !epn.normalize_rows && !y_inv);
#else
        finish_chunk(c, r0, rows, false);
#endif
    }
    flush_norm();  // the last chunk's
    for (; hook && c < chunks; ++c) finish_chunk(c, n, 0, false);
    if (main_s != d.stream) {
        RVX_HIP(hipEventRecord(ev[chunks + 1], main_s));
        RVX_HIP(hipStreamWaitEvent(d.stream, ev[chunks + 1], 0));
    }
    if (norm_side) {  // the normalise stream's last chunk (and hooks) before anything after the layer
        RVX_HIP(hipEventRecord(evg[chunks], d.aux2));
        RVX_HIP(hipStreamWaitEvent(d.stream, evg[chunks], 0));
    }
    if (norm_aux) {  // the gather stream's last normalisation before anything after the layer
        RVX_HIP(hipEventRecord(evg[chunks], gath_s));
        RVX_HIP(hipStreamWaitEvent(d.stream, evg[chunks], 0));
    }
}

__global__ void k_gcn_isolated(const int32_t* iso, int64_t n_iso, const float* x, int dim, float* y) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = n_iso * dim;
    if (i >= total) return;
    const int64_t r = iso[i / dim];
    const int c = (int)(i % dim);
    y[r * dim + c] = fmaxf(x[r * dim + c], 0.0f);
}

void gcn_forward_dev(const rvx_gcn_layer* l, const rvx_graph* g, bool use_w, const float* x, float* y) {
    const int64_t n = g->n;
    RVX_REQUIRE(g->n_isolated == 0 || l->in == l->out, RVX_ERR_INVALID_SHAPE,
                "GCN passes isolated nodes through unchanged (message_passing.rs:75-78); needs in == out");
    const float* w = use_w ? g->w : nullptr;
    float* agg = scratch_f32("gcn_agg", n * (int64_t)l->in);
    aggregate_rows(g->row_ptr, g->col, w, n, x, l->in, AGG_SUM, 0, l->normalize ? 1 : 0, agg, "gcn_aggregate");
    GemmOperand s0{agg, l->in, l->w_t.as<float>(), l->in, l->in};
    GemmEpilogue ep;
    ep.epi = GEMM_EPI_RELU;
    ep.bias0 = l->bias.as<float>();
    gemm_nt(n, l->out, s0, nullptr, ep, y, l->out, "gcn_gemm");
    if (g->n_isolated) {
        const int64_t total = g->n_isolated * l->in;
        hipLaunchKernelGGL(k_gcn_isolated, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream(), g->isolated,
                           g->n_isolated, x, l->in, y);
        RVX_HIP(hipGetLastError());
    }
}

}  // namespace

extern "C" {

rvx_status rvx_scratch_release(void) {
    return guard([&] {
        ComputeLock cl;
        scratch_release_all();
    });
}


rvx_status rvx_graph_from_edges(int64_t n, const int64_t* src, const int64_t* dst, int64_t ne, const float* ew,
                                rvx_graph** out) {
    return guard([&] {
        RVX_REQUIRE(out && n >= 0 && n < ((int64_t)1 << 31) && ne >= 0, RVX_ERR_INVALID_PARAMETER, "bad graph args");
        RVX_REQUIRE(ne == 0 || (src && dst), RVX_ERR_INVALID_PARAMETER, "null edge arrays");
        // Stable counting sort by destination, dropping out-of-range edges
        // (build_adjacency_list, message_passing.rs:43-47).
        std::vector<int64_t> rp(n + 1, 0);
        for (int64_t e = 0; e < ne; ++e)
            if (src[e] >= 0 && src[e] < n && dst[e] >= 0 && dst[e] < n) rp[dst[e] + 1]++;
        for (int64_t i = 0; i < n; ++i) rp[i + 1] += rp[i];
        const int64_t kept = rp[n];
        std::vector<int32_t> col(std::max<int64_t>(kept, 1));
        std::vector<float> w(ew ? std::max<int64_t>(kept, 1) : 0);
        std::vector<int64_t> fill(rp.begin(), rp.end() - 1);
        for (int64_t e = 0; e < ne; ++e) {
            if (!(src[e] >= 0 && src[e] < n && dst[e] >= 0 && dst[e] < n)) continue;
            const int64_t p = fill[dst[e]]++;
            col[p] = (int32_t)src[e];
            if (ew) w[p] = ew[e];
        }
        auto g = std::make_unique<rvx_graph>();
        g->n = n;
        g->e = kept;
        upload_csr(g.get(), rp, col.data(), ew ? w.data() : nullptr);
        *out = g.release();
    });
}

rvx_status rvx_graph_from_csr(int64_t n, const int64_t* row_ptr, const int32_t* col, const float* ew, rvx_graph** out) {
    return guard([&] {
        RVX_REQUIRE(out && row_ptr && n >= 0 && n < ((int64_t)1 << 31), RVX_ERR_INVALID_PARAMETER, "bad CSR args");
        RVX_REQUIRE(row_ptr[0] == 0, RVX_ERR_INVALID_PARAMETER, "row_ptr[0] must be 0");
        std::vector<int64_t> rp(row_ptr, row_ptr + n + 1);
        const int64_t e = rp[n];
        for (int64_t i = 0; i < e; ++i)
            RVX_REQUIRE(col[i] >= 0 && col[i] < n, RVX_ERR_INDEX, "column index out of range");
        auto g = std::make_unique<rvx_graph>();
        g->n = n;
        g->e = e;
        upload_csr(g.get(), rp, col, ew);
        *out = g.release();
    });
}

rvx_status rvx_graph_from_device_csr(int64_t n, int64_t e, rvx_buffer* rp, rvx_buffer* col, rvx_buffer* w,
                                     rvx_graph** out) {
    return guard([&] {
        RVX_REQUIRE(out && rp && col && n >= 0, RVX_ERR_INVALID_PARAMETER, "bad device CSR args");
        RVX_REQUIRE(rp->mem.bytes >= (n + 1) * 8 && col->mem.bytes >= e * 4, RVX_ERR_INVALID_PARAMETER,
                    "CSR buffers too small");
        auto g = std::make_unique<rvx_graph>();
        g->n = n;
        g->e = e;
        g->row_ptr = rp->mem.as<int64_t>();
        g->col = col->mem.as<int32_t>();
        if (w) {
            RVX_REQUIRE(w->mem.bytes >= e * 4, RVX_ERR_INVALID_PARAMETER, "weights too small");
            g->w = w->mem.as<float>();
            g->host_w.resize(e);
            w->mem.download(g->host_w.data(), e * 4);
        }
        std::vector<int64_t> h(n + 1);
        rp->mem.download(h.data(), (n + 1) * 8);
        RVX_REQUIRE(h[0] == 0 && h[n] == e, RVX_ERR_INVALID_PARAMETER, "row_ptr inconsistent with num_edges");
        finish_graph(g.get(), h);
        *out = g.release();
    });
}

rvx_status rvx_graph_info(const rvx_graph* g, int64_t* n, int64_t* e, int32_t* max_deg) {
    return guard([&] {
        check_graph(g);
        if (n) *n = g->n;
        if (e) *e = g->e;
        if (max_deg) *max_deg = g->max_deg;
    });
}

rvx_status rvx_graph_destroy(rvx_graph* g) {
    return guard([&] { delete g; });
}

rvx_status rvx_aggregate_device(const rvx_graph* g, int32_t agg, int32_t use_w, int32_t keep_isolated,
                                const rvx_buffer* x, int32_t dim, rvx_buffer* out) {
    return guard([&] {
        check_graph(g);
        RVX_REQUIRE(x && out && dim > 0, RVX_ERR_INVALID_PARAMETER, "null buffers");
        RVX_REQUIRE(x->mem.bytes >= g->n * dim * 4 && out->mem.bytes >= g->n * dim * 4, RVX_ERR_DIMENSION_MISMATCH,
                    "feature buffers smaller than n*dim");
        RVX_REQUIRE(!use_w || g->w, RVX_ERR_INVALID_PARAMETER, "graph has no edge weights");
        ComputeLock cl;
        aggregate_rows(g->row_ptr, g->col, use_w ? g->w : nullptr, g->n, x->mem.as<float>(), dim, agg,
                       keep_isolated ? 1 : 0, 0, out->mem.as<float>(), "aggregate");
    });
}

rvx_status rvx_sage_layer_create(int32_t in, int32_t out_f, int32_t num_samples, int32_t aggregator, int32_t normalize,
                                 const float* wn, const float* ws, rvx_sage_layer** out) {
    return guard([&] {
        RVX_REQUIRE(out && in > 0 && out_f > 0 && num_samples >= 0, RVX_ERR_LAYER_CONFIG, "bad GraphSAGE dims");
        RVX_REQUIRE(aggregator >= 0 && aggregator <= 2, RVX_ERR_LAYER_CONFIG, "unknown aggregator");
        RVX_REQUIRE((wn == nullptr) == (ws == nullptr), RVX_ERR_INVALID_PARAMETER, "give both weight matrices or none");
        auto l = std::make_unique<rvx_sage_layer>();
        l->in = in; l->out = out_f; l->num_samples = num_samples; l->aggregator = aggregator;
        l->normalize = normalize ? 1 : 0;
        if (wn) {
            l->wn.assign(wn, wn + (size_t)in * out_f);
            l->ws.assign(ws, ws + (size_t)in * out_f);
        } else {
            l->wn = det_init(in, out_f, 0);
            l->ws = det_init(in, out_f, 1000);
        }
        upload_transposed(l->wn_t, l->wn, in, out_f);
        upload_transposed(l->ws_t, l->ws, in, out_f);
        l->wn_x3.reset((int64_t)in * out_f * 6);
        l->ws_x3.reset((int64_t)in * out_f * 6);
        split_x3(l->wn_t.as<float>(), (int64_t)in * out_f, l->wn_x3.as<uint16_t>());
        split_x3(l->ws_t.as<float>(), (int64_t)in * out_f, l->ws_x3.as<uint16_t>());
        l->wn_h2.reset((int64_t)in * out_f * 4);
        l->ws_h2.reset((int64_t)in * out_f * 4);
        l->w_inv.reset((int64_t)out_f * 4);
        split_h2_rows(l->wn_t.as<float>(), l->ws_t.as<float>(), out_f, in, l->wn_h2.as<_Float16>(),
                      l->ws_h2.as<_Float16>(), l->w_inv.as<float>());
        sync();
        *out = l.release();
    });
}

rvx_status rvx_sage_sample_positions(int32_t len, int32_t k, int32_t* out) {
    return guard([&] {
        RVX_REQUIRE(out && k >= 0 && len > k, RVX_ERR_INVALID_PARAMETER, "need len > k >= 0");
        sage_sample_positions(len, k, out);
    });
}

rvx_status rvx_sage_layer_destroy(rvx_sage_layer* l) {
    return guard([&] { delete l; });
}

rvx_status rvx_sage_forward_device(const rvx_sage_layer* l, const rvx_graph* g, const rvx_buffer* x, rvx_buffer* y) {
    return guard([&] {
        check_graph(g);
        RVX_REQUIRE(l && x && y, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(x->mem.bytes >= g->n * l->in * 4, RVX_ERR_DIMENSION_MISMATCH, "x smaller than n*in");
        RVX_REQUIRE(y->mem.bytes >= g->n * l->out * 4, RVX_ERR_DIMENSION_MISMATCH, "y smaller than n*out");
        ComputeLock cl;
        sage_forward_dev(l, g, x->mem.as<float>(), y->mem.as<float>());
    });
}

rvx_status rvx_sage_forward_shard_device(const rvx_sage_layer* l, const rvx_graph* g, const rvx_buffer* x_full,
                                         int64_t row_offset, rvx_buffer* y) {
    return guard([&] {
        check_graph(g);
        RVX_REQUIRE(l && x_full && y && row_offset >= 0, RVX_ERR_INVALID_PARAMETER, "bad argument");
        RVX_REQUIRE(x_full->mem.bytes >= (row_offset + g->n) * l->in * 4, RVX_ERR_DIMENSION_MISMATCH,
                    "x_full does not cover the shard rows");
        RVX_REQUIRE(y->mem.bytes >= g->n * l->out * 4, RVX_ERR_DIMENSION_MISMATCH, "y smaller than rows*out");
        ComputeLock cl;
        sage_forward_dev(l, g, x_full->mem.as<float>(), y->mem.as<float>(), row_offset);
    });
}

rvx_status rvx_sage_forward_exchange(const rvx_sage_layer* l, const rvx_graph* g, const rvx_buffer* x_full,
                                     rvx_buffer* y_full, const int64_t* offsets, rvx_comm* comm, int32_t exchange) {
    // without x_rowmul the input is never rescaled
    return rvx_sage_forward_exchange2(l, g, const_cast<rvx_buffer*>(x_full), nullptr, y_full, nullptr, offsets, comm,
                                      exchange);
}

rvx_status rvx_sage_forward_exchange2(const rvx_sage_layer* l, const rvx_graph* g, rvx_buffer* x_full,
                                      const rvx_buffer* x_rowmul, rvx_buffer* y_full, rvx_buffer* y_rowinv,
                                      const int64_t* offsets, rvx_comm* comm, int32_t exchange) {
    return rvx_sage_forward_exchange3(l, g, x_full, x_rowmul, nullptr, y_full, y_rowinv, nullptr, offsets, comm,
                                      exchange);
}

rvx_status rvx_row_image_bytes(int64_t n, int32_t dim, int64_t* bytes) {
    return guard([&] {
        RVX_REQUIRE(bytes && n >= 0 && n < ((int64_t)1 << 40), RVX_ERR_INVALID_PARAMETER, "bad row-image arguments");
        RVX_REQUIRE(row_image_ok(dim), RVX_ERR_UNSUPPORTED, "row images need 512 < dim <= 768, dim % 4 == 0");
        *bytes = n * (IMG_SLOT + 2) + 16;  // slots, then the nnz array (u16 per row)
    });
}

namespace {
RowImage image_of(rvx_buffer* b, int64_t n, int dim, const char* what) {
    if (!b) return RowImage();
    RVX_REQUIRE(row_image_ok(dim), RVX_ERR_UNSUPPORTED, std::string(what) + ": row images need 512 < dim <= 768");
    RVX_REQUIRE(b->mem.bytes >= n * (IMG_SLOT + 2) + 16, RVX_ERR_DIMENSION_MISMATCH,
                std::string(what) + " smaller than rvx_row_image_bytes");
    RowImage im;
    im.slots = b->mem.as<unsigned char>();
    im.nnz = reinterpret_cast<uint16_t*>(im.slots + n * IMG_SLOT);
    return im;
}
RowImage image_rows(RowImage im, int64_t r0) {  // the same image seen from row r0 on
    if (im) { im.slots += r0 * IMG_SLOT; im.nnz += r0; }
    return im;
}
}  // namespace

rvx_status rvx_row_image_pack(const rvx_buffer* x, int64_t n_total, int64_t r0, int64_t rows, int32_t dim,
                              rvx_buffer* image) {
    return guard([&] {
        RVX_REQUIRE(x && image && r0 >= 0 && rows >= 0 && r0 + rows <= n_total, RVX_ERR_INVALID_PARAMETER,
                    "bad row-image pack arguments");
        RVX_REQUIRE(x->mem.bytes >= n_total * dim * 4, RVX_ERR_DIMENSION_MISMATCH, "x smaller than n_total*dim");
        const RowImage im = image_of(image, n_total, dim, "image");
        ComputeLock cl;
        rows_image_pack(x->mem.as<float>(), r0, rows, dim, im);
    });
}

namespace {
// Page-locked host words per device (the exchange's small device-to-host reads that the host
// picks up later without stalling the stream); callers hold the device's ComputeLock.
unsigned long long* pinned_words(int64_t n) {
    static std::mutex mu;
    static std::map<int, std::pair<unsigned long long*, int64_t>> held;
    std::lock_guard<std::mutex> lk(mu);
    auto& h = held[device().id];
    if (h.second < n) {
        if (h.first) RVX_HIP(hipHostFree(h.first));
        RVX_HIP(hipHostMalloc((void**)&h.first, (size_t)n * 8, 0));
        h.second = n;
    }
    return h.first;
}
// the broadcast buffer of the dense-row pass: cnt ids (int64), then their rows
float* ids_rows(int64_t* ids, int64_t cnt) { return reinterpret_cast<float*>(ids + cnt); }
}  // namespace

rvx_status rvx_sage_forward_exchange3(const rvx_sage_layer* l, const rvx_graph* g, rvx_buffer* x_full,
                                      const rvx_buffer* x_rowmul, rvx_buffer* x_image, rvx_buffer* y_full,
                                      rvx_buffer* y_rowinv, rvx_buffer* y_image, const int64_t* offsets,
                                      rvx_comm* comm, int32_t exchange) {
    return guard([&] {
        check_graph(g);
        RVX_REQUIRE(l && x_full && y_full && offsets, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(x_full != y_full, RVX_ERR_INVALID_PARAMETER, "x_full and y_full must be different buffers");
        const int world = comm_size(comm), me = comm_rank(comm);
        for (int p = 0; p < world; ++p)
            RVX_REQUIRE(offsets[p] >= 0 && offsets[p] <= offsets[p + 1], RVX_ERR_INVALID_PARAMETER,
                        "offsets must be non-decreasing");
        RVX_REQUIRE(offsets[me + 1] - offsets[me] == g->n, RVX_ERR_DIMENSION_MISMATCH,
                    "graph rows differ from this rank's shard");
        const int64_t N = offsets[world];
        RVX_REQUIRE(x_full->mem.bytes >= N * l->in * 4, RVX_ERR_DIMENSION_MISMATCH, "x_full smaller than N*in");
        RVX_REQUIRE(y_full->mem.bytes >= N * l->out * 4, RVX_ERR_DIMENSION_MISMATCH, "y_full smaller than N*out");
        RVX_REQUIRE(!x_rowmul || x_rowmul->mem.bytes >= N * 4, RVX_ERR_DIMENSION_MISMATCH, "x_rowmul smaller than N");
        RVX_REQUIRE(!y_rowinv || y_rowinv->mem.bytes >= N * 4, RVX_ERR_DIMENSION_MISMATCH, "y_rowinv smaller than N");
        RVX_REQUIRE(!x_image || x_image != y_image, RVX_ERR_INVALID_PARAMETER, "x_image and y_image must differ");
        const RowImage ximg = image_of(x_image, N, l->in, "x_image");
        const RowImage yimg = image_of(y_image, N, l->out, "y_image");
        ComputeLock cl;
        float* y = y_full->mem.as<float>();
        const float* x = x_full->mem.as<float>();
        // deferred normalisation where this layer's GEMM path takes it; otherwise the
        // multiplied input is materialised in place and the output normalised as usual
        // (then every 1/|y| is 1)
        const bool can = sage_defer_path(l, g->n, x, y + offsets[me] * l->out, offsets[me]);
        const float* xm = x_rowmul ? x_rowmul->mem.as<float>() : nullptr;
        if (xm && !can) {
            const int64_t tot = N * l->in;
            RVX_LAUNCH("scale_rows", k_scale_rows, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                       x_full->mem.as<float>(), N, l->in, xm);
            xm = nullptr;
        }
        // `can` is this rank's own decision (its GEMM path and alignment). Whenever the
        // caller passed y_rowinv, every rank exchanges it: a rank that normalises in place
        // ships 1.0 for its rows, so the ranks' collective sequences stay identical
        // whatever each one decided.
        float* yinv_xchg = y_rowinv ? y_rowinv->mem.as<float>() : nullptr;
        float* yinv = yinv_xchg;
        if (yinv && !can) {
            fill_value(yinv, N, 1.0f);
            yinv = nullptr;
        }
        float* yinv_rows = yinv ? yinv + offsets[me] : nullptr;
        // (x_image describes x as the caller passed it: a rescale in place above would stale it)
        const RowImage xi = xm || !x_rowmul ? ximg : RowImage();
        if (!exchange || (world == 1 && !comm_self_p2p(comm))) {
            sage_forward_dev(l, g, x, y + offsets[me] * l->out, offsets[me], 0, nullptr, xm, yinv_rows, xi,
                             image_rows(yimg, offsets[me]));
            return;
        }
        const std::vector<ExchangeRound> plan = exchange_plan(PLAN_SAGE, offsets, world);
        const int chunks = (int)plan.size();
        Device& d = device();
        hipEvent_t* ev = pipeline_events(SAGE_PIPE_EVENTS(chunks) + chunks + 1) + SAGE_PIPE_EVENTS(chunks);  // after sage_forward_dev's
        // Compact records (kernels.hpp rows_xchg_pack): a layer's output rows are ReLU-sparse
        // (graphsage.rs:172-176), so a round's rows travel as their image records — bitmap + the
        // values other than +0.0 — back to back, with a u32 count per row, and are expanded
        // back into the dense rows bit for bit on arrival. RCCL p2p needs both sides to know a
        // message's size, with no host wait per round: each rank's round block gets a byte
        // budget of rows x (bytes per row), the rate agreed once per call from chunk 0 (every
        // rank's mean record bytes over its chunk-0 rows, all-gathered, the largest + 2% +
        // 16 B; one host wait, at the first round). Records sit at the prefix sums of their
        // sizes, which the receiver recomputes from the counts; rows whose record ends past
        // the budget (or holds more than IMG_CAP values) travel dense after the rounds (counts
        // all-gathered, then each owner's broadcast). Where records would save less than 15%
        // of a dense row the call exchanges dense rows. At 768 dims with about half the values
        // +0.0: ~1,700 + 4 B per 3,072-B row. RVX_XCHG_IMAGE=0 exchanges dense rows;
        // RVX_XCHG_ROW_BYTES fixes the rate (tests force overflows). Every rank decides alike.
        const bool xallow = row_image_ok(l->out) && env_int("RVX_XCHG_IMAGE", 1) != 0 && ((uintptr_t)y & 15) == 0;
        const int rate_env = env_int("RVX_XCHG_ROW_BYTES", 0);
        double rate = 0.0;  // budget bytes per row, decided in round 0
        bool xrec = false;
        int64_t round_rows = 0;  // staging rows per rank and round (the largest block of any round)
        for (const ExchangeRound& r : plan)
            for (int p = 0; p < world; ++p) round_rows = std::max(round_rows, r.rows[p]);
        unsigned char* xs = nullptr;
        uint32_t* xcnt = nullptr;
        uint64_t* xoff = nullptr;
        int64_t* ovf_ids = nullptr;
        // [0] own overflow rows, [1 .. world] all-gathered; [world + 1], [world + 2] own chunk-0
        // record bytes and rows, [world + 3 ..] all-gathered pairs
        unsigned long long* ctr = nullptr;
        void* scan_tmp = nullptr;
        size_t scan_bytes = 0;
        std::vector<int64_t> st(world), st16(world), blk16(world);  // staging: rank p's block at p * round_rows
        for (int p = 0; p < world; ++p) {
            st[p] = p * round_rows;
            st16[p] = p * round_rows * (IMG_SLOT / 16);
        }
        if (xallow) {  // (every scratch slot taken before the pipeline queues work that could use it)
            xs = (unsigned char*)scratch_bytes("sage_xchg_rec", (int64_t)world * round_rows * IMG_SLOT);
            xcnt = (uint32_t*)scratch_bytes("sage_xchg_cnt", (int64_t)world * round_rows * 4);
            xoff = (uint64_t*)scratch_bytes("sage_xchg_off", (int64_t)world * round_rows * 8);
            ovf_ids = (int64_t*)scratch_bytes("sage_xchg_ovf_ids", std::max<int64_t>(g->n, 1) * 8);
            ctr = (unsigned long long*)scratch_bytes("sage_xchg_ctr", 8 * (3 * world + 3));
            scan_bytes = rec_offsets_temp_bytes(round_rows);
            scan_tmp = scratch_bytes("sage_xchg_scan", (int64_t)std::max<size_t>(scan_bytes, 16));
            RVX_HIP(hipMemsetAsync(ctr, 0, 8 * (size_t)(3 * world + 3), d.xfer));
        }
        // one-rank RCCL (RVX_COMM_SELF_P2P): the rank's own records come back through RCCL and
        // are expanded into this shadow by the receivers' unpack kernel, then compared with the
        // rows they encode (comm_selfcheck_rows) — the record path's receive side runs behind a
        // real RCCL transfer on a one-GPU box
        float* shadow = xallow && comm_self_p2p(comm) ? scratch_f32("sage_xchg_shadow", round_rows * l->out) : nullptr;
        auto budget = [&](int64_t rows) { return ((uint64_t)std::ceil((double)rows * rate) + 15) / 16 * 16; };
        // the all-gathered chunk-0 record bytes land in pinned host memory; with more than one
        // round the host reads them at round 1 (chunk 1 already queued), so the GPU never idles
        // on this wait, and round 0's exchange goes out then
        RVX_REQUIRE(!xallow || world <= 1024, RVX_ERR_INVALID_PARAMETER, "compact exchange: at most 1024 ranks");
        unsigned long long* pinned = xallow && rate_env <= 0 ? pinned_words(2 * 1024) : nullptr;
        bool rate_pending = false;
        auto settle_rate = [&]() {  // xfer holds the chunk-0 count, its all-gather and the copy
            RVX_HIP(hipStreamSynchronize(d.xfer));
            for (int p = 0; p < world; ++p)
                if (pinned[2 * p + 1] > 0) rate = std::max(rate, (double)pinned[2 * p] / (double)pinned[2 * p + 1]);
            rate = rate * 1.02 + 16.0;
            xrec = rate + 4.0 <= 0.85 * 4.0 * l->out;
            rate_pending = false;
        };
        auto round = [&](int c, bool counted) {  // round c's exchange on the transfer stream (ev[c] waited)
            const std::vector<int64_t>& rows = plan[c].rows;
            if (xrec) {
                if (!counted) rows_rec_count(y, plan[c].r0[me], rows[me], l->out, xcnt + st[me], nullptr);
                rec_offsets(xcnt + st[me], rows[me], xoff + st[me], scan_tmp, scan_bytes);
                rows_xchg_pack(y, plan[c].r0[me], rows[me], l->out, xs + st16[me] * 16, budget(rows[me]), xcnt + st[me],
                               xoff + st[me], ovf_ids, ctr);
                for (int p = 0; p < world; ++p) blk16[p] = (int64_t)(budget(rows[p]) / 16);
                comm_exchange_rows(comm, reinterpret_cast<float*>(xcnt), 1, st.data(), rows.data(), d.xfer);
                comm_exchange_rows(comm, reinterpret_cast<float*>(xs), 4, st16.data(), blk16.data(), d.xfer);
            } else {
                comm_exchange_rows(comm, y, l->out, plan[c].r0.data(), rows.data(), d.xfer);
            }
            if (yinv_xchg) comm_exchange_rows(comm, yinv_xchg, 1, plan[c].r0.data(), rows.data(), d.xfer);
            for (int p = 0; p < world; ++p) {
                if (p == me) {
                    if (xrec && shadow && rows[p] > 0) {
                        const float* own = y + plan[c].r0[p] * l->out;
                        RVX_HIP(hipMemcpyAsync(shadow, own, (size_t)(rows[p] * l->out * 4), hipMemcpyDeviceToDevice,
                                               d.xfer));  // rows past the budget stay as they are
                        rec_offsets(xcnt + st[p], rows[p], xoff + st[p], scan_tmp, scan_bytes);
                        rows_xchg_unpack(shadow, 0, rows[p], l->out, xs + st16[p] * 16, budget(rows[p]), xcnt + st[p],
                                         xoff + st[p], RowImage());
                        comm_selfcheck_rows(comm, shadow, own, rows[p], l->out, d.xfer);
                    }
                    continue;
                }
                if (xrec) {  // records back into dense rows (and the image, when asked for)
                    rec_offsets(xcnt + st[p], rows[p], xoff + st[p], scan_tmp, scan_bytes);
                    rows_xchg_unpack(y, plan[c].r0[p], rows[p], l->out, xs + st16[p] * 16, budget(rows[p]),
                                     xcnt + st[p], xoff + st[p], yimg);
                } else if (yimg) {  // the rows that arrived, imaged where they land (this rank's own: sage_forward_dev)
                    rows_image_pack(y, plan[c].r0[p], rows[p], l->out, yimg);
                }
            }
        };
        auto hook = [&](int c, int64_t, int64_t) {
            RVX_HIP(hipEventRecord(ev[c], stream()));  // chunk c's rows are complete on the pipeline's main stream
            StreamScope on_xfer(d.xfer);
            ProfScope ps("halo_exchange");
            if (rate_pending) {  // round 1: chunk 0's rate is on its way; round 0 goes out first
                settle_rate();
                round(0, true);
            }
            RVX_HIP(hipStreamWaitEvent(d.xfer, ev[c], 0));
            if (c == 0 && xallow) {
                if (rate_env > 0) {
                    rate = rate_env;
                    xrec = rate + 4.0 <= 0.85 * 4.0 * l->out;
                } else {
                    unsigned long long* acc = ctr + world + 1;
                    rows_rec_count(y, plan[0].r0[me], plan[0].rows[me], l->out, xcnt + st[me], acc);
                    comm_allgather_bytes(comm, acc, acc + 2, 16, d.xfer);
                    RVX_HIP(hipMemcpyAsync(pinned, acc + 2, 2 * 8 * (size_t)world, hipMemcpyDeviceToHost, d.xfer));
                    rate_pending = true;
                    if (chunks > 1) return;  // round 0 leaves with round 1
                    settle_rate();
                    round(0, true);
                    return;
                }
            }
            round(c, false);
        };
        sage_forward_dev(l, g, x, y + offsets[me] * l->out, offsets[me], chunks, hook, xm, yinv_rows, xi,
                         image_rows(yimg, offsets[me]));
        if (xrec) {
            // rows past the slot: counts all-gathered, then each owner broadcasts its rows (ids
            // + dense values) and the others scatter them. A host wait per layer, at its end.
            StreamScope on_xfer(d.xfer);
            ProfScope ps("halo_exchange_dense_rows");
            auto* cnt_d = reinterpret_cast<int64_t*>(ctr) + 1;
            comm_allgather_bytes(comm, ctr, cnt_d, 8, d.xfer);
            std::vector<int64_t> cnt(world, 0);
            RVX_HIP(hipMemcpyAsync(cnt.data(), cnt_d, (size_t)world * 8, hipMemcpyDeviceToHost, d.xfer));
            RVX_HIP(hipStreamSynchronize(d.xfer));
            int64_t tot = 0, most = 0;
            for (int p = 0; p < world; ++p) {
                tot += cnt[p];
                most = std::max(most, cnt[p]);
            }
            if (tot > 0) {
                RVX_HIP(hipStreamSynchronize(d.stream));  // nothing of this layer may still use scratch
                DevMem buf(most * (8 + (int64_t)l->out * 4));
                auto* ids = buf.as<int64_t>();
                for (int p = 0; p < world; ++p) {
                    if (cnt[p] == 0) continue;
                    const int64_t bytes = cnt[p] * (8 + (int64_t)l->out * 4);
                    if (p == me) {  // ids first, then their rows, contiguous for the broadcast
                        RVX_HIP(hipMemcpyAsync(ids, ovf_ids, (size_t)cnt[p] * 8, hipMemcpyDeviceToDevice, d.xfer));
                        rows_by_id(y, l->out, ids, cnt[p], ids_rows(ids, cnt[p]), false);
                    }
                    comm_broadcast_bytes(comm, buf.p, bytes, p, d.xfer);
                    if (p != me) {
                        rows_by_id(y, l->out, ids, cnt[p], ids_rows(ids, cnt[p]), true);
                        if (yimg) rows_image_pack_ids(y, ids, cnt[p], l->out, yimg);
                    }
                }
                RVX_HIP(hipStreamSynchronize(d.xfer));  // buf is freed on return
            }
        }
        RVX_HIP(hipEventRecord(ev[chunks], d.xfer));
        {
            // the exchange's tail the compute stream waits for: from the last chunk's
            // compute to the last round's arrival (what the overlap did not hide)
            ProfScope ps("exchange_wait");
            RVX_HIP(hipStreamWaitEvent(d.stream, ev[chunks], 0));
        }
    });
}

rvx_status rvx_sage_forward(const rvx_sage_layer* l, const rvx_graph* g, const float* x, int64_t n, float* y) {
    return guard([&] {
        check_graph(g);
        RVX_REQUIRE(l && x && y, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(n == g->n, RVX_ERR_DIMENSION_MISMATCH, "feature rows != graph nodes");
        ComputeLock cl;
        float* dx = scratch_f32("sage_x", n * (int64_t)l->in);
        float* dy = scratch_f32("sage_y", n * (int64_t)l->out);
        RVX_HIP(hipMemcpyAsync(dx, x, (size_t)(n * l->in * 4), hipMemcpyHostToDevice, stream()));
        sage_forward_dev(l, g, dx, dy);
        RVX_HIP(hipMemcpyAsync(y, dy, (size_t)(n * l->out * 4), hipMemcpyDeviceToHost, stream()));
        sync();
    });
}

rvx_status rvx_gcn_layer_create(int32_t in, int32_t out_f, int32_t normalize, const float* w, const float* b,
                                rvx_gcn_layer** out) {
    return guard([&] {
        RVX_REQUIRE(out && in > 0 && out_f > 0, RVX_ERR_LAYER_CONFIG, "bad GCN dims");
        auto l = std::make_unique<rvx_gcn_layer>();
        l->in = in; l->out = out_f; l->normalize = normalize ? 1 : 0;
        l->w = w ? std::vector<float>(w, w + (size_t)in * out_f) : det_init(in, out_f, 0);
        l->b = b ? std::vector<float>(b, b + out_f) : std::vector<float>(out_f, 0.0f);
        upload_transposed(l->w_t, l->w, in, out_f);
        l->bias.reset(out_f * 4);
        l->bias.upload(l->b.data(), out_f * 4);
        *out = l.release();
    });
}

rvx_status rvx_gcn_layer_destroy(rvx_gcn_layer* l) {
    return guard([&] { delete l; });
}

rvx_status rvx_gcn_forward(const rvx_gcn_layer* l, const rvx_graph* g, int32_t use_w, const float* x, int64_t n,
                           float* y) {
    return guard([&] {
        check_graph(g);
        RVX_REQUIRE(l && x && y, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(n == g->n, RVX_ERR_DIMENSION_MISMATCH, "feature rows != graph nodes");
        RVX_REQUIRE(!use_w || g->w, RVX_ERR_INVALID_PARAMETER, "graph has no edge weights");
        ComputeLock cl;
        float* dx = scratch_f32("gcn_x", n * (int64_t)l->in);
        float* dy = scratch_f32("gcn_y", n * (int64_t)l->out);
        RVX_HIP(hipMemcpyAsync(dx, x, (size_t)(n * l->in * 4), hipMemcpyHostToDevice, stream()));
        gcn_forward_dev(l, g, use_w != 0, dx, dy);
        RVX_HIP(hipMemcpyAsync(y, dy, (size_t)(n * l->out * 4), hipMemcpyDeviceToHost, stream()));
        sync();
    });
}

rvx_status rvx_exchange_plan(int32_t kind, const int64_t* offsets, int32_t world, int32_t* n_rounds, int64_t* r0,
                             int64_t* rows) {
    return guard([&] {
        RVX_REQUIRE(offsets && n_rounds && world > 0 && (kind == PLAN_SAGE || kind == PLAN_WHOLE),
                    RVX_ERR_INVALID_PARAMETER, "bad plan arguments");
        for (int p = 0; p < world; ++p)
            RVX_REQUIRE(offsets[p] >= 0 && offsets[p] <= offsets[p + 1], RVX_ERR_INVALID_PARAMETER,
                        "offsets must be non-decreasing");
        const std::vector<ExchangeRound> plan = exchange_plan(kind, offsets, world);
        *n_rounds = (int32_t)plan.size();
        if (!r0) return;
        RVX_REQUIRE(rows, RVX_ERR_INVALID_PARAMETER, "null rows");
        for (size_t c = 0; c < plan.size(); ++c)
            for (int p = 0; p < world; ++p) {
                r0[c * world + p] = plan[c].r0[p];
                rows[c * world + p] = plan[c].rows[p];
            }
    });
}

}  // extern "C"
