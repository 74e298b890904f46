// graph.hpp — the HBM-resident CSR graph handle and a per-device scratch pool.
#pragma once
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "common.hpp"

// CSR by destination: row i lists the sources j of edges (j -> i) in edge order,
// exactly build_adjacency_list's adj[dst].push(src)
// (crates/ruvector-postgres/src/gnn/message_passing.rs:34-50).
struct rvx_graph {
    int64_t n = 0, e = 0;
    int32_t max_deg = 0;
    rvx::DevMem row_ptr_mem, col_mem, w_mem, isolated_mem;  // owned storage (may be empty)
    const int64_t* row_ptr = nullptr;                       // device [n+1]
    const int32_t* col = nullptr;                           // device [e]
    const float* w = nullptr;                               // device [e] or null
    const int32_t* isolated = nullptr;                      // device list of rows with no neighbours
    int64_t n_isolated = 0;
    std::vector<float> host_w;                              // host copy of weights (RuvectorLayer sums)
    // GraphSAGE sampled CSRs by num_samples (k_sample.hip), built on first use
    mutable std::mutex sampled_mu;
    mutable std::map<int32_t, std::unique_ptr<rvx_graph>> sampled;
};

namespace rvx {

// Scratch buffers reused across calls on one device; callers hold the device
// lock (ComputeLock) for the duration of the op that uses them.
float* scratch_f32(const std::string& slot, int64_t count);
void* scratch_bytes(const std::string& slot, int64_t bytes);
// Frees every scratch slot of the calling thread's device (after a device sync).
void scratch_release_all();
// Bytes the slot holds now (0 if never used).
int64_t scratch_held(const std::string& slot);

// Serialises compute entry points per device (they share scratch and stream).
struct ComputeLock {
    std::unique_lock<std::recursive_mutex> lk;
    ComputeLock();
};

void check_graph(const rvx_graph* g);

// GraphSAGE neighbour sampling (k_sample.hip): the graph itself when no row
// has more than k neighbours, else its cached sampled CSR.
const rvx_graph* sampled_graph(const rvx_graph* g, int32_t k);
// Positions sample_neighbors keeps from a list of `len` > k (graphsage.rs:92-102).
void sage_sample_positions(int32_t len, int32_t k, int32_t* out);

}  // namespace rvx
