// graph.hpp — the HBM-resident CSR graph handle and a per-device scratch pool.
#pragma once
#include <map>
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
};

namespace rvx {

// Scratch buffers reused across calls on one device; callers hold the device
// lock (ComputeLock) for the duration of the op that uses them.
float* scratch_f32(const std::string& slot, int64_t count);
void* scratch_bytes(const std::string& slot, int64_t bytes);

// Serialises compute entry points per device (they share scratch and stream).
struct ComputeLock {
    std::unique_lock<std::recursive_mutex> lk;
    ComputeLock();
};

void check_graph(const rvx_graph* g);

}  // namespace rvx
