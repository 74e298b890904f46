// comm.hpp — internal RCCL helpers shared by the layer drivers.
#pragma once
#include <functional>
#include <utility>
#include <vector>

#include "common.hpp"

struct rvx_comm;

namespace rvx {

int comm_rank(const rvx_comm* c);
int comm_size(const rvx_comm* c);

// One grouped point-to-point round on stream `s`: this rank sends its rows
// [r0[me], r0[me]+rows[me]) of `table` to every peer and receives each peer
// p's rows [r0[p], r0[p]+rows[p]) into the same rows of its own `table`
// (row = row_elems floats). On xGMI every pair has its own link, so the
// round moves all peers' chunks concurrently.
void comm_exchange_rows(rvx_comm* c, float* table, int64_t row_elems, const int64_t* r0, const int64_t* rows,
                        hipStream_t s);

// Exchange round plan (rvx_exchange_plan): plan[c] = {r0[p], rows[p]} of round c.
enum { PLAN_SAGE = 0, PLAN_WHOLE = 1 };
struct ExchangeRound {
    std::vector<int64_t> r0, rows;
};
std::vector<ExchangeRound> exchange_plan(int kind, const int64_t* offsets, int world);
// Row chunks of a GraphSAGE layer pipeline over n rows (same on every rank).
int sage_chunks_for(int64_t n);
int64_t chunk_step(int64_t n, int chunks);

// Produce-then-exchange in row chunks (SURVEY.md §8e "chunked all-gather
// pipelined with compute"): for each round c of exchange_plan(PLAN_SAGE),
// produce(r0, rows) queues this rank's rows [r0, r0 + rows) (global ids, may be
// empty) of every table on the library stream; the round's rows of every
// (table, row_elems) then move to and from every peer on the transfer stream
// while round c+1 computes. Returns with the library stream ordered after the
// last round. World 1: one produce over the rank's rows, no exchange.
using TableRef = std::pair<float*, int64_t>;
void produce_and_exchange(rvx_comm* comm, const int64_t* offsets, const std::vector<TableRef>& tables,
                          const std::function<void(int64_t r0, int64_t rows)>& produce);

}  // namespace rvx
