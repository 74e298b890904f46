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
// An RCCL communicator of one rank with RVX_COMM_SELF_P2P=1: the exchange and search
// drivers still run their collectives (to the rank itself) instead of skipping them.
bool comm_self_p2p(const rvx_comm* c);

// RVX_COMM_SELF_P2P record check: the rank's own compact records, after their round trip
// through RCCL, expanded into `shadow` (rows_xchg_unpack, the receivers' kernel), compared word
// for word with the rows they came from (`rows` rows of `dim` floats) on stream `s`; mismatches
// accumulate in the communicator (rvx_comm_selfcheck).
void comm_selfcheck_rows(rvx_comm* c, const float* shadow, const float* rows, int64_t nrows, int dim, hipStream_t s);

// One grouped point-to-point round on stream `s`: this rank sends its rows
// [r0[me], r0[me]+rows[me]) of `table` to every peer and receives each peer
// p's rows [r0[p], r0[p]+rows[p]) into the same rows of its own `table`
// (row = row_elems floats). On xGMI every pair has its own link, so the
// round moves all peers' chunks concurrently.
void comm_exchange_rows(rvx_comm* c, float* table, int64_t row_elems, const int64_t* r0, const int64_t* rows,
                        hipStream_t s);

// Sharded search collectives (SURVEY.md §8e option 2, shard.rs:354-373), on stream `s`,
// over RCCL or the host-staged transport:
// broadcast `bytes` of device memory `buf` from rank `root` to every rank (in place);
void comm_broadcast_bytes(rvx_comm* c, void* buf, int64_t bytes, int root, hipStream_t s);
// all-gather: every rank's `bytes` at `send` into recv [nranks][bytes] (rank-major).
void comm_allgather_bytes(rvx_comm* c, const void* send, void* recv, int64_t bytes, hipStream_t s);

// ShardedHyperbolicHnsw::search merge (shard.rs:354-373) across ranks: this rank's
// per-query hits gid/lid/dist [nq][k] (ascending; an empty slot has gid -1 and
// +inf) are all-gathered and every rank merges all ranks' lists by distance,
// ties in rank order then list order (for node-range shards: by global id), and
// keeps the first k: out_gid/out_lid/out_dist [nq][k], out_count [nq] (nullable:
// out_lid, out_count). Device pointers, library stream; lid may be null (zeros).
void sharded_merge(rvx_comm* c, const int64_t* gid, const int64_t* lid, const float* dist, int64_t nq, int k,
                   int64_t* out_gid, int64_t* out_lid, float* out_dist, int32_t* out_count);

// Collective precondition check of a sharded search, before any other collective: every
// rank passes its local verdict (status, message) and its {nq, k, ef, mode, dim}; a fixed-
// size all-gather lets every rank see every verdict, and all ranks throw the same way when
// any rank failed or the arguments differ — no rank is left waiting in a collective.
void shard_agree(rvx_comm* c, rvx_status status, const std::string& why, const int64_t (&args)[5]);

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
