/*
 * rvx.h — C ABI of the MI355X-native GNN-learned-index engine (librvx.so).
 *
 * This is the drop-in boundary for ruvector's hot path. Every entry point
 * names the reference interface it replaces (paths relative to the
 * Mu-L/ruvector checkout). Conventions:
 *   - every function returns rvx_status (0 = RVX_OK); the status codes map
 *     1:1 onto the reference error enums RuvectorError
 *     (crates/ruvector-core/src/error.rs:8-60) and GnnError
 *     (crates/ruvector-gnn/src/error.rs:12-55);
 *   - rvx_last_error() returns the thread-local message of the last failure;
 *   - inputs are caller-owned host pointers that the library copies on entry
 *     (the `_device` / rvx_buffer variants take device-resident data instead);
 *   - the library owns every handle it returns; handles are freed with the
 *     matching *_destroy / *_free;
 *   - search calls on one handle may run concurrently from several threads;
 *     add/load calls need external exclusion (mirrors VectorDB's RwLock,
 *     crates/ruvector-core/src/vector_db.rs:22-26).
 * No torch, CUDA or compatibility types appear in these signatures.
 */
#ifndef RVX_RVX_H
#define RVX_RVX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t rvx_status;

enum {
    RVX_OK = 0,
    RVX_ERR_DIMENSION_MISMATCH = 1, /* RuvectorError::DimensionMismatch / GnnError::DimensionMismatch */
    RVX_ERR_INVALID_PARAMETER = 2,  /* RuvectorError::InvalidParameter */
    RVX_ERR_INDEX = 3,              /* RuvectorError::IndexError */
    RVX_ERR_LAYER_CONFIG = 4,       /* GnnError::LayerConfig (layer.rs:100-106, :353-358) */
    RVX_ERR_INVALID_SHAPE = 5,      /* GnnError::InvalidShape */
    RVX_ERR_DEVICE = 6,             /* HIP runtime failure (no reference analogue) */
    RVX_ERR_OUT_OF_MEMORY = 7,
    RVX_ERR_UNSUPPORTED = 8,
    RVX_ERR_SERIALIZATION = 9,      /* serde / bincode errors */
    RVX_ERR_COMM = 10,              /* RCCL failure */
    RVX_ERR_NOT_FOUND = 11          /* RuvectorError::VectorNotFound */
};

/* Distance metrics: crates/ruvector-core/src/types.rs:10-20 (DistanceMetric),
 * plus the Poincaré ball distance of crates/ruvector-hyperbolic-hnsw/src/poincare.rs:227-255. */
enum {
    RVX_METRIC_L2 = 0,        /* Euclidean  -> distance.rs:27-43  */
    RVX_METRIC_COSINE = 1,    /* Cosine     -> distance.rs:47-64  */
    RVX_METRIC_DOT = 2,       /* DotProduct -> distance.rs:68-80  */
    RVX_METRIC_L1 = 3,        /* Manhattan  -> distance.rs:84-86  */
    RVX_METRIC_POINCARE = 4,  /* poincare_distance (curvature c)  */
    RVX_METRIC_HYP_L2 = 5     /* HyperbolicHnsw DistanceMetric::Euclidean: sqrt of fused_norms'
                                 chunked |a-b|^2 (ruvector-hyperbolic-hnsw hnsw.rs:182-185) */
};

/* ------------------------------------------------------------------ */
/* Library / device                                                    */
/* ------------------------------------------------------------------ */
int32_t rvx_last_error(char* buf, size_t len);     /* copies message; returns its length */
const char* rvx_version(void);
rvx_status rvx_device_count(int32_t* count);
/* Select the HIP device used by the calling thread's library calls (default 0). */
rvx_status rvx_set_device(int32_t device);
rvx_status rvx_get_device(int32_t* device);
/* Wait for all work the library queued on the current device. */
rvx_status rvx_synchronize(void);
/* Free the per-device scratch pool (pipeline chunk buffers, scan images, ...) that compute
 * calls keep for reuse; the next call re-allocates what it needs. */
rvx_status rvx_scratch_release(void);
/* Device properties: CU count, HBM bytes, arch name (e.g. "gfx950"). */
rvx_status rvx_device_info(int32_t* num_cus, int64_t* hbm_bytes, char* arch, size_t arch_len);

/* ------------------------------------------------------------------ */
/* Device buffers (HBM-resident tensors; row-major, 256-B aligned)     */
/* ------------------------------------------------------------------ */
typedef struct rvx_buffer rvx_buffer;
rvx_status rvx_buffer_alloc(int64_t bytes, rvx_buffer** out);
rvx_status rvx_buffer_free(rvx_buffer* buf);
int64_t    rvx_buffer_bytes(const rvx_buffer* buf);
void*      rvx_buffer_device_ptr(rvx_buffer* buf);
rvx_status rvx_buffer_upload(rvx_buffer* buf, const void* src, int64_t bytes, int64_t offset);
rvx_status rvx_buffer_download(const rvx_buffer* buf, void* dst, int64_t bytes, int64_t offset);
rvx_status rvx_buffer_zero(rvx_buffer* buf);
/* Position-keyed 64-bit checksum of bytes [offset, offset + bytes) of a buffer (integer
 * arithmetic, launch-independent): multi-rank runs compare the exchanged node tables of
 * every rank with it. Not part of the reference API. */
rvx_status rvx_buffer_checksum(const rvx_buffer* buf, int64_t offset, int64_t bytes, uint64_t* out);
/* Rows ids[0..n) of a [rows][dim] f32 table to host out [n][dim] (one device gather per
 * 256 MB; parity checks and stored-row export). Errors: IndexError for an id outside [0, rows). */
rvx_status rvx_buffer_gather_rows_f32(const rvx_buffer* table, int64_t rows, int32_t dim, const int64_t* ids,
                                     int64_t n, float* out);

/* Synthetic data generators (device side; the integer stream is shared with
 * oracle/oracle.cpp so the CPU baseline sees identical inputs).
 * uniform:  x_i = lo + (hi-lo) * u_i,  u_i = (h(seed,i) >> 40) * 2^-24
 * normal:   Box–Muller on two uniforms (ruvector-bench DatasetGenerator,
 *           crates/ruvector-bench/src/lib.rs:112-114)
 * random_csr: out-degree `deg` per node, col = h(seed, i*deg+t) mod N. */
rvx_status rvx_fill_uniform(rvx_buffer* buf, int64_t n_floats, uint64_t seed, float lo, float hi);
/* Elements [first, first+n_floats) of the rvx_fill_uniform(seed) stream (counter-based),
 * so a node-range shard generates exactly its slice of the global edge weights. */
rvx_status rvx_fill_uniform_at(rvx_buffer* buf, int64_t n_floats, uint64_t seed, int64_t first, float lo, float hi);
rvx_status rvx_fill_normal(rvx_buffer* buf, int64_t n_floats, uint64_t seed);
/* C5 corpus rows [first_row, first_row + rows) (direction ~ N(0,1)
 * normalised, radius rmax * U[0,1)), row-deterministic so node-range shards generate
 * their rows of the single-GPU corpus: buf [rows][dim]. */
rvx_status rvx_fill_ball_rows(rvx_buffer* buf, int64_t rows, int32_t dim, uint64_t seed, int64_t first_row,
                              float rmax);
rvx_status rvx_normalize_rows(rvx_buffer* buf, int64_t rows, int32_t dim); /* L2, as hnsw_integration_test.rs:21-28 */
rvx_status rvx_random_csr(int64_t n, int32_t deg, uint64_t seed, rvx_buffer* row_ptr_i64, rvx_buffer* col_i32);
/* Rows [row_begin, row_begin+n_rows) of the same n_total-node random CSR
 * (local row_ptr, global column ids): one node-range shard. */
rvx_status rvx_random_csr_shard(int64_t n_total, int64_t row_begin, int64_t n_rows, int32_t deg, uint64_t seed,
                                rvx_buffer* row_ptr_i64, rvx_buffer* col_i32);

/* ------------------------------------------------------------------ */
/* Graph (CSR by destination, neighbours in edge order)                */
/* Replaces build_adjacency_list (crates/ruvector-postgres/src/gnn/     */
/* message_passing.rs:34-50): adj[dst].push(src) in edge order, edges   */
/* with an out-of-range endpoint dropped.                              */
/* ------------------------------------------------------------------ */
typedef struct rvx_graph rvx_graph;
/* From (src,dst) edge pairs, optional per-edge weights (nullable). */
rvx_status rvx_graph_from_edges(int64_t num_nodes, const int64_t* src, const int64_t* dst,
                                int64_t num_edges, const float* edge_weights, rvx_graph** out);
/* From a host CSR: row_ptr[n+1] (int64), col[E] (int32), weights[E] nullable. */
rvx_status rvx_graph_from_csr(int64_t num_nodes, const int64_t* row_ptr, const int32_t* col,
                              const float* edge_weights, rvx_graph** out);
/* Adopt device-resident CSR buffers (copied by reference; caller keeps them alive). */
rvx_status rvx_graph_from_device_csr(int64_t num_nodes, int64_t num_edges, rvx_buffer* row_ptr_i64,
                                     rvx_buffer* col_i32, rvx_buffer* weights_f32 /*nullable*/,
                                     rvx_graph** out);
rvx_status rvx_graph_info(const rvx_graph* g, int64_t* num_nodes, int64_t* num_edges, int32_t* max_degree);
rvx_status rvx_graph_destroy(rvx_graph* g);

/* ------------------------------------------------------------------ */
/* Message passing aggregators (aggregators.rs:35-92)                  */
/* ------------------------------------------------------------------ */
enum { RVX_AGG_SUM = 0, RVX_AGG_MEAN = 1, RVX_AGG_MAX = 2 };
/* out[i] = agg_{j in adj(i)} (w_ij * x_j) over device buffers. Rows with no
 * neighbours get zeros (sum/mean) or -inf (max) unless `keep_isolated`,
 * in which case they get x_i (propagate, message_passing.rs:75-78). */
rvx_status rvx_aggregate_device(const rvx_graph* g, int32_t agg, int32_t use_edge_weights,
                                int32_t keep_isolated, const rvx_buffer* x, int32_t dim, rvx_buffer* out);

/* ------------------------------------------------------------------ */
/* GraphSAGE (crates/ruvector-postgres/src/gnn/graphsage.rs:25-196)    */
/* ------------------------------------------------------------------ */
typedef struct rvx_sage_layer rvx_sage_layer;
typedef struct rvx_comm rvx_comm; /* RCCL communicator, see Multi-GPU below */
enum { RVX_SAGE_MEAN = 0, RVX_SAGE_MAXPOOL = 1, RVX_SAGE_LSTM = 2 /* = mean, graphsage.rs:159 */ };
/* w_neighbor/w_self: [in][out] row-major as GraphSAGELayer stores them; NULL
 * for both selects the deterministic init of graphsage.rs:56-78.
 * Rows with more than num_samples neighbours aggregate the subset
 * sample_neighbors keeps (StdRng::seed_from_u64(42) + partial_shuffle, then
 * the prefix; graphsage.rs:92-102), built once per graph as a sampled CSR. */
rvx_status rvx_sage_layer_create(int32_t in_features, int32_t out_features, int32_t num_samples,
                                 int32_t aggregator, int32_t normalize, const float* w_neighbor,
                                 const float* w_self, rvx_sage_layer** out);
rvx_status rvx_sage_layer_destroy(rvx_sage_layer* l);
/* GraphSAGELayer::sample_neighbors (graphsage.rs:92-102) on positions
 * 0..len-1 (len > k): writes the k positions the reference keeps, in order.
 * Host-only (rand 0.8.5 StdRng + SliceRandom::partial_shuffle restated). */
rvx_status rvx_sage_sample_positions(int32_t len, int32_t k, int32_t* out);
/* GraphSAGELayer::forward (graphsage.rs:190-196) over host arrays. */
rvx_status rvx_sage_forward(const rvx_sage_layer* l, const rvx_graph* g, const float* x, int64_t n,
                            float* y);
/* Same over HBM-resident buffers: x [n][in], y [n][out]. */
rvx_status rvx_sage_forward_device(const rvx_sage_layer* l, const rvx_graph* g, const rvx_buffer* x,
                                   rvx_buffer* y);
/* Node-range shard: g holds this rank's destination rows
 * [row_offset, row_offset + g.n) with GLOBAL column ids; x_full [N][in] is the
 * all-gathered node table; y [g.n][out] receives the owned rows. */
rvx_status rvx_sage_forward_shard_device(const rvx_sage_layer* l, const rvx_graph* g, const rvx_buffer* x_full,
                                         int64_t row_offset, rvx_buffer* y);
/* One layer of a node-range-sharded stack with the halo exchange fused in
 * (replaces the per-node loop of
 * GraphSAGELayer::forward, graphsage.rs:190-196, over the shard). Rank r
 * (of comm; NULL = single GPU) owns rows [offsets[r], offsets[r+1]) and g
 * holds those CSR rows with GLOBAL column ids. Reads x_full [N][in]; writes the
 * owned rows of y_full [N][out] and, when `exchange` != 0, receives every
 * peer's rows of y_full over RCCL point-to-point as they are produced, so the
 * next layer can read the whole table. The exchange of chunk c overlaps the
 * compute of chunk c+1; the call returns with all of it queued on the library
 * stream. x_full and y_full must differ. offsets has comm_size+1 entries. */
rvx_status rvx_sage_forward_exchange(const rvx_sage_layer* l, const rvx_graph* g, const rvx_buffer* x_full,
                                     rvx_buffer* y_full, const int64_t* offsets, rvx_comm* comm, int32_t exchange);
/* rvx_sage_forward_exchange for a stack with the L2 normalisation (graphsage.rs:177-182)
 * carried between layers instead of materialised (an rvx extension; the values are the
 * reference's within the 1e-5 bar). x_rowmul (NULL = none) [N] floats: row i of x_full
 * enters the layer as x_full[i] * x_rowmul[i] (the previous layer's y_rowinv). y_rowinv
 * (NULL = none) [N] floats: the owned rows of y_full are left unnormalised and
 * y_rowinv[i] = 1 / |y_full[i]| (1 where the norm is 0 or NaN) is written instead, and
 * exchanged with the rows. Where the layer's GEMM path cannot take it (not the split-f16
 * h2g path), x_full is rescaled in place by x_rowmul and y_full normalised as usual, with
 * y_rowinv set to 1. A stack's last layer passes y_rowinv = NULL. */
rvx_status rvx_sage_forward_exchange2(const rvx_sage_layer* l, const rvx_graph* g, rvx_buffer* x_full,
                                      const rvx_buffer* x_rowmul, rvx_buffer* y_full, rvx_buffer* y_rowinv,
                                      const int64_t* offsets, rvx_comm* comm, int32_t exchange);
/* ReLU-sparse row images (an rvx extension, no reference counterpart; values unchanged).
 * A GraphSAGE layer's output rows are (n + s).max(0.0) (graphsage.rs:172-176): about half of
 * every entry is +0.0. An image of an [n][dim] f32 table keeps, per row, a 3 KiB slot with the
 * row's entries other than +0.0 (bit patterns preserved) and a bitmap, when there are at most
 * 736 of them (beyond that the dense row is fewer bytes), plus a u16 count per row; a gather over the image adds exactly the terms, in
 * exactly the order, of a gather over the table (mean / sum aggregators), reading about half
 * the bytes. Needs 512 < dim <= 768, dim % 4 == 0.
 * rvx_row_image_bytes: the image buffer size for n rows.
 * rvx_row_image_pack: rows [r0, r0 + rows) of x (n_total x dim) into the image.
 * rvx_sage_forward_exchange3 = rvx_sage_forward_exchange2 plus: x_image (NULL = none), an image
 * of x_full's current contents (every row; the caller keeps it current — e.g. the previous
 * layer's y_image), read by the overlapped gather for neighbour rows; y_image (NULL = none)
 * receives the image of every row of y_full the call writes or receives. Same output bits
 * with or without images. */
rvx_status rvx_row_image_bytes(int64_t n, int32_t dim, int64_t* bytes);
rvx_status rvx_row_image_pack(const rvx_buffer* x, int64_t n_total, int64_t r0, int64_t rows, int32_t dim,
                              rvx_buffer* image);
rvx_status rvx_sage_forward_exchange3(const rvx_sage_layer* l, const rvx_graph* g, rvx_buffer* x_full,
                                      const rvx_buffer* x_rowmul, rvx_buffer* x_image, rvx_buffer* y_full,
                                      rvx_buffer* y_rowinv, rvx_buffer* y_image, const int64_t* offsets,
                                      rvx_comm* comm, int32_t exchange);


/* ------------------------------------------------------------------ */
/* GCN (crates/ruvector-postgres/src/gnn/gcn.rs:12-149)                */
/* ------------------------------------------------------------------ */
typedef struct rvx_gcn_layer rvx_gcn_layer;
/* weights [in][out] (NULL = deterministic init gcn.rs:32-41), bias [out] (NULL = zeros). */
rvx_status rvx_gcn_layer_create(int32_t in_features, int32_t out_features, int32_t normalize,
                                const float* weights, const float* bias, rvx_gcn_layer** out);
rvx_status rvx_gcn_layer_destroy(rvx_gcn_layer* l);
/* GCNLayer::forward (gcn.rs:93-112): propagate(_weighted) then ReLU. */
rvx_status rvx_gcn_forward(const rvx_gcn_layer* l, const rvx_graph* g, int32_t use_edge_weights,
                           const float* x, int64_t n, float* y);

/* ------------------------------------------------------------------ */
/* RuvectorLayer (crates/ruvector-gnn/src/layer.rs:313-457)            */
/* ------------------------------------------------------------------ */
typedef struct rvx_layer rvx_layer;
/* RuvectorLayer::new (layer.rs:347-368). Weights are drawn from a seeded
 * normal(0, sqrt(2/(in+out))) stream (the reference draws them from
 * thread_rng, layer.rs:21-34, so they are an input for parity). */
rvx_status rvx_gnn_layer_create(int32_t input_dim, int32_t hidden_dim, int32_t heads, float dropout,
                                uint64_t seed, rvx_layer** out);
/* serde_json form of RuvectorLayer (layer.rs:313-333; ndarray {v,dim,data}). */
rvx_status rvx_gnn_layer_from_json(const char* json, rvx_layer** out);
/* Writes the JSON into buf (NUL-terminated) if it fits; *len receives the size
 * needed including the NUL. */
rvx_status rvx_gnn_layer_to_json(const rvx_layer* l, char* buf, size_t* len);
rvx_status rvx_gnn_layer_dims(const rvx_layer* l, int32_t* input_dim, int32_t* hidden_dim, int32_t* heads,
                              float* dropout);
rvx_status rvx_gnn_layer_destroy(rvx_layer* l);
/* RuvectorLayer::forward for one node (layer.rs:379-418): node [in],
 * nbrs [deg][in] contiguous, w [num_weights]. */
rvx_status rvx_gnn_forward_one(const rvx_layer* l, const float* node, const float* nbrs, int32_t deg,
                               const float* w, int32_t num_weights, float* out);
/* Batched: every node i of the graph as `node`, its CSR row as neighbours
 * (in edge order) and the CSR edge weights as `edge_weights`
 * (nullable graph weights = empty weight slice, layer.rs:422-424). */
rvx_status rvx_gnn_forward_graph(const rvx_layer* l, const rvx_graph* g, const float* x, int64_t n,
                                 float* y);
rvx_status rvx_gnn_forward_graph_device(const rvx_layer* l, const rvx_graph* g, const rvx_buffer* x,
                                        rvx_buffer* y);
/* Node-range-sharded RuvectorLayer forward, one process per GPU: this
 * rank owns destination rows [offsets[rank], offsets[rank+1]) and `g` holds their CSR
 * rows with GLOBAL column ids. x_full / y_full are [N][in] / [N][hidden] tables, of which
 * only the owned rows of x_full are read and only the owned rows of y_full written.
 * Phase 1 (M = w_msg(x), K|V) runs on the owned rows; their rows of M and K|V go to every
 * peer over RCCL p2p (comm, rvx_comm_init); phase 2 (attention over neighbours, GRU,
 * LayerNorm; layer.rs:379-418) runs on the owned rows. The next layer needs only the
 * owned rows of y_full, so stacked layers exchange M|K|V once per layer and nothing
 * else. comm NULL: one process, offsets {0, N}; identical to rvx_gnn_forward_graph_device. */
rvx_status rvx_gnn_forward_exchange(const rvx_layer* l, const rvx_graph* g, const rvx_buffer* x_full,
                                    rvx_buffer* y_full, const int64_t* offsets, rvx_comm* comm);

/* RuvectorLayer::forward(node, neighbours, edge_weights) (layer.rs:379-423), batched over
 * nq independent nodes whose neighbours are rows of a resident table:
 * nodes [nq][input_dim], table [table_rows][input_dim], cand_ids [nq][c] int64 (ids outside
 * [0, table_rows) are absent neighbours), weights [nq][c] raw edge weights or NULL (no
 * weights -> the zero weighted aggregate, layer.rs:427-429) -> out [nq][hidden_dim].
 * The query-time re-embedding of RuvectorQuery's neural search (query.rs:44-58). */
rvx_status rvx_gnn_forward_star_device(const rvx_layer* l, const rvx_buffer* nodes, int64_t nq, const rvx_buffer* table,
                                       int64_t table_rows, const rvx_buffer* cand_ids, int32_t c,
                                       const rvx_buffer* weights, rvx_buffer* out);

/* hierarchical_forward (crates/ruvector-gnn/src/search.rs:105-162) for nq queries at once,
 * all in HBM. Walks zip(levels, layers): level s (level_rows[s] rows of the current
 * embedding dim, row-major; 0 rows = skipped) gives differentiable_search top-min(5, rows)
 * at temperature 1 over ALL its rows, the soft-weighted row sum agg, combined =
 * (cur + agg) / 2, then cur = layers[s]->forward(combined, top rows, top weights).
 * q [nq][dim] -> out [nq][*out_dim] (out_dim = last applied layer's hidden_dim, or dim).
 * Errors: DimensionMismatch when a layer's input_dim differs from the embedding dim
 * (the reference asserts in cosine_similarity, search.rs:5). Replaces the per-query
 * Rust call; the reference has no batched form. */
rvx_status rvx_hierarchical_forward_device(const rvx_layer* const* layers, int32_t n_layers,
                                           const rvx_buffer* const* levels, const int64_t* level_rows,
                                           int32_t n_levels, const rvx_buffer* q, int64_t nq, int32_t dim,
                                           rvx_buffer* out, int32_t* out_dim);
/* differentiable_search (crates/ruvector-gnn/src/search.rs:56-94), batched:
 * q [nq][d], cand [nq][c][d] -> idx [nq][k] (int64, -1 padded), w [nq][k]. */
rvx_status rvx_differentiable_search_batch(const float* q, int64_t nq, const float* cand, int32_t c,
                                           int32_t d, int32_t k, float temperature, int64_t* idx, float* w);
/* Device form over candidates gathered by id from a resident table (every id must be a
 * table row): q [nq][d], cand_ids [nq][c] -> idx [nq][k] (positions in the candidate
 * list), w [nq][k]; soft (nullable) [nq][c] = the softmax weights in candidate order. */
rvx_status rvx_differentiable_search_device(const rvx_buffer* q, int64_t nq, const rvx_buffer* table, int64_t table_rows,
                                            const rvx_buffer* cand_ids, int32_t c, int32_t d, int32_t k,
                                            float temperature, rvx_buffer* idx, rvx_buffer* w, rvx_buffer* soft);

/* ------------------------------------------------------------------ */
/* Graph attention head: EdgeFeaturedAttention                         */
/* (crates/ruvector-attention/src/graph/edge_featured.rs:87-320)       */
/* ------------------------------------------------------------------ */
typedef struct rvx_edge_attention rvx_edge_attention;
typedef struct {
    int32_t node_dim, edge_dim, num_heads; float dropout; int32_t concat_heads, add_self_loops;
    float negative_slope;
} rvx_edge_attention_config; /* EdgeFeaturedConfig, edge_featured.rs:11-33 */
/* Deterministic LCG init of EdgeFeaturedAttention::new (edge_featured.rs:98-141). */
rvx_status rvx_edge_attention_create(const rvx_edge_attention_config* cfg, rvx_edge_attention** out);
rvx_status rvx_edge_attention_destroy(rvx_edge_attention* a);
rvx_status rvx_edge_attention_dim(const rvx_edge_attention* a, int32_t* out_dim);
/* compute_with_edges for one query (edge_featured.rs:196-258): keys/values [n][node_dim],
 * edges [n][edge_dim] (NULL = zero edge features, i.e. Attention::compute, :267-288). */
rvx_status rvx_edge_attention_compute(const rvx_edge_attention* a, const float* query, const float* keys,
                                      const float* values, const float* edges, int32_t n, float* out);
/* Whole graph: query = x_i, keys = values = x_j for j in adj(i),
 * edges [E][edge_dim] in CSR order (nullable). Rows without neighbours
 * return RVX_ERR_INVALID_PARAMETER unless add_self_loops (then key = x_i). */
rvx_status rvx_edge_attention_forward_graph_device(const rvx_edge_attention* a, const rvx_graph* g,
                                                   const rvx_buffer* x, const rvx_buffer* edge_feat,
                                                   rvx_buffer* y);
/* Node-range sharded form of the above (one process per GPU): g holds this rank's
 * rows [offsets[rank], offsets[rank+1]) with global column ids, edge_feat its
 * edges, x_full/y_full are whole-table [N][*] buffers of which only the owned
 * rows are read/written. The transformed rows x W_node^T are exchanged once
 * (one grouped RCCL p2p round); comm NULL = one process, offsets {0, N}. */
rvx_status rvx_edge_attention_forward_exchange(const rvx_edge_attention* a, const rvx_graph* g,
                                               const rvx_buffer* x_full, const rvx_buffer* edge_feat,
                                               rvx_buffer* y_full, const int64_t* offsets, rvx_comm* comm);

/* DualSpaceAttention (crates/ruvector-attention/src/graph/dual_space.rs:95-293):
 * Euclidean (scaled dot of x W_euclidean^T) and hyperbolic (-poincare_dist of
 * project_to_ball(x W_hyperbolic^T)) scores combined as (we*e + wh*h)/temperature,
 * stable_softmax, weighted sum of values, output projection W_out when the values
 * have `dim` columns. Weights: the reference's LCG stream (seed 42, new():107-131). */
typedef struct rvx_dual_attention rvx_dual_attention;
typedef struct {                  /* DualSpaceConfig (dual_space.rs:30-50) */
    int32_t dim;                  /* 256 */
    float   curvature;            /* 1.0 */
    float   euclidean_weight;     /* 0.5 */
    float   hyperbolic_weight;    /* 0.5 */
    float   temperature;          /* 1.0 */
} rvx_dual_attention_config;
rvx_status rvx_dual_attention_create(const rvx_dual_attention_config* cfg, rvx_dual_attention** out);
rvx_status rvx_dual_attention_destroy(rvx_dual_attention* a);
/* Attention::compute (dual_space.rs:207-268): query [dim], keys [n][dim], values
 * [n][value_dim] (value_dim <= 1024) -> out [value_dim]. n == 0 -> RVX_ERR_INVALID_PARAMETER
 * ("Empty keys", the reference's InvalidConfig). */
rvx_status rvx_dual_attention_compute(const rvx_dual_attention* a, const float* query, const float* keys,
                                      const float* values, int32_t n, int32_t value_dim, float* out);
/* Every node of a CSR graph attends over its neighbours (keys = values = their rows
 * of x [N][dim]); y [N][dim]; isolated rows give zeros. */
rvx_status rvx_dual_attention_forward_graph_device(const rvx_dual_attention* a, const rvx_graph* g,
                                                   const rvx_buffer* x, rvx_buffer* y);

/* ------------------------------------------------------------------ */
/* Vector index: VectorIndex (crates/ruvector-core/src/index.rs:11-36) */
/*   FlatIndex (index/flat.rs) and HnswIndex (index/hnsw.rs)           */
/* ------------------------------------------------------------------ */
typedef struct rvx_index rvx_index;
enum { RVX_INDEX_FLAT = 0, RVX_INDEX_HNSW = 1 };
typedef struct {
    int32_t kind;            /* RVX_INDEX_FLAT / RVX_INDEX_HNSW (VectorDB picks HNSW iff hnsw_config, vector_db.rs:81-98) */
    int32_t dim;
    int32_t metric;          /* RVX_METRIC_* */
    int32_t m;               /* HnswConfig::m (types.rs:87-96: 32); the GPU build takes m <= 128 (layer 0: 2m) */
    int32_t ef_construction; /* 200 */
    int32_t ef_search;       /* 100 */
    int64_t max_elements;    /* 10_000_000 */
    float   curvature;       /* POINCARE only */
    uint64_t seed;           /* level-generator seed (the reference uses StdRng::from_entropy) */
} rvx_index_config;
rvx_status rvx_index_create(const rvx_index_config* cfg, rvx_index** out);
rvx_status rvx_index_destroy(rvx_index* idx);
/* add_batch: vecs [n][dim]; ids are the caller's dense u64 keys (VectorId). */
rvx_status rvx_index_add_batch(rvx_index* idx, const float* vecs, const uint64_t* ids, int64_t n);
rvx_status rvx_index_add_batch_device(rvx_index* idx, const rvx_buffer* vecs, int64_t n, uint64_t first_id);
rvx_status rvx_index_len(const rvx_index* idx, int64_t* len);
/* remove(id) (index/hnsw.rs:322-338): the id disappears from results; graph kept. */
rvx_status rvx_index_remove(rvx_index* idx, uint64_t id, int32_t* removed);
/* search (VectorIndex::search / HnswIndex::search_with_ef, index/hnsw.rs:231-260):
 * q [nq][dim] -> out_ids [nq][k], out_dist [nq][k] ascending, out_count [nq].
 * ef <= 0 selects cfg.ef_search. Unused slots: id UINT64_MAX, dist +inf. */
rvx_status rvx_index_search(const rvx_index* idx, const float* q, int64_t nq, int32_t k, int32_t ef,
                            uint64_t* out_ids, float* out_dist, int32_t* out_count);
rvx_status rvx_index_search_device(const rvx_index* idx, const rvx_buffer* q, int64_t nq, int32_t k,
                                   int32_t ef, rvx_buffer* out_ids_u64, rvx_buffer* out_dist_f32);
/* Exact scan (FlatIndex::search, index/flat.rs:36-76): ties broken by id. */
rvx_status rvx_index_brute_force(const rvx_index* idx, const float* q, int64_t nq, int32_t k,
                                 uint64_t* out_ids, float* out_dist);
rvx_status rvx_index_brute_force_device(const rvx_index* idx, const rvx_buffer* q, int64_t nq, int32_t k,
                                        rvx_buffer* out_ids_u64, rvx_buffer* out_dist_f32);
/* Node-range-sharded search across processes (SURVEY.md §8e option 2; the merge of
 * ShardedHyperbolicHnsw::search, crates/ruvector-hyperbolic-hnsw/src/shard.rs:354-373,
 * applied to VectorIndex shards): one index shard per rank of `comm` (NULL = one
 * process). Rank 0's queries q [nq][dim] are broadcast (q is ignored on other ranks;
 * nq, k, ef, exact must agree on every rank), every rank searches its shard
 * (exact != 0: the FlatIndex scan), one all-gather moves every rank's top-k and every
 * rank merges them by distance, ties in rank order. Outputs as rvx_index_search (user
 * ids are the caller's global keys), identical on every rank. */
rvx_status rvx_index_sharded_search(const rvx_index* idx, rvx_comm* comm, const float* q, int64_t nq, int32_t k,
                                    int32_t ef, int32_t exact, uint64_t* out_ids, float* out_dist,
                                    int32_t* out_count);
rvx_status rvx_index_sharded_search_device(const rvx_index* idx, rvx_comm* comm, const rvx_buffer* q, int64_t nq,
                                           int32_t k, int32_t ef, int32_t exact, rvx_buffer* out_ids_u64,
                                           rvx_buffer* out_dist_f32);
/* Work of the most recent HNSW search launch in this process (any index): distance
 * evaluations, layer-0 expansions and queries — the algorithmic traffic of the search is
 * n_dist * dim * 4 + n_expand * deg_cap * 4 bytes. */
rvx_status rvx_hnsw_last_search_stats(int64_t* n_dist, int64_t* n_expand, int64_t* nq);
/* Visited-set form of that launch: bitmap 1 = per-slot bitmaps over all nodes (when
 * min(nq, 1024) slots fit min(16 GiB, 1/4 of free HBM)), 0 = the tagged hash; slots =
 * concurrent search slots. */
rvx_status rvx_hnsw_last_search_visited(int32_t* bitmap, int32_t* slots);
/* Kernel form of that launch (an rvx extension for tests and benchmarks; results are the same
 * in every form): r_in_hbm 1 = the result list R in an HBM row per search slot (past one wave's
 * LDS, or where an LDS R would leave < 4 waves per CU), 0 = in LDS; stages = LDS-staged distance
 * stages per wave (0: per-lane distances), visited_overflow 1 = a query's visited hash filled. */
rvx_status rvx_hnsw_last_search_form(int32_t* r_in_hbm, int32_t* stages, int32_t* visited_overflow);
/* Path taken by the most recent exact scan in this process (rvx_index_brute_force*, FlatIndex
 * search): queries ranked by the MFMA filter + exact re-rank, queries scanned by the exact VALU
 * kernel, and queries the filter handed back to the VALU kernel (completeness not provable).
 * Results are identical either way; this is for tests and benchmarks. */
rvx_status rvx_scan_last_stats(int64_t* mfma_queries, int64_t* valu_queries, int64_t* fallback_queries);
/* Queries of that scan the MFMA filter ran a second time with the most splits the re-rank holds
 * (one conversion chunk), after their first lists could not prove completeness; those still
 * unsure are the fallback queries above (an rvx extension for tests and benchmarks). */
rvx_status rvx_scan_last_second_pass(int64_t* second_pass_queries);
/* Queries of that scan still unsure after the list passes that took the band pass: every row whose
 * filter value is within the bound the re-rank proved, then those rows' reference distances (one
 * conversion chunk); a band past its capacity is a fallback query (an rvx extension for tests and
 * benchmarks). */
rvx_status rvx_scan_last_band(int64_t* band_queries);

/* HNSW graph interchange (fixed-graph parity and GNN topology).
 * Layer 0: CSR over all n points in stored neighbour order (hnsw_rs keeps
 * every list sorted by distance to its owner, hnsw.rs:1186,1268).
 * Upper layers l=1..max_level: points with level >= l, as a per-layer CSR
 * over that sorted point list. */
typedef struct {
    int64_t n; int32_t max_level; int64_t entry_point;
    const uint8_t* levels;          /* [n] */
    const int64_t* row_ptr0;        /* [n+1] */
    const int32_t* col0;            /* [row_ptr0[n]] */
    const int64_t* upper_count;     /* [max_level+1], upper_count[0] unused */
    const int32_t* const* upper_ids;      /* per layer l>=1: sorted point ids [upper_count[l]] */
    const int64_t* const* upper_row_ptr;  /* per layer: [upper_count[l]+1] */
    const int32_t* const* upper_col;      /* per layer */
} rvx_hnsw_graph;
rvx_status rvx_index_load_graph(rvx_index* idx, const rvx_hnsw_graph* g);
/* Export the searchable graph (built by add_batch on the GPU, or loaded) in the
 * rvx_hnsw_graph layout: sizes first (upper_count/upper_edges [17]), then the
 * arrays; upper layers are concatenated in layer order (1..max_level), each
 * row_ptr block holding upper_count[l]+1 entries. */
rvx_status rvx_index_graph_sizes(const rvx_index* idx, int64_t* n, int32_t* max_level, int64_t* entry_point,
                                 int64_t* num_edges0, int64_t* upper_count, int64_t* upper_edges);
rvx_status rvx_index_export_graph(const rvx_index* idx, uint8_t* levels, int64_t* row_ptr0, int32_t* col0,
                                  int32_t* upper_ids, int64_t* upper_row_ptr, int32_t* upper_col);
/* Layer-0 adjacency export for the GNN (edge weight = stored distance). */
rvx_status rvx_index_layer0_size(const rvx_index* idx, int64_t* n, int64_t* num_edges);
rvx_status rvx_index_export_layer0(const rvx_index* idx, int64_t* row_ptr, int32_t* col, float* dist);

/* hnsw_rs dump files `<dir>/<basename>.hnsw.graph` + `.hnsw.data`
 * (patches/hnsw_rs/src/hnswio.rs: Description::dump :878-919,
 * PointIndexation::dump :1301-1332, dump_point :1063-1110; reload
 * load_description :937-1040, load_point_indexation :615-790). Written in
 * format 4, Full mode (the only mode the reference reloads), distance named
 * after the anndists type of the metric; user ids are the origin ids.
 * rvx_index_file_dump replaces Hnsw::file_dump; rvx_index_file_load replaces
 * HnswIo::load_hnsw and puts the dumped graph (and vectors) on the GPU as the
 * searchable graph (metric < 0: from the distance name). */
typedef struct {
    int32_t format_version;      /* 2, 3, 4 (MAGICDESCR_*) */
    int32_t dump_mode;           /* 1 = Full */
    int32_t max_nb_connection;
    int32_t nb_layer;
    double  level_scale;
    int64_t ef_construction;
    int64_t nb_point;
    int64_t dimension;
    char    distname[257];
    char    t_name[257];
} rvx_hnswio_description;
rvx_status rvx_hnswio_describe(const char* dir, const char* basename, rvx_hnswio_description* out);
rvx_status rvx_index_file_dump(const rvx_index* idx, const char* dir, const char* basename);
rvx_status rvx_index_file_load(const char* dir, const char* basename, int32_t metric, int32_t ef_search,
                               uint64_t seed, rvx_index** out);
/* Stored rows [row0, row0+count) of an index (insertion order): vectors
 * (count x dim), user ids, tombstones; total_rows = rows stored. The data
 * behind VectorDB::get and HnswIndex::serialize (index/hnsw.rs:136-169). */
rvx_status rvx_index_export_rows(const rvx_index* idx, int64_t row0, int64_t count, float* vecs, uint64_t* ids,
                                 uint8_t* deleted, int64_t* total_rows);

/* ------------------------------------------------------------------ */
/* Node-feature files <-> HBM                                          */
/* ------------------------------------------------------------------ */
/* RVX_FEATURE_RAW: MmapManager's embedding file (crates/ruvector-gnn/src/
 *   mmap.rs:147-218): row i at byte i*dim*4, no header (dim given by caller).
 * RVX_FEATURE_COLD_TIER: FeatureStorage (crates/ruvector-gnn/src/cold_tier.rs:
 *   17-151): header {dim, num_nodes, block_size} u64 LE, row i at
 *   24 + i*block_size, block_size = dim*4 rounded up to the page size.
 * Loads stream through pinned double-buffered staging (pread overlaps DMA). */
enum { RVX_FEATURE_RAW = 0, RVX_FEATURE_COLD_TIER = 1 };
rvx_status rvx_feature_file_info(const char* path, int32_t layout, int64_t dim, int64_t* rows, int64_t* dim_out,
                                 int64_t* block_size);
rvx_status rvx_feature_file_load(const char* path, int32_t layout, int64_t dim, int64_t row0, int64_t nrows,
                                 rvx_buffer* dst, int64_t dst_row0);
/* block_size (COLD_TIER only): page size to align blocks to; 0 = the host's. */
rvx_status rvx_feature_file_store(const char* path, int32_t layout, const rvx_buffer* src, int64_t dim, int64_t nrows,
                                  int64_t block_size);

/* ------------------------------------------------------------------ */
/* Distances (distance.rs:9-107, poincare.rs:227-301)                  */
/* ------------------------------------------------------------------ */
/* out[i][j] = distance(q_i, x_j) for q [nq][d], x [n][d], in the reference's
 * scalar accumulation order. */
rvx_status rvx_distance_matrix(int32_t metric, const float* q, int64_t nq, const float* x, int64_t n,
                               int32_t d, float curvature, float* out);

/* Self-test of the device libm restatements that make Poincaré distances, log maps and
 * exp maps bit-identical to the reference (f32::ln -> glibc logf, f32::ln_1p -> log1pf,
 * f32::tanh -> tanhf, f32::atanh -> Rust std's 0.5 * ln_1p(2x / (1 - x)); poincare.rs:259-276,
 * :407-451): out[i] = f(bits(start + i * stride)) evaluated on the GPU, f = 0 logf,
 * 1 log1pf, 2 expm1f, 3 tanhf, 4 atanh. Not part of the reference API. */
rvx_status rvx_selftest_libm(int32_t fn, uint64_t start, uint64_t stride, int64_t count, float* out);

/* ------------------------------------------------------------------ */
/* HyperbolicHnsw: Poincaré-ball HNSW                                  */
/* (crates/ruvector-hyperbolic-hnsw/src/hnsw.rs:127-528, tangent.rs)   */
/* ------------------------------------------------------------------ */
typedef struct rvx_hyperbolic rvx_hyperbolic;
typedef struct {                 /* HyperbolicHnswConfig (hnsw.rs:36-72), metric Poincaré or Euclidean */
    int32_t dim;
    int32_t max_connections;     /* M, 16 (<= 128 for the GPU build) */
    int32_t max_connections_0;   /* M0 at layer 0, 32 (<= 256 for the GPU build) */
    int32_t ef_construction;     /* 200 */
    int32_t ef_search;           /* 50 */
    float   level_mult;          /* 1 / ln(16) */
    float   curvature;           /* 1.0, > 0 */
    int32_t prune_factor;        /* 10: search_with_pruning keeps k * prune_factor (<= 128) */
    uint64_t seed;               /* level draws (the reference uses rand::random) */
    int32_t metric;              /* RVX_METRIC_POINCARE (default) or RVX_METRIC_HYP_L2 (DistanceMetric::Euclidean) */
} rvx_hyperbolic_config;
/* HyperbolicHnswConfig::default() with dim = 0 (set it). */
void rvx_hyperbolic_default_config(rvx_hyperbolic_config* cfg);
/* HyperbolicHnsw::new (hnsw.rs:143-151). curvature <= 0 -> RVX_ERR_INVALID_PARAMETER (InvalidCurvature). */
rvx_status rvx_hyperbolic_create(const rvx_hyperbolic_config* cfg, rvx_hyperbolic** out);
rvx_status rvx_hyperbolic_destroy(rvx_hyperbolic* h);
/* The underlying graph index (borrowed; owned by h): rvx_index_graph_sizes /
 * export_graph / load_graph / len work on it. */
rvx_status rvx_hyperbolic_index(rvx_hyperbolic* h, rvx_index** out);
/* insert / insert_batch (hnsw.rs:226-305): each vector is projected into the
 * ball; ids are insertion order (first_id returns the first new id). Invalidates
 * the tangent cache. */
rvx_status rvx_hyperbolic_insert_batch(rvx_hyperbolic* h, const float* vecs, int64_t n, int64_t* first_id);
rvx_status rvx_hyperbolic_insert_batch_device(rvx_hyperbolic* h, const rvx_buffer* vecs, int64_t n, int64_t* first_id);
rvx_status rvx_hyperbolic_len(const rvx_hyperbolic* h, int64_t* len);
/* search (hnsw.rs:427-447): ids [nq][k] (-1 past the end), distances ascending;
 * ef = max(ef or ef_search when 0, k). */
rvx_status rvx_hyperbolic_search(const rvx_hyperbolic* h, const float* q, int64_t nq, int32_t k, int32_t ef,
                                 int64_t* ids, float* dist, int32_t* counts);
/* search_with_pruning (hnsw.rs:450-489); without a tangent cache: search. */
rvx_status rvx_hyperbolic_search_with_pruning(const rvx_hyperbolic* h, const float* q, int64_t nq, int32_t k,
                                              int64_t* ids, float* dist, int32_t* counts);
/* Exact scan by HyperbolicHnsw::distance (ground truth; k <= 128, dim % 4 == 0). */
rvx_status rvx_hyperbolic_brute_force(const rvx_hyperbolic* h, const float* q, int64_t nq, int32_t k, int64_t* ids,
                                      float* dist);
/* HBM-resident queries/outputs; mode 0 search, 1 exact, 2 with pruning. */
rvx_status rvx_hyperbolic_search_device(const rvx_hyperbolic* h, const rvx_buffer* q, int64_t nq, int32_t k, int32_t ef,
                                        int32_t mode, rvx_buffer* ids_i64, rvx_buffer* dist);
/* build_tangent_cache (hnsw.rs:492-503): Fréchet-mean centroid + log maps. */
rvx_status rvx_hyperbolic_build_tangent_cache(rvx_hyperbolic* h);
rvx_status rvx_hyperbolic_tangent_centroid(const rvx_hyperbolic* h, float* centroid);
rvx_status rvx_hyperbolic_get_vector(const rvx_hyperbolic* h, int64_t id, float* out);
/* set_curvature (hnsw.rs:511-530): reprojects all vectors, rebuilds an existing cache. */
rvx_status rvx_hyperbolic_set_curvature(rvx_hyperbolic* h, float curvature);
/* ShardedHyperbolicHnsw::search (shard.rs:354-373) across processes: this rank's
 * HyperbolicHnsw holds the node-range shard of global ids [id_base, id_base + len).
 * Rank 0's queries q [nq][dim] are broadcast (ignored on other ranks; nq, k, ef and
 * mode must agree on every rank), every rank runs mode 0 search (what shard.search
 * calls, hnsw.rs:427), 1 exact scan or 2 search_with_pruning on its shard, one
 * all-gather of every rank's top-k, and every rank merges by distance (ties in rank
 * order, i.e. by global id) and keeps k. Results, identical on every rank, in the
 * reference's shape Vec<(global_id, SearchResult{id: local_id, distance})>:
 * out_gid / out_lid [nq][k] (-1 past the end), out_dist ascending, out_count [nq]
 * (out_lid / out_count nullable). comm NULL: one process (a plain search with id_base). */
rvx_status rvx_hyperbolic_sharded_search(const rvx_hyperbolic* h, rvx_comm* comm, int64_t id_base, const float* q,
                                         int64_t nq, int32_t k, int32_t ef, int32_t mode, int64_t* out_gid,
                                         int64_t* out_lid, float* out_dist, int32_t* out_count);
rvx_status rvx_hyperbolic_sharded_search_device(const rvx_hyperbolic* h, rvx_comm* comm, int64_t id_base,
                                                const rvx_buffer* q, int64_t nq, int32_t k, int32_t ef, int32_t mode,
                                                rvx_buffer* out_gid_i64, rvx_buffer* out_lid_i64 /*nullable*/,
                                                rvx_buffer* out_dist);

/* ------------------------------------------------------------------ */
/* Profiling: per-kernel device time measured with HIP events on the   */
/* stream the kernels run on.                                          */
/* ------------------------------------------------------------------ */
rvx_status rvx_profile_enable(int32_t on);
rvx_status rvx_profile_reset(void);
/* Total milliseconds and launch count of every launch tagged `name`. */
rvx_status rvx_profile_query(const char* name, double* total_ms, int64_t* launches);
/* Comma-separated list of tags seen since the last reset. */
rvx_status rvx_profile_names(char* buf, size_t len);

/* ------------------------------------------------------------------ */
/* Multi-GPU: node-range sharding with RCCL over xGMI   */
/* ------------------------------------------------------------------ */
#define RVX_COMM_ID_BYTES 128
rvx_status rvx_comm_unique_id(uint8_t id[RVX_COMM_ID_BYTES]);
rvx_status rvx_comm_init(const uint8_t id[RVX_COMM_ID_BYTES], int32_t nranks, int32_t rank, rvx_comm** out);
rvx_status rvx_comm_destroy(rvx_comm* c);
/* All-gather of equal row blocks: send [rows][cols] f32 from every rank into
 * recv [nranks*rows][cols] (rank-major), on the library stream. */
rvx_status rvx_comm_allgather_f32(rvx_comm* c, const rvx_buffer* send, int64_t count, rvx_buffer* recv);
rvx_status rvx_comm_allreduce_max_f64(rvx_comm* c, double* value);
/* Host scalars reduced over every rank (sum / max / min), in place; also the
 * bench's barrier and its max-over-ranks clock, so no launcher-side collective
 * library is needed (the unique id travels over a TCP rendezvous,
 * ruvector_amd.shard.rendezvous_unique_id). */
#define RVX_REDUCE_SUM 0
#define RVX_REDUCE_MAX 1
#define RVX_REDUCE_MIN 2
rvx_status rvx_comm_allreduce_f64(rvx_comm* c, double* values, int32_t count, int32_t op);

/* Host-staged transport (tests and hosts without RCCL peers, e.g. several ranks
 * sharing one GPU): behind the same row exchange the *_forward_exchange entry
 * points use, each round stages this rank's rows in host memory and calls
 * `fn(user, send, send_bytes, recv, recv_bytes)` once: send this rank's block to
 * every peer and fill recv[p] (recv_bytes[p] bytes; recv[me] is NULL) from peer p.
 * Returns 0 on success. The sharded searches' broadcast (only the root sends) and
 * all-gather of per-rank top-k run through the same call; the f32 all-gather and
 * the all-reduces need RCCL. */
typedef int32_t (*rvx_host_exchange_fn)(void* user, const void* send, int64_t send_bytes, void* const* recv,
                                        const int64_t* recv_bytes);
rvx_status rvx_comm_init_host(int32_t nranks, int32_t rank, rvx_host_exchange_fn fn, void* user, rvx_comm** out);
/* Payload bytes this rank has handed to the transport (sent: a row block shipped to k peers
 * counts k times) and taken from it, over every exchange, broadcast and all-gather since the
 * communicator was made (an rvx extension: the exchange's measured bytes for bench reports). */
rvx_status rvx_comm_traffic(const rvx_comm* c, int64_t* sent, int64_t* recv);
/* RVX_COMM_SELF_P2P=1 on a one-rank RCCL communicator (an rvx extension for one-GPU boxes): the
 * GraphSAGE exchange's compact row records go out and come back through RCCL's p2p path and are
 * expanded by the receivers' unpack kernel into a shadow of the rows they came from; `rows` is
 * the number of rows so checked since the communicator was made, `mismatched_words` the 32-bit
 * words that differed (0: the record path is bit-exact behind a real RCCL transfer). Waits for
 * the device. */
rvx_status rvx_comm_selfcheck(rvx_comm* c, int64_t* rows, int64_t* mismatched_words);

/* The p2p round plan of the node-range exchange that the
 * *_forward_exchange entry points run: kind 0 = GraphSAGE (rvx_sage_forward_exchange:
 * the owned rows in row chunks, one round per chunk after that chunk's GEMM; every
 * rank uses the chunk count of the largest shard), kind 1 = RuvectorLayer / edge
 * attention tables (one round per table, whole shards). offsets [world+1]. With
 * r0 == NULL only *n_rounds is written; else r0/rows [n_rounds][world]: in round c
 * rank p ships rows [r0, r0+rows) (rows may be 0). Host-only: no device work. */
rvx_status rvx_exchange_plan(int32_t kind, const int64_t* offsets, int32_t world, int32_t* n_rounds, int64_t* r0,
                             int64_t* rows);

#ifdef __cplusplus
}
#endif
#endif /* RVX_RVX_H */
