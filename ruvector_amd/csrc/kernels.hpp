// kernels.hpp — internal launch wrappers shared by the C-ABI translation units.
// All launches go to rvx::stream() and are tagged for the event profiler.
#pragma once
#include <cstdint>

namespace rvx {

// ---- GEMM (gemm_f32.hip) ------------------------------------------------
enum { GEMM_EPI_STORE = 0, GEMM_EPI_RELU = 1, GEMM_EPI_SIGMOID = 2, GEMM_EPI_TANH = 3 };
struct GemmOperand {
    const float* A; int64_t lda;  // A [M][K]
    const float* B; int64_t ldb;  // B [N][K]  (C = A · B^T)
    int K;
    // optional exact 3-way bf16 split of B (split_x3): planes of [N][ldb]
    // uint16 at Bx3 + p*Bx3_plane; selects the split-bf16 MFMA kernel
    const uint16_t* Bx3 = nullptr;
    int64_t Bx3_plane = 0;
    // optional split-f16 planes of B (split_h2_rows): [hi][lo] f16 at
    // Bh + p*Bh_plane, b_inv[n] = 1 / column scale; selects gemm_nt_h2 in
    // gemm_auto (dual operands need planes split with one common column scale)
    const _Float16* Bh = nullptr;
    int64_t Bh_plane = 0;
    const float* b_inv = nullptr;
    // optional per-row max |a| of this operand, written by its producer (GemmEpilogue
    // row_absmax, mul_rows): [M][ROWSUMSQ_SLOTS] partial maxima (unused slots 0) that
    // gemm_auto turns into the split-f16 row scales instead of re-reading A
    const float* amax = nullptr;
};
// One row chunk of the overlapped GraphSAGE gather in its dynamic form (aggregate_rows_help):
// destination rows are taken from *counter (zeroed before either kernel starts), both by the
// chunk's own gather kernel and by the previous chunk's persistent GEMM once its tiles are done
// (GemmEpilogue::help). Arguments as aggregate_rows with the vector path's overlapped settings
// (no edge weights, zero-filled empty rows, no post-scale, no planes).
// ReLU-sparse row image of a node table (rows_image_pack): a GraphSAGE layer's output is
// (n + s).max(0.0) (graphsage.rs:172-176), so about half of every row is +0.0. Row r keeps a
// 3 KiB slot at slots + r * IMG_SLOT — a 128-B header (u16 per lane: bit 4j+k set <=> column
// 4*lane + 256*j + k is not +0.0) followed by those values in column order — when it has at
// most IMG_CAP such values; nnz[r] says which (nnz > IMG_CAP: the slot is unused and readers
// take the dense row). A reader reproduces every value bit for bit (omitted columns are
// exactly +0.0), so a gather over the image adds the same terms in the same order as over
// the table. For 512 < dim <= 768 (three 256-column blocks per row).
constexpr int IMG_SLOT = 3072, IMG_CAP = (IMG_SLOT - 128) / 4;  // 736: beyond it the dense row is fewer bytes
constexpr int IMG_WIN = 2 * IMG_SLOT + 16;  // LDS per gathering wave (two row windows + read slack)
struct RowImage {
    unsigned char* slots = nullptr; uint16_t* nnz = nullptr;
    explicit operator bool() const { return slots && nnz; }
};
bool row_image_ok(int dim);
// rows [r0, r0 + rows) of x (row stride dim) into the image
void rows_image_pack(const float* x, int64_t r0, int64_t rows, int dim, const RowImage& img);
// Compact exchange records of the node-range exchange (rvx_sage_forward_exchange3 at world > 1):
// a block of rows travels as the rows' image records back to back within a byte budget, and
// their counts; record i sits at off[i] = exclusive prefix sum of the record bytes (16-B
// rounded 128 + 4 * count; none past IMG_CAP) before it. Rows whose record ends past the budget
// (or have none) are overflow rows, sent dense after the rounds.
// counts of rows r0 + i into cnt[i]; acc (nullable) += {record bytes (dense bytes for rows past
// IMG_CAP), rows}
void rows_rec_count(const float* x, int64_t r0, int64_t rows, int dim, uint32_t* cnt, unsigned long long* acc);
// off[0 .. rows) from cnt (rocPRIM scan; temp of rec_offsets_temp_bytes(>= rows))
size_t rec_offsets_temp_bytes(int64_t rows);
void rec_offsets(const uint32_t* cnt, int64_t rows, uint64_t* off, void* temp, size_t temp_bytes);
// the sender: records of rows r0 + i at xs + off[i]; overflow rows' global ids appended to ovf_ids
void rows_xchg_pack(const float* x, int64_t r0, int64_t rows, int dim, unsigned char* xs, uint64_t budget,
                    const uint32_t* cnt, const uint64_t* off, int64_t* ovf_ids, unsigned long long* ovf_n);
// the receiver: records back into the dense rows r0 + i of x, bit for bit (and into img when
// given); overflow rows are left for rows_by_id
void rows_xchg_unpack(float* x, int64_t r0, int64_t rows, int dim, const unsigned char* xs, uint64_t budget,
                      const uint32_t* cnt, const uint64_t* off, const RowImage& img);
// Dense rows by global id: rows[i] = x[ids[i]] (gather) or x[ids[i]] = rows[i] (scatter).
void rows_by_id(float* x, int dim, const int64_t* ids, int64_t cnt, float* rows, bool scatter);
// rows ids[0 .. cnt) of x into the image (as rows_image_pack)
void rows_image_pack_ids(const float* x, const int64_t* ids, int64_t cnt, int dim, const RowImage& img);

struct AggHelp {
    const int64_t* rp; const int32_t* col; int64_t n;
    const float* x; int dim; int agg;
    float* out; const float* self_x; float* row_scale;
    const float* row_mul; const float* self_mul;
    unsigned* counter;
    // optional image of x (mean / sum, row_image_ok(dim)): neighbour rows are read from it
    const unsigned char* img_slots; const uint16_t* img_nnz;
    // 1: imaged rows expanded in registers (header, then each lane's values straight from
    // the record); 0: through the wave's LDS windows (RVX_IMG_REG)
    int img_reg;
};
// Epilogue: C = epi(alpha * acc + bias0 + bias1 + addend[row][col])
constexpr int ROWSUMSQ_SLOTS = 8;  // per-row partial sums of squares (column tiles >= 128 wide, N <= 1024)
struct GemmEpilogue {
    int epi = GEMM_EPI_STORE;
    float alpha = 1.0f;
    const float* bias0 = nullptr;
    const float* bias1 = nullptr;
    const float* addend = nullptr;
    int64_t ld_addend = 0;
    // gemm_nt_h2 only: then x /= |x| over each row of C (rows with norm 0 or NaN left as they
    // are), bit-identical to normalize_rows(C, M, N, only_positive = true); see gemm_h2_rownorm_ok
    bool normalize_rows = false;
    // gemm_nt_h2 only, for a normalisation deferred to the next layer (N <= 1024):
    // row_sumsq[row * ROWSUMSQ_SLOTS + t] receives sum of v^2 over output column tile t of
    // the row (v after the activation; fixed order; t < the tile count gemm_nt_h2 returns), and
    // a1_rowmul[row] multiplies the phase-1 (A1) operand row before the split (the previous
    // layer's 1 / |y|)
    float* row_sumsq = nullptr;
    const float* a1_rowmul = nullptr;
    // gemm_auto / gemm_nt_h2: row_absmax[row * ROWSUMSQ_SLOTS + t] receives max |v| over
    // output column tile t of the row (v as stored), every other slot 0 — the next GEMM's
    // row scale from the producer (GemmOperand::amax) instead of a pass over C
    float* row_absmax = nullptr;
    // gemm_nt_h2, persistent 256 x 192 tiles only: after the tile queue runs dry the blocks
    // take rows of this gather (the next row chunk's) — see AggHelp
    const AggHelp* help = nullptr;
    // gemm_auto with row_absmax (C4's z|r GEMM): columns >= gate_col0 are not stored in C;
    // gate_out[row][c - gate_col0] = v * gate_h[row][c - gate_col0] is (RuvectorLayer's r ⊙ h,
    // the same product as mul_rows), and row_absmax then holds the maxima of those products
    const float* gate_h = nullptr; int64_t ld_gate_h = 0;
    float* gate_out = nullptr; int64_t ld_gate_out = 0;
    int gate_col0 = 0;
};
// C[M][N] = epilogue(A0·B0^T [+ A1·B1^T])
void gemm_nt(int64_t M, int N, const GemmOperand& s0, const GemmOperand* s1, const GemmEpilogue& ep, float* C,
             int64_t ldc, const char* tag);

// dst[p*n + i] = bf16 part p of src[i] (exact split src = p0 + p1 + p2)
void split_x3(const float* src, int64_t n, uint16_t* dst);

// Split-f16 GEMM (gemm_nt_h2g): A rows pre-scaled in-kernel by a_scale[row]
// (powers of two from aggregate_rows' row_scale), B given as two f16 planes
// ([2][N][K], from split_h2_rows) with b_inv[n] its inverse column scale.
bool gemm_h2_ok(int64_t M, int N, const GemmOperand& s0, const GemmOperand* s1);
// persist: blocks per CU of a persistent grid (0 = one block per tile; -1 = RVX_GEMM_CAP, default 0)
// ep.normalize_rows is honoured when this holds (N % 4 == 0, N <= 1024, aligned C rows, opt-in RVX_GEMM_ROWNORM=1)
bool gemm_h2_rownorm_ok(int N, const float* C, int64_t ldc);
// returns the number of output column tiles (the row_sumsq slots it wrote per row)
int gemm_nt_h2(int64_t M, int N, const GemmOperand& s0, const _Float16* B0h, const GemmOperand* s1,
               const _Float16* B1h, const float* a_scale, const float* b_inv, const GemmEpilogue& ep, float* C,
               int64_t ldc, const char* tag, int persist = -1);
// Pre-split A (gemm_nt_h2p): Ah holds A*a_scale as f16 planes [2][M][lda]
// (plane stride a_plane), phase 0 in columns [0, s0.K), phase 1 (s1) in
// [s0.K, s0.K + s1->K); s0/s1 give K and the B planes as for gemm_nt_h2.
bool gemm_h2p_ok(int64_t M, int N, int64_t lda, int64_t a_plane, const GemmOperand& s0, const GemmOperand* s1);
void gemm_nt_h2p(int64_t M, int N, const _Float16* Ah, int64_t lda, int64_t a_plane, const GemmOperand& s0,
                 const _Float16* B0h, const GemmOperand* s1, const _Float16* B1h, const float* a_scale,
                 const float* b_inv, const GemmEpilogue& ep, float* C, int64_t ldc, const char* tag);
// gemm_nt_h2 when every operand carries f16 planes and the shapes allow it
// (per-row A scales computed here, row_scale_h2), else gemm_nt.
void gemm_auto(int64_t M, int N, const GemmOperand& s0, const GemmOperand* s1, const GemmEpilogue& ep, float* C,
               int64_t ldc, const char* tag);
// scale[r] = power of two putting max(|A0 row r|, |A1 row r|) in [2^14, 2^15).
// max |C[row][:]| into row_absmax slot 0 (slots 1.. zeroed): GemmEpilogue::row_absmax for
// GEMM paths whose epilogue does not write it
void row_absmax_pass(const float* C, int64_t ldc, int64_t M, int N, float* out);
void row_scale_h2(const float* A0, int64_t lda0, int K0, const float* A1, int64_t lda1, int K1, int64_t M,
                  float* scale);
// Common power-of-two scale t_n per row n of B0 (and B1), planes P = [hi][lo]
// of B*t_n in f16, inv[n] = 1/t_n.
void split_h2_rows(const float* B0, const float* B1, int N, int K, _Float16* P0, _Float16* P1, float* inv);

// ---- data generators (k_data.hip) ---------------------------------------
void fill_uniform(float* p, int64_t n, uint64_t seed, float lo, float hi);
void fill_uniform_at(float* p, int64_t n, uint64_t seed, int64_t first, float lo, float hi);
// GraphSAGE dual GEMM with ReLU + row L2 normalisation fused, one block per 64 rows x
// all N columns (k_sage_gemm.hip; N in {256, 512, 768, 1024}); bit-identical to
// gemm_nt_h2 + normalize_rows. Opt-in: RVX_SAGE_FUSED=1 (read per call).
bool sage_gemm_fused_ok(int64_t M, int N, int K0, int K1, int64_t lda0, int64_t lda1, int64_t ldb0, int64_t ldb1,
                        int64_t plane0, int64_t plane1, int64_t ldc, const void* A0, const void* A1, const void* C);
void sage_gemm_fused(int64_t M, int N, const float* A0, int64_t lda0, int K0, const float* A1, int64_t lda1, int K1,
                     const _Float16* B0h, int64_t ldb0, int64_t plane0, const _Float16* B1h, int64_t ldb1,
                     int64_t plane1, const float* a_scale, const float* b_inv, float* C, int64_t ldc, bool normalize,
                     const char* tag);
void fill_normal(float* p, int64_t n, uint64_t seed);
// *out_dev = sum over the 8-byte words of p of a position-keyed 64-bit mix (mod 2^64)
void checksum(const void* p, int64_t bytes, uint64_t* out_dev);
void fill_ball_rows(float* p, int64_t rows, int dim, uint64_t seed, int64_t first_row, float rmax);
void normalize_rows(float* p, int64_t rows, int dim, bool divide_only_if_positive, const char* tag);
void random_csr(int64_t n, int deg, uint64_t seed, int64_t* row_ptr, int32_t* col);
void random_csr_shard(int64_t n_total, int64_t row_begin, int64_t n_rows, int deg, uint64_t seed, int64_t* row_ptr,
                      int32_t* col);
void transpose(const float* in, int64_t rows, int64_t cols, float* out);  // out[c][r] = in[r][c]

// ---- gather / aggregate (k_aggregate.hip) -------------------------------
enum { AGG_SUM = 0, AGG_MEAN = 1, AGG_MAX = 2 };
// out[i] = agg over CSR row i of (w_e * x[col_e]) ; empty row -> `empty_fill`
// (0 = zeros, 1 = copy x[i], 2 = -inf for max). post_scale: 0 none, 1 = ×1/sqrt(deg) (GCN).
// row_scale (optional): also writes, per row, the power-of-two scale putting
// max(|out row|, |self row|) in [2^14, 2^15) for the split-f16 GEMM, where
// self = self_x + row*dim.
void aggregate_rows(const int64_t* row_ptr, const int32_t* col, const float* w, int64_t n, const float* x,
                    int dim, int agg, int empty_fill, int post_scale, float* out, const char* tag,
                    bool overlapped = false,  // true: runs beside a GEMM (capped grid)
                    const float* self_x = nullptr, float* row_scale = nullptr,
                    // with row_scale: write [aggregate | self] * row_scale as f16 planes
                    // [2][n][2*dim] (plane stride plane_stride) instead of out
                    _Float16* planes = nullptr, int64_t plane_stride = 0,
                    // deferred normalisation of x: gathered row c is x[c] * row_mul[c], the
                    // self row i (for row_scale) self_x[i] * self_mul[i]
                    const float* row_mul = nullptr, const float* self_mul = nullptr);
// The overlapped gather in its dynamic form (AggHelp; same rows, same bits as aggregate_rows
// overlapped with row_scale): agg_help_ok says whether the settings allow it (vector path,
// dim <= 768 so the helping GEMM keeps its register budget, the overlapped kernel's U = 8 NT
// loads, RVX_SAGE_HELP != 0).
bool agg_help_ok(int dim, const float* x, const float* out, const float* self_x);
// blocks_per_cu > 0 overrides the overlapped cap (RVX_AGG_BLOCKS_PER_CU): the first chunk of a
// layer has no GEMM beside it
void aggregate_rows_help(const AggHelp& h, const char* tag, int blocks_per_cu = 0);

}  // namespace rvx
