/*
 * gnnrec.h — C ABI of the MI355X-native propagation hot path (libgnnrec.so).
 *
 * The reference (timur1arkhipov/gnn-recommendations) is pure Python and has no FFI:
 * its hot path is the PyTorch call `torch.sparse.mm(adj_matrix, x)` inside the model
 * classes. Each entry point below replaces one such op call site (or a fused chain of
 * them); the citations name the reference lines (paths relative to
 * gnn-recommendations/). The Python host layer (gnn-recommendations_amd/src/ops/_lib.py)
 * binds these with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions (all entry points):
 *   - Device pointers are owned by the caller (PyTorch caching allocator); nothing is
 *     allocated, freed or synchronised inside a compute call, so every call is legal
 *     inside hipGraph capture. Work is queued on `stream` (NULL = legacy default stream).
 *   - Return 0 (GNNREC_OK) on success or a negative gnnrec_status; the message of the
 *     last failure on the calling thread is returned by gnnrec_last_error().
 *   - No C++ exception crosses the ABI. All functions are reentrant.
 *   - Graph operand = CSR over destination rows: `row_ptr[n_rows+1]` (int64, absolute
 *     offsets into col/val, row_ptr[0] need not be 0), `col[]` (int32, ascending within
 *     each row), `val[]` (fp32). Ascending columns are what makes the SpMM bit-exact with
 *     the reference's COO `torch.sparse.mm` (per-row sequential fmaf, col order).
 *   - Dense tables are fp32 row-major with an explicit leading dimension in ELEMENTS.
 */
#ifndef GNNREC_H_
#define GNNREC_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GNNREC_ABI_VERSION 11

typedef struct ihipStream_t* gnnrec_stream_t;

enum gnnrec_status {
  GNNREC_OK = 0,
  GNNREC_EINVAL = -1,       /* bad argument (null pointer, bad size, unsupported d) */
  GNNREC_EHIP = -2,         /* a HIP runtime call failed (launch error) */
  GNNREC_EUNSUPPORTED = -3  /* combination not implemented */
};

/* Epilogue flags of gnnrec_spmm_csr_f32 (bit set). They fuse the LightGCN layer mean
 * `torch.stack(all_embeddings).mean(0)` (baselines/lightgcn.py:94-95) into the hop:
 *   ACC_INIT: acc[r] = self[r] + y[r]          (first hop: x0 + x1)
 *   ACC_ADD : acc[r] = acc[r] + y[r]           (later hops, sequential like torch.mean)
 *   ACC_DIV : then acc[r] = acc[r] / acc_div   (last hop: / (K+1))
 *   NO_Y    : do not store y (last hop when the layer output itself is not needed)
 * gnnrec_spmm_tiled_f32 only (ABI 6; the CSR entry points return GNNREC_EUNSUPPORTED):
 *   ACC_INIT|ACC_ADD: acc[r] = (self[r] + acc[r]) + y[r]   (an earlier layer parked in acc)
 *   ACC_X   : the previous layer's row prev[r] (default: the hop's input row x[r], square
 *             operand; a sharded caller passes its own rows of the layer) is added after the
 *             self/acc terms and before y[r]: acc[r] = ((self[r] [+ acc[r]]) + prev[r]) + y[r]
 *   With them the layer mean is formed once, on the last hop, from the parked layers
 *   (hops 1..K-1 store y only): same additions in the same order, so the same bits. */
#define GNNREC_EPI_ACC_INIT 1
#define GNNREC_EPI_ACC_ADD 2
#define GNNREC_EPI_ACC_DIV 4
#define GNNREC_EPI_NO_Y 8
#define GNNREC_EPI_ACC_X 16

/* ---- library identity ------------------------------------------------------------ */
const char* gnnrec_version(void);
int gnnrec_abi_version(void);
const char* gnnrec_last_error(void);

/* ---- a4: normalised-adjacency SpMM -------------------------------------------------
 * Replaces torch.sparse.mm(adj_matrix, x) at baselines/lightgcn.py:88,178,
 * baselines/ngcf.py:70, orthogonal_bundle/model.py:172,184,333,344, baselines/kgtore.py:310.
 *   y[r, :] = sum_k val[k] * x[col[k], :]   for k in row r, ascending k, starting at +0.0f,
 *   each term applied with fmaf (bit-exact with the reference CPU path).
 * `self`/`acc` are only read/written when an ACC_* flag is set (see above); `self` is the
 * input-table row of destination r (x0 for LightGCN's first hop).
 * Any d >= 1 is accepted; d in {8,16,32,64,128,256} take the vectorised fast path. */
int gnnrec_spmm_csr_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                        int64_t n_rows, const float* x, int64_t ldx, float* y, int64_t ldy,
                        int32_t d, int32_t epi, const float* self, int64_t ld_self,
                        float* acc, int64_t ld_acc, float acc_div, gnnrec_stream_t stream);

/* ---- a5: whole LightGCN propagation (K hops + fused layer mean) ----------------------
 * Replaces the body of LightGCN.forward (baselines/lightgcn.py:76-95) on one device:
 *   out = (((x0 + A x0) + A^2 x0) + ... + A^K x0) / (K+1)
 * work0/work1: two [n_rows, d] scratch tables (ping-pong hop outputs); `layers`, if not
 * NULL, receives the K hop outputs x1..xK as K consecutive [n_rows, ld_out] tables
 * (get_layer_embeddings, lightgcn.py:153-183) and then work0/work1 may be NULL.
 * Requires a square operand (n_rows == rows of x0). */
int gnnrec_lightgcn_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                        int64_t n_rows, const float* x0, int32_t d, int32_t n_layers,
                        float* work0, float* work1, float* layers, float* out, int64_t ld_out,
                        gnnrec_stream_t stream);

/* Heavy-row split of the two calls above (same results, bit for bit). Rows with more than
 * heavy_threshold neighbours are skipped by the row-parallel kernel and run instead one
 * workgroup per row (512 threads, 136 KB LDS): the whole workgroup gathers the next 64 KB of
 * neighbour rows into an LDS double buffer while one wave runs the row's ordered fmaf chain.
 * heavy_rows (device int64 [n_heavy]) must list exactly the rows longer than heavy_threshold;
 * heavy_threshold == 0 disables the split. Needs d % 4 == 0, 16 <= d <= 256, 16-B aligned x with
 * ldx % 4 == 0 when enabled. Power-law operands (popular items) stop being latency-bound on
 * their longest rows. */
int gnnrec_spmm_csr_split_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                              int64_t n_rows, const float* x, int64_t ldx, float* y, int64_t ldy,
                              int32_t d, int32_t epi, const float* self, int64_t ld_self,
                              float* acc, int64_t ld_acc, float acc_div,
                              const int64_t* heavy_rows, int64_t n_heavy,
                              int64_t heavy_threshold, gnnrec_stream_t stream);

int gnnrec_lightgcn_split_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                              int64_t n_rows, const float* x0, int32_t d, int32_t n_layers,
                              float* work0, float* work1, float* layers, float* out,
                              int64_t ld_out, const int64_t* heavy_rows, int64_t n_heavy,
                              int64_t heavy_threshold, gnnrec_stream_t stream);

/* Sparse-input / row-subset hop: gnnrec_spmm_csr_split_f32 where x_nonzero (device uint8
 * [rows of x], may be NULL) marks the rows of x that hold any non-zero, and y_active (uint8
 * [n_rows], may be NULL) the destination rows to compute. The row-parallel kernel does not
 * gather unmarked x rows (their terms are fmaf(v, +-0, acc) == acc from +0: same bits) and
 * does not walk inactive rows: their y is written as +0 (or, for heavy rows and the any-d
 * path, the true value) and the epilogue applied to it. Two uses:
 *  - backward: the BPR gradient touches a few thousand of 2M rows, so y_active = rows with a
 *    non-zero neighbour (gnnrec_mark_active_rows) loses nothing and skips almost everything;
 *  - training forward: the loss reads a few thousand output rows, so the last hops need only
 *    those rows and their neighbourhoods (the values of the other rows are then not defined).
 * gnnrec_row_nonzero_f32 builds x_nonzero; gnnrec_mark_active_rows sets y_active[c] = 1 for
 * every c listed in a marked row of (row_ptr_t, col_t) and 0 elsewhere — given the operand's
 * transpose it marks the rows a non-zero input row reaches, given the operand itself the
 * inputs the marked rows read (the same thing when the operand is symmetric). */
int gnnrec_spmm_csr_masked_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                               int64_t n_rows, const float* x, int64_t ldx,
                               const uint8_t* x_nonzero, const uint8_t* y_active, float* y,
                               int64_t ldy, int32_t d,
                               int32_t epi, const float* self, int64_t ld_self, float* acc,
                               int64_t ld_acc, float acc_div, const int64_t* heavy_rows,
                               int64_t n_heavy, int64_t heavy_threshold, gnnrec_stream_t stream);

/* The CSR hop with its heavy rows tuned (ABI 11): gnnrec_spmm_csr_masked_f32 /
 * gnnrec_lightgcn_split_f32 plus
 *  - n_sliced: the first n_sliced entries of heavy_rows (which must then be sorted longest
 *    first, as every caller in this package lists them) run as feature slices, one workgroup
 *    each (d = 32: 2 x 16 features; d = 64: 4 x 16 on operands of at most 65536 rows, else
 *    2 x 32; d = 128: 4 x 32; d = 256: 4 x 64; ignored for other d): each gathers its slice of
 *    every neighbour row, so the longest chains finish in fewer LDS rounds. Same bits.
 *  - flags: GNNREC_CSR_FORK runs the heavy-row kernel on an internal high-priority side
 *    stream forked from and joined back into `stream` with events (capture-safe), so the
 *    row-parallel rows run beside the heavy chains instead of after them (the two write
 *    disjoint rows; measured slower than one stream on config 2, so off by default; the
 *    caller's stream must belong to the current device). GNNREC_CSR_LIGHT_LATENCY /
 *    _THROUGHPUT force the row-parallel chain's form (default: the latency form — the next
 *    step's indices loaded one step ahead — for operands of at most 65536 rows, whose rows
 *    cannot fill the chip; see csrc/gather.h). On such operands (d = 32 / 64 / 128, no
 *    x_nonzero / y_active, latency form) the row-parallel rows run as extra workgroups of
 *    the heavy-row launch, dispatched after the heavy ones: one launch per hop.
 *    GNNREC_CSR_TWO_LAUNCHES keeps them a launch of their own, before the heavy rows.
 * Replaces the same torch.sparse.mm calls (lightgcn.py:88, ngcf.py:70). */
#define GNNREC_CSR_FORK 1
#define GNNREC_CSR_LIGHT_LATENCY 2
#define GNNREC_CSR_LIGHT_THROUGHPUT 4
#define GNNREC_CSR_TWO_LAUNCHES 8
int gnnrec_spmm_csr_heavy_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                              int64_t n_rows, const float* x, int64_t ldx,
                              const uint8_t* x_nonzero, const uint8_t* y_active, float* y,
                              int64_t ldy, int32_t d, int32_t epi, const float* self,
                              int64_t ld_self, float* acc, int64_t ld_acc, float acc_div,
                              const int64_t* heavy_rows, int64_t n_heavy, int64_t heavy_threshold,
                              int64_t n_sliced, int32_t flags, gnnrec_stream_t stream);
int gnnrec_lightgcn_heavy_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                              int64_t n_rows, const float* x0, int32_t d, int32_t n_layers,
                              float* work0, float* work1, float* layers, float* out,
                              int64_t ld_out, const int64_t* heavy_rows, int64_t n_heavy,
                              int64_t heavy_threshold, int64_t n_sliced, int32_t flags,
                              gnnrec_stream_t stream);

/* Column-ordered ("tiled") hop, the same y and epilogue bits as gnnrec_spmm_csr_f32 for any
 * d that is a multiple of 32. A persistent workgroup per CU owns
 * `rows_per_block` destination rows per pass with their accumulators in LDS and walks their
 * edges panel by panel in ascending source-column order (a step = one panel of `panel`
 * columns; steps are separated by a workgroup barrier; the workgroups of a blockIdx%8 group
 * start each pass together), so the rows of an XCD gather each source row while it is in that
 * XCD's L2. The features are done in 32-wide slices (one 128-B cache line of a source row per
 * gather), one slice per pass of a block, so a 160 KB LDS holds 1279 rows' accumulators. A
 * wave runs GNNREC_TILED_GROUPS slot streams, one per 8-lane group (16 B of the line per
 * lane). Every row is still +0 then one fmaf per neighbour in ascending column order:
 * bit-exact.
 *
 * The operand is re-laid out once on the host from the CSR (gnnrec_tiled_plan_build, then
 * gnnrec_tiled_plan_emit into caller buffers, then gnnrec_tiled_plan_free); the plan depends
 * on neither d nor the x table's stride. Per (block, wave) the plan is a run of chunks; a
 * chunk is GNNREC_TILED_STEPS steps x GNNREC_TILED_GROUPS streams = GNNREC_TILED_CHUNK slots,
 * entry 8 g + t = slot t of stream g (ABI 7; ABI 6 had two 16-slot halves); a slot is one
 * uint32 word ((col - panel base) << 11 | local row; row rows_per_block = a padding slot) and
 * one fp32 value; per chunk hdr[4] = {step barriers before the chunk, chain mask bits 0-31,
 * bits 32-63 (bit 8 g + t = slot t of stream g continues slot t-1's row), panel base column
 * (every slot of a chunk lies in one panel of at most 2^20 columns)}. Inside a stream a row
 * appears in each group of 4 slots (steps 0-3, 4-7 of a chunk) as at most one run of
 * consecutive slots. Slot arrays hold (n_chunks + GNNREC_TILED_TAIL) * GNNREC_TILED_CHUNK
 * entries, hdr 4 * (n_chunks + GNNREC_TILED_TAIL) (tail chunks read by the last prefetches);
 * wave_ptr [n_blocks * GNNREC_TILED_WAVES + 1] are chunk offsets; n_steps [n_blocks].
 * rows_per_block <= GNNREC_TILED_MAX_ROWS. gnnrec_spmm_tiled_f32 needs d % 32 == 0,
 * d <= ldx <= GNNREC_TILED_MAX_LDX (any table size), every table 16-B aligned with its
 * leading dimension a multiple of 4, `sync`: a device scratch of GNNREC_TILED_SYNC_WORDS
 * uint32 (zeroed per call), and meet_us: the bound of the pass-start meeting in microseconds
 * (0: no meeting — e.g. when other kernels share the device). */
#ifndef GNNREC_TILED_WAVES   /* experiment builds may override it (plan and kernel together) */
#define GNNREC_TILED_WAVES 8
#endif
#define GNNREC_TILED_GROUPS 8
#define GNNREC_TILED_STEPS 8
#define GNNREC_TILED_CHUNK 64
#define GNNREC_TILED_TAIL 8
#define GNNREC_TILED_QUAD_TAIL 16   /* tail chunks of the quad layout (prefetch 11 chunks ahead) */
#define GNNREC_TILED_MAX_ROWS 1279
#define GNNREC_TILED_SYNC_WORDS 256
/* sync[GNNREC_TILED_SYNC_ERR_WORD] != 0 after a gnnrec_spmm_tiled_f32 launch: the plan's wave
 * ranges were not quad-aligned (chunk-major arrays passed to a quad-layout build, see
 * gnnrec_tiled_plan_quad); the launch's output rows (y, acc) are then UNDEFINED: a flagged wave
 * skips its chunks, but every block still runs its epilogue. The launch zeroes the word. */
#define GNNREC_TILED_SYNC_ERR_WORD 1
#define GNNREC_TILED_HDR_WORDS 4
#define GNNREC_TILED_MAX_LDX 1024
#define GNNREC_TILED_MAX_CLASSES 256
#define GNNREC_TILED_MAX_ROWS_FACTORED 1232

int gnnrec_tiled_plan_build(const int64_t* row_ptr, const int32_t* col, const float* val,
                            int64_t n_rows, int32_t rows_per_block, int32_t panel,
                            int32_t sub_panel, int32_t n_threads, void** plan,
                            int64_t* n_chunks, int64_t* n_blocks);
int gnnrec_tiled_plan_emit(void* plan, uint32_t* slot, float* val, uint32_t* hdr,
                           int64_t* wave_ptr, int32_t* n_steps);
int gnnrec_tiled_plan_free(void* plan);

/* The same plan built on the device from a device-resident CSR (bit-identical arrays).
 * Two calls on `stream`: the COUNT pass (wave_ptr == NULL) writes chunks[n_blocks *
 * GNNREC_TILED_WAVES] (chunks per block and wave) and n_steps[n_blocks]; the caller forms
 * wave_ptr = [0, cumsum(chunks)] and sizes slot / val_out / hdr for wave_ptr[last] +
 * GNNREC_TILED_TAIL chunks; the EMIT pass (wave_ptr != NULL) writes them, tail chunks
 * included. scratch: gnnrec_tiled_plan_device_scratch_words(max_block_nnz, workgroups)
 * uint64 words where max_block_nnz bounds the edges of one step of a block (always safe:
 * the largest row_ptr[min(n_rows, (b+1) R)] - row_ptr[b R]; a smaller bound that a step
 * exceeds fails the pass with error 2, to be retried with a larger one); err: one device
 * int32, zeroed by the caller, non-zero after a failed pass (1 negative column, 2 scratch
 * too small, 3 a run — one row's slots in one step — longer than 32 767, 4 count / emit
 * mismatch). */
int64_t gnnrec_tiled_plan_device_scratch_words(int64_t max_block_nnz, int32_t workgroups);
/* Row statistics of a device CSR (ABI 11), written to the device int64 out[2]: out[0] = the
 * longest row, out[1] = the most edges in any block of block_rows consecutive rows (the
 * planner's max_block_nnz; 0 when block_rows <= 0). One single-workgroup kernel. */
int gnnrec_csr_row_stats(const int64_t* row_ptr, int64_t n_rows, int64_t block_rows, int64_t* out,
                         gnnrec_stream_t stream);
int gnnrec_tiled_plan_device(const int64_t* row_ptr, const int32_t* col, const float* val,
                             int64_t n_rows, int32_t rows_per_block, int32_t panel,
                             int32_t sub_panel, int64_t max_block_nnz, uint64_t* scratch,
                             int32_t workgroups, int64_t* chunks, int32_t* n_steps,
                             const int64_t* wave_ptr, uint32_t* slot, float* val_out,
                             uint32_t* hdr, int32_t* err, gnnrec_stream_t stream);

/* 1 when `device` grants gnnrec_spmm_tiled_f32 the dynamic LDS of `rows_per_block` rows
 * ((rows_per_block + 1) * 128 B; the attribute is set once per device), else 0 — a caller
 * then keeps the row-parallel hop (gnnrec_spmm_csr_masked_f32). */
int gnnrec_spmm_tiled_supported(int32_t device, int32_t rows_per_block);

/* The plan layout gnnrec_spmm_tiled_f32 of this build reads (ABI 9): 1 = quad-interleaved
 * (the default): the planners' chunk-major arrays (gnnrec_tiled_plan_emit /
 * gnnrec_tiled_plan_device, factored by gnnrec_tiled_plan_factor) go through
 * gnnrec_tiled_plan_quad_offsets + gnnrec_tiled_plan_quad_layout first; 0 = chunk-major
 * (GNNREC_TILED_QUAD=0 builds read the planner arrays directly). */
int gnnrec_tiled_plan_quad(void);

/* Quad layout, step 1 (device, async): wave_ptr_out[n_waves + 1] = the exclusive scan of each
 * wave's chunk count (wave_ptr[s+1] - wave_ptr[s]) rounded up to a multiple of 4. The caller
 * reads total_chunks = wave_ptr_out[n_waves] and allocates the step-2 outputs for
 * total_chunks + GNNREC_TILED_QUAD_TAIL chunks. */
int gnnrec_tiled_plan_quad_offsets(const int64_t* wave_ptr, int64_t n_waves, int64_t* wave_ptr_out,
                                   gnnrec_stream_t stream);

/* Quad layout, step 2 (device, async): every wave's chunks at the start of its padded range,
 * empty chunks after them and in the GNNREC_TILED_QUAD_TAIL tail chunks (slot word =
 * rows_per_block: column offset 0, the scratch row; class 0 / value 0; header 0); then the
 * slot words and the class bytes (slot_class != NULL, a factored plan) or the values of
 * chunks 4q .. 4q+3 as [q][lane][4]; headers stay [chunk][4]. */
int gnnrec_tiled_plan_quad_layout(const int64_t* wave_ptr, const int64_t* wave_ptr_out,
                                  int64_t n_waves, int64_t total_chunks, int32_t rows_per_block,
                                  const uint32_t* slot, const float* val,
                                  const uint8_t* slot_class, const uint32_t* hdr,
                                  uint32_t* slot_out, float* val_out, uint8_t* class_out,
                                  uint32_t* hdr_out, gnnrec_stream_t stream);

/* Factored plans (ABI 8): when every value of the operand is fl(row_factor[r] *
 * class_table[k]) for a class k of its column (the symmetric normalisation fl(dis_r * dis_c)
 * of graph_builder.py:119-126 when the column degrees take at most GNNREC_TILED_MAX_CLASSES
 * distinct values), a slot carries the 1-byte class instead of its 4-byte value: 5.25 instead
 * of 8.25 plan bytes per slot, the value formed in the kernel as the same fp32 product (same
 * bits). gnnrec_tiled_plan_factor derives slot_class [(n_chunks + TAIL) * CHUNK, zeroed by the
 * caller] from a plan and col_class [n_cols] and counts into *mismatches (a device uint32,
 * zeroed by the caller) every real slot whose value is not that product; with zero
 * mismatches gnnrec_spmm_tiled_f32 may take slot_class, row_factor [n_rows], class_table
 * [n_classes] and val = NULL (rows_per_block <= GNNREC_TILED_MAX_ROWS_FACTORED: the factors
 * share the LDS). slot_class = NULL: explicit values, the other three are ignored. */
int gnnrec_tiled_plan_factor(const uint32_t* slot, const float* val, const uint32_t* hdr,
                             const int64_t* wave_ptr, int64_t n_blocks, int32_t rows_per_block,
                             int64_t n_rows, int64_t n_cols, const float* row_factor,
                             const uint8_t* col_class, const float* class_table,
                             int32_t n_classes, uint8_t* slot_class, uint32_t* mismatches,
                             gnnrec_stream_t stream);

int gnnrec_spmm_tiled_f32(const uint32_t* slot, const float* val, const uint8_t* slot_class,
                          const float* row_factor, const float* class_table, int32_t n_classes,
                          const uint32_t* hdr,
                          const int64_t* wave_ptr, const int32_t* n_steps, int64_t n_blocks,
                          int32_t rows_per_block, const float* x, int64_t x_rows, int64_t ldx,
                          float* y, int64_t ldy, int64_t n_rows, int32_t d, int32_t epi,
                          const float* self, int64_t ld_self, float* acc, int64_t ld_acc,
                          float acc_div, const float* prev, int64_t ld_prev, uint32_t* sync,
                          int32_t meet_us, gnnrec_stream_t stream);

/* Hop with a row-sparse input (ABI 8): y = A^T x where x is zero outside the n_src rows
 * src_rows (ascending int64) — the training backward's first hop, whose input (the BPR
 * gradient, trainer.py:199-281 through lightgcn.py:88) touches the 3B rows of a batch. The
 * sources' rows of A (row_ptr/col/val: n_rows x n_cols, the forward operand) are scattered as
 * (output row, source) pairs, sorted, and every reached output row of y ([n_cols, ldy]) is one
 * fmaf chain from +0 over its sources in ascending order: the bits of the dense hop over A^T
 * (a left-out term is fmaf(v, 0, acc) = acc). Rows no source reaches are not written (zero y
 * first). max_pairs >= the sources' stored entries (exact count or a bound; a short bound
 * fails with GNNREC_EINVAL). Two calls: workspace == NULL returns its size in
 * *workspace_bytes; the second call synchronises `stream` once (the bound check). */
int gnnrec_spmm_sparse_src_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                               int64_t n_rows, int64_t n_cols, const int64_t* src_rows,
                               int64_t n_src, int64_t max_pairs, const float* x, int64_t ldx,
                               float* y, int64_t ldy, int32_t d, void* workspace,
                               size_t* workspace_bytes, gnnrec_stream_t stream);

int gnnrec_row_nonzero_f32(const float* x, int64_t ldx, int64_t n_rows, int32_t d,
                           uint8_t* mask, gnnrec_stream_t stream);

int gnnrec_mark_active_rows(const int64_t* row_ptr_t, const int32_t* col_t, int64_t n_src,
                            const uint8_t* x_nonzero, int64_t n_dst, uint8_t* y_active,
                            gnnrec_stream_t stream);

/* ---- a7: Group-and-Shuffle transform -----------------------------------------------
 * Replaces GroupShuffleLayer.forward (orthogonal_bundle/group_shuffle_layer.py:88-94):
 *   y = (x @ blockdiag(W_0..W_{d/bs-1}))[:, perm]
 *   y[r, j] = sum_{c<bs} x[r, bs*b + c] * W_b[c, e]   with perm[j] = bs*b + e.
 * blocks: [d/bs, bs, bs] row-major (W_b[c][e] = blocks[(b*bs + c)*bs + e]); perm: [d]. */
int gnnrec_gas_f32(const float* x, int64_t ldx, int64_t n_rows, int32_t d, int32_t bs,
                   const float* blocks, const int32_t* perm, float* y, int64_t ldy,
                   gnnrec_stream_t stream);

/* Fused hop + GAS: y = GAS(A x) (SpMM epilogue; one HBM round trip fewer). */
int gnnrec_spmm_gas_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                        int64_t n_rows, const float* x, int64_t ldx, float* y, int64_t ldy,
                        int32_t d, int32_t bs, const float* blocks, const int32_t* perm,
                        gnnrec_stream_t stream);

/* ---- a6: NGCF layer (SpMM + two 64x64 Linear on MFMA + LeakyReLU [+ GAS]) -----------
 * Replaces NGCFLayer.forward (baselines/ngcf.py:69-84) in eval mode (dropout = identity):
 *   n   = A x
 *   out = LeakyReLU_slope( (n @ W1^T + b1) + ((x_self * n) @ W2^T + b2) )
 * W1, W2: [d, d] in nn.Linear layout (out_features x in_features); b1, b2: [d].
 * x_self: the input-table rows of the destination rows ([n_rows, ld_self]).
 * If gas_blocks != NULL, GAS(gas_blocks, gas_perm, gas_bs) is applied to `out` before the
 * store (BASELINE config 3: x_{l+1} = GS_l(NGCFLayer_l(x_l))).
 * work: NULL = one fused kernel; else an [n_rows, d] scratch table (16-B aligned): the hop
 * runs as gnnrec_spmm_csr_f32 into it and a streaming MFMA kernel applies the rest (faster
 * on gather-bound graphs: the hop keeps its occupancy). Same results either way.
 * d must be 32, 64 or 128 (MFMA f32 16x16x4 tiles). */
int gnnrec_spmm_ngcf_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                         int64_t n_rows, const float* x, int64_t ldx, const float* x_self,
                         int64_t ld_self, float* y, int64_t ldy, int32_t d, const float* W1,
                         const float* b1, const float* W2, const float* b2, float slope,
                         const float* gas_blocks, const int32_t* gas_perm, int32_t gas_bs,
                         float* work, gnnrec_stream_t stream);

/* ---- a9: OrthogonalBundle layer (SpMM + composed 64x64 transform + residual) ---------
 * Replaces orthogonal_bundle/model.py:171-195 (adjacency path) plus the softmax-weighted
 * layer sum of model.py:204-207:
 *   out = c_out * ((A x) @ M) + c_res * resid
 * with M = W_conn @ W_gs[:, perm] composed on the host (d x d, row-major) and
 * c_out = 1 - alpha, c_res = alpha, resid = x_init rows of the destinations.
 * acc_mode 0: no layer sum; 1: acc = fl(w_res*resid) + fl(w_out*out) (layer 0 + layer 1);
 * 2: acc = acc + fl(w_out*out). `y` may be NULL when only acc is wanted; `resid` may be
 * NULL (no residual term, out = c_out * ((A x) @ M)) unless acc_mode is 1.
 * work: as gnnrec_spmm_ngcf_f32 (NULL = fused, else [n_rows, d] scratch for the split form).
 * d must be 32, 64 or 128. */
int gnnrec_spmm_dense_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                          int64_t n_rows, const float* x, int64_t ldx, float* y, int64_t ldy,
                          int32_t d, const float* M, float c_out, const float* resid,
                          int64_t ld_resid, float c_res, float* acc, int64_t ld_acc,
                          int32_t acc_mode, float w_out, float w_res, float* work,
                          gnnrec_stream_t stream);

/* Transform-only halves of the two calls above: `n` already holds A x (for instance from
 * gnnrec_spmm_csr_split_f32, whose heavy-row kernel keeps power-law operands fast); the
 * rest is applied exactly as in their split form. n: [n_rows, ldn]. */
int gnnrec_ngcf_transform_f32(int64_t n_rows, const float* n, int64_t ldn, const float* x_self,
                              int64_t ld_self, float* y, int64_t ldy, int32_t d, const float* W1,
                              const float* b1, const float* W2, const float* b2, float slope,
                              const float* gas_blocks, const int32_t* gas_perm, int32_t gas_bs,
                              gnnrec_stream_t stream);

int gnnrec_dense_transform_f32(int64_t n_rows, const float* n, int64_t ldn, float* y, int64_t ldy,
                               int32_t d, const float* M, float c_out, const float* resid,
                               int64_t ld_resid, float c_res, float* acc, int64_t ld_acc,
                               int32_t acc_mode, float w_out, float w_res, gnnrec_stream_t stream);

/* ---- a11: GAT sparse edge-softmax aggregation ---------------------------------------
 * Replaces the dense masked softmax + mm of GATLayer.forward (baselines/gat.py:99-149)
 * plus the F.elu between layers (gat.py:283) and the layer mean (gat.py:287-288):
 * for every head h and destination row r with neighbours j (CSR pattern; values ignored):
 *   e_j = LeakyReLU_slope(s_self[r, h] + s_neigh[j, h]);  a = softmax_j(e)
 *   o[r, h, :] = sum_j a_j * hfeat[j, h, :]
 * (single pass, online max/sum rescaling per block of 8 neighbours in base 2, fp32).
 * hfeat[j, h, :] starts at
 * hfeat + j*ldh + h*head_stride (ldh < 2^30: the kernels form a row's offset as one 32-bit x
 * 32-bit multiply of j and ldh*4): head_stride = o_dim for the head-major [N, heads*o_dim]
 * table of the per-head W_h x; head_stride = 0 lets every head aggregate the same row (the
 * layer input x, with W_h applied by the caller afterwards: sum_j a_j W_h x_j =
 * W_h sum_j a_j x_j — the head-averaged last layer then gathers o_dim instead of heads*o_dim
 * floats per neighbour). s_self / s_neigh: [N, heads] with row strides ld_ss / ld_sn
 * (>= heads; e.g. columns of the projection's [N, heads*o_dim + 2*heads] output in place).
 * mean_heads = 0: out[r] = cat_h o[r,h,:] ([n_rows, heads*o_dim]); 1: out[r] = mean_h
 * o[r,h,:] ([n_rows, o_dim]). apply_elu: out = ELU(out) (alpha 1). epi: the ACC_* flags of
 * gnnrec_spmm_csr_f32 applied to the (ELU'd) output with `self` = the layer input rows.
 * An empty row yields NaN (softmax over an empty set, as the reference's all -inf row).
 * heads*o_dim must be 16, 32, 64, 128 or 256 (o_dim a multiple of 4).
 * max_row_len > 0: rows with more neighbours are skipped here and must be finished by
 * gnnrec_gat_heavy_f32 (power-law degree buckets; 0 = every row here). */
int gnnrec_gat_aggregate_f32(const int64_t* row_ptr, const int32_t* col, int64_t n_rows,
                             const float* hfeat, int64_t ldh, int64_t head_stride,
                             const float* s_self, const float* s_neigh, int64_t ld_ss,
                             int64_t ld_sn, int32_t heads, int32_t o_dim, float slope,
                             int32_t mean_heads, int32_t apply_elu, float* out, int64_t ldo,
                             int32_t epi, const float* self, int64_t ld_self, float* acc,
                             int64_t ld_acc, float acc_div, int64_t max_row_len,
                             gnnrec_stream_t stream);

/* Heavy-row bucket of the GAT aggregation: every heavy row is cut into segments (seg_row /
 * seg_beg / seg_end: its row id and CSR range, n_seg in all; heavy_seg_ptr[n_heavy+1] the
 * segments of heavy_rows[h]); one row group per segment computes a partial (sum, max, total)
 * and a merge pass rescales and combines them, then applies the same epilogue as
 * gnnrec_gat_aggregate_f32. work: n_seg * (heads*o_dim + 2*heads) floats, 16-B aligned. */
int gnnrec_gat_heavy_f32(const int32_t* col, const int64_t* seg_row, const int64_t* seg_beg,
                         const int64_t* seg_end, int64_t n_seg, const int64_t* heavy_rows,
                         const int64_t* heavy_seg_ptr, int64_t n_heavy, float* work,
                         const float* hfeat, int64_t ldh, int64_t head_stride,
                         const float* s_self, const float* s_neigh, int64_t ld_ss,
                         int64_t ld_sn, int32_t heads, int32_t o_dim, float slope,
                         int32_t mean_heads, int32_t apply_elu,
                         float* out, int64_t ldo, int32_t epi, const float* self,
                         int64_t ld_self, float* acc, int64_t ld_acc, float acc_div,
                         gnnrec_stream_t stream);

/* Scores from the rows (ABI 10): the same aggregation and epilogue as gnnrec_gat_aggregate_f32 /
 * gnnrec_gat_heavy_f32, with the attention scores formed in the kernel from the rows it reads
 * instead of gathered from score tables (gat.py:113-118: s_self = h_r a_self, s_neigh = h_j
 * a_neigh, per head): att = [2][heads][o_dim] fp32 (att[0][h] = a_self of head h, att[1][h] =
 * a_neigh; for head_stride = 0 the row vectors W_h^T a_h acting on the shared row), and
 *   s_self[r, h]  = att[0][h] . hself[r, h, :]   (hself + r*ld_hself + h*head_stride)
 *   s_neigh[j, h] = att[1][h] . hfeat[j, h, :]   (the gathered row itself)
 * in fp32 (tolerance-level: the reference's torch.mm(h, a) summed in another order). A 256-B
 * gathered row then costs 2 instead of 3 random 128-B lines per neighbour. o_dim <= 64 and
 * o_dim / 4 a power of two; the shared-row fast path is heads = 4, o_dim = 64. */
int gnnrec_gat_aggregate_att_f32(const int64_t* row_ptr, const int32_t* col, int64_t n_rows,
                                 const float* hfeat, int64_t ldh, int64_t head_stride,
                                 const float* hself, int64_t ld_hself, const float* att,
                                 int32_t heads, int32_t o_dim, float slope, int32_t mean_heads,
                                 int32_t apply_elu, float* out, int64_t ldo, int32_t epi,
                                 const float* self, int64_t ld_self, float* acc, int64_t ld_acc,
                                 float acc_div, int64_t max_row_len, gnnrec_stream_t stream);

int gnnrec_gat_heavy_att_f32(const int32_t* col, const int64_t* seg_row, const int64_t* seg_beg,
                             const int64_t* seg_end, int64_t n_seg, const int64_t* heavy_rows,
                             const int64_t* heavy_seg_ptr, int64_t n_heavy, float* work,
                             const float* hfeat, int64_t ldh, int64_t head_stride,
                             const float* hself, int64_t ld_hself, const float* att,
                             int32_t heads, int32_t o_dim, float slope, int32_t mean_heads,
                             int32_t apply_elu, float* out, int64_t ldo, int32_t epi,
                             const float* self, int64_t ld_self, float* acc, int64_t ld_acc,
                             float acc_div, const int64_t* seg_pos, int32_t xcd_order,
                             gnnrec_stream_t stream);
/* gnnrec_gat_heavy_att_f32's segment order: seg_row / seg_beg / seg_end may list the segments
 * in any order (e.g. by their first column, so that segments of different heavy rows over the
 * same columns run at the same time and share gathered lines in L2); seg_pos[j] gives the
 * position of the j-th segment of heavy_seg_ptr's row-grouped numbering (NULL: the arrays are
 * row-grouped). xcd_order = 1: XCD x runs the x-th eighth of the segment list (blocks are
 * otherwise dealt round-robin to the 8 XCDs, spreading neighbouring segments over 8 L2s). */

/* ---- f1 for GAT: the training aggregation and its backward (csrc/gat_train.hip) ----------
 * Forward: out[r, q*o:(q+1)*o] = sum_j alpha_rjq keep_rjq / (1 - drop_p) hfeat[j, q*o:(q+1)*o]
 * with alpha = softmax over the row's neighbours of LeakyReLU_slope(s_self[r, q] +
 * s_neigh[j, q]) (gat.py:113-141) and keep a Bernoulli(1 - drop_p) draw of a counter-based hash
 * of (seed, r, j, q) — the reference's F.dropout on the attention weights, gat.py:137 —
 * regenerated (not stored) by the backward. hfeat: the head-major [N, heads*o_dim] table
 * (ldh), s_self / s_neigh: [N, heads] (row stride ld_s); out [n_rows, heads*o_dim] (ldo).
 * No epilogue (the caller's autograd applies head mean / ELU / layer mean); the _split
 * variants below cut long rows into segments.
 * Backward (two passes over the CSR; the pattern must be SYMMETRIC, as the normalised
 * bipartite adjacency is: row j lists the rows that aggregate j): given dout, writes
 * dh [n, heads*o_dim] (lddh), d_self and d_neigh [n, heads] (contiguous); stats is a scratch of
 * n_rows * heads * 4 floats (softmax max / sum / g.out per row and head). fp32, any order
 * (tolerance-level vs the reference's dense autograd). heads*o_dim in {16 .. 256}, o_dim / 4 a
 * power of two. */
int gnnrec_gat_train_forward_f32(const int64_t* row_ptr, const int32_t* col, int64_t n_rows,
                                 const float* hfeat, int64_t ldh, const float* s_self,
                                 const float* s_neigh, int64_t ld_s, int32_t heads, int32_t o_dim,
                                 float slope, float drop_p, uint32_t seed, float* out, int64_t ldo,
                                 gnnrec_stream_t stream);
int gnnrec_gat_train_backward_f32(const int64_t* row_ptr, const int32_t* col, int64_t n_rows,
                                  const float* hfeat, int64_t ldh, const float* s_self,
                                  const float* s_neigh, int64_t ld_s, int32_t heads, int32_t o_dim,
                                  float slope, float drop_p, uint32_t seed, const float* out,
                                  int64_t ldo, const float* dout, int64_t lddo, float* stats,
                                  float* dh, int64_t lddh, float* d_self, float* d_neigh,
                                  gnnrec_stream_t stream);
/* The same two calls with a heavy-row split (ABI 11; rows longer than max_row_len, e.g. the
 * 4e5-neighbour hubs of config 5, which one lane group would walk serially): the segment plan
 * of CsrGraph.heavy_plan (seg_row / seg_beg / seg_end [n_seg], heavy_rows [n_heavy] and
 * heavy_seg_ptr [n_heavy + 1], every heavy row's segments contiguous), a 16-B aligned work
 * buffer of n_seg * (heads * o_dim + 2 heads) floats. Each segment's partial sums are computed
 * by one lane group and merged per row in segment order (deterministic). The forward writes
 * the softmax statistics into stats (n_rows * heads * 4 floats: max, sum); the backward reads
 * them from there (no recount pass) — it must get the stats of the forward of the same inputs.
 * max_row_len == 0 or n_heavy == 0: no split. */
int gnnrec_gat_train_forward_split_f32(
    const int64_t* row_ptr, const int32_t* col, int64_t n_rows, const float* hfeat, int64_t ldh,
    const float* s_self, const float* s_neigh, int64_t ld_s, int32_t heads, int32_t o_dim,
    float slope, float drop_p, uint32_t seed, float* out, int64_t ldo, float* stats,
    int64_t max_row_len, const int64_t* seg_row, const int64_t* seg_beg, const int64_t* seg_end,
    int64_t n_seg, const int64_t* heavy_rows, const int64_t* heavy_seg_ptr, int64_t n_heavy,
    float* work, gnnrec_stream_t stream);
int gnnrec_gat_train_backward_split_f32(
    const int64_t* row_ptr, const int32_t* col, int64_t n_rows, const float* hfeat, int64_t ldh,
    const float* s_self, const float* s_neigh, int64_t ld_s, int32_t heads, int32_t o_dim,
    float slope, float drop_p, uint32_t seed, const float* out, int64_t ldo, const float* dout,
    int64_t lddo, float* stats, float* dh, int64_t lddh, float* d_self, float* d_neigh,
    int64_t max_row_len, const int64_t* seg_row, const int64_t* seg_beg, const int64_t* seg_end,
    int64_t n_seg, const int64_t* heavy_rows, const int64_t* heavy_seg_ptr, int64_t n_heavy,
    float* work, gnnrec_stream_t stream);

/* Dense projections of the GAT layer (gat.py:113-118 W_h x and the attention halves, one
 * fused weight; and the head-averaged last layer's W_h applied after the aggregation,
 * gat.py:149): y[r, :p] = x[r, :k] @ B[k, p], B row-major [k][p], on the matrix cores
 * (fp32 accumulate; the k order is a fixed permutation: an fp32-tolerance path). Replaces the
 * tall-skinny torch.matmul / hipBLASLt calls. Then, as gnnrec_gat_aggregate_f32's epilogue:
 * apply_elu: y = ELU(y); epi: the ACC_* flags (acc = (self or acc) + y [/ acc_div]). y may be
 * NULL when epi writes acc. k in {64, 128, 256}; p % 4 == 0; p <= 80 for k = 64, p <= 64
 * otherwise; x, y, self, acc rows 16-B aligned (ld % 4 == 0). */
int gnnrec_rows_gemm_f32(int64_t n_rows, const float* x, int64_t ldx, int32_t k, const float* B,
                         int32_t p, float* y, int64_t ldy, int32_t apply_elu, int32_t epi,
                         const float* self, int64_t ld_self, float* acc, int64_t ld_acc,
                         float acc_div, gnnrec_stream_t stream);

/* ---- a13: scoring + seen-item mask + top-K ------------------------------------------
 * Replaces evaluator.py:96-105 / trainer.py:327-336 for one batch of users:
 *   score[b, i] = sum_{f<d} u[b, f] * v[i, f]   (sequential fmaf over f, from +0.0f)
 *   score[b, i] = -inf for items i in the seen list of user b (CSR seen_ptr/seen_col)
 *   top-k by (score desc, item index asc) -> out_idx[b, :k] (int64), out_score[b, :k].
 * k <= 128; d in {16, 32, 64, 128, 256} (callers zero-pad other widths: exact). */
int gnnrec_score_topk_f32(const float* u, int64_t ldu, int64_t n_users_batch,
                          const float* v, int64_t ldv, int64_t n_items, int32_t d,
                          const int64_t* seen_ptr, const int32_t* seen_col, int32_t k,
                          int64_t* out_idx, float* out_score, gnnrec_stream_t stream);

/* Item-split form (same results, bit for bit): the catalogue is cut into n_split ranges
 * (grid.y), each range's exact top-k per user goes to work_idx/work_score
 * ([n_users_batch, n_split, k]), and a merge kernel ranks the n_split*k candidates of each
 * user into out_*. Small user batches (the reference evaluates 2048 users at a time) then
 * still fill the chip. n_split == 1 is gnnrec_score_topk_f32 (work buffers unused). */
int gnnrec_score_topk_split_f32(const float* u, int64_t ldu, int64_t n_users_batch,
                                const float* v, int64_t ldv, int64_t n_items, int32_t d,
                                const int64_t* seen_ptr, const int32_t* seen_col, int32_t k,
                                int32_t n_split, int64_t* work_idx, float* work_score,
                                int64_t* out_idx, float* out_score, gnnrec_stream_t stream);

/* ---- a1-a3: host-side operand construction (native, no GPU) -------------------------
 * build_bipartite_graph + normalize_adjacency_matrix (data/graph_builder.py:16-144):
 * CSR over N = n_users + n_items rows of A = [[0, R], [R^T, 0]] with columns ascending,
 * duplicate (user,item) pairs summed (coo -> csr semantics, graph_builder.py:107).
 * col/cnt must hold 2*n_pairs (+N with self_loop) entries; the number used is returned in
 * *nnz_out. Fills row_ptr[N+1], col[nnz], cnt[nnz] (edge multiplicity as float) and deg[N]
 * (float32 row sums, graph_builder.py:111). users/items must be in range (else EINVAL).
 * flags: GNNREC_BUILD_SELF_LOOP adds the identity (graph_builder.py:73-74);
 * GNNREC_BUILD_BINARY keeps duplicate pairs once with weight 1 (the deduplicated input
 * preprocessing.py:185-218 guarantees), instead of summing them. n_threads <= 0: all cores. */
#define GNNREC_BUILD_SELF_LOOP 1
#define GNNREC_BUILD_BINARY 2
int gnnrec_build_bipartite_csr(const int64_t* users, const int64_t* items, int64_t n_pairs,
                               int64_t n_users, int64_t n_items, int32_t flags,
                               int64_t* row_ptr, int32_t* col, float* cnt, float* deg,
                               int64_t* nnz_out, int32_t n_threads);

/* Symmetric normalisation values (graph_builder.py:116-126):
 *   val[k] = fl32(fl32(dis[r] * cnt[k]) * dis[col[k]])  with dis = deg^-1/2 computed by the
 * caller with numpy float32 power (graph_builder.py:119), bit-identical to scipy's
 * D^-1/2 @ A @ D^-1/2. mode 1 = 'row' normalisation: val = fl32(dis[r] * cnt[k]). */
int gnnrec_normalize_values(const int64_t* row_ptr, const int32_t* col, const float* cnt,
                            int64_t n_rows, const float* dis, int32_t mode, float* val,
                            int32_t n_threads);

/* ---- §8f3: on-device operand construction ----------------------------------------------
 * Same contract and output as gnnrec_build_bipartite_csr (graph_builder.py:16-111) with every
 * array in device memory: users/items int64 [n_pairs]; row_ptr int64 [N+1]; col int32 and
 * cnt fp32 with capacity 2*n_pairs (+N with GNNREC_BUILD_SELF_LOOP); deg fp32 [N]. Sort-based
 * (64-bit row|col keys, radix sort, run-length encode), so rows come out with ascending
 * columns and duplicate pairs merged exactly as the host builder does. *nnz_out is a HOST
 * pointer: the call synchronises `stream` before returning. Call first with
 * workspace == NULL to get *workspace_bytes (about 20 bytes per key, keys = 2*n_pairs (+N)),
 * then again with a device buffer of that size. Requires 2*n_pairs (+N) < 2^31 and degrees
 * below 2^24 (they are exact fp32 integers). */
int gnnrec_build_bipartite_csr_device(const int64_t* users, const int64_t* items,
                                      int64_t n_pairs, int64_t n_users, int64_t n_items,
                                      int32_t flags, int64_t* row_ptr, int32_t* col, float* cnt,
                                      float* deg, int64_t* nnz_out, void* workspace,
                                      size_t* workspace_bytes, gnnrec_stream_t stream);

/* Device form of gnnrec_normalize_values (graph_builder.py:116-126): same values, async. */
int gnnrec_normalize_values_device(const int64_t* row_ptr, const int32_t* col, const float* cnt,
                                   int64_t n_rows, const float* dis, int32_t mode, float* val,
                                   gnnrec_stream_t stream);

/* ---- §8f1: optimizer step of the training path ------------------------------------------
 * Replaces torch.optim.Adam.step (L2 weight decay, no amsgrad) that the reference trainer
 * runs after every batch (trainer.py:59-63, 271-272) for one fp32 parameter of n elements:
 * param, grad, exp_avg, exp_avg_sq device arrays, 16-B aligned. The caller keeps the step
 * count and passes step_size = lr / (1 - beta1^t) and bias_correction2_sqrt =
 * sqrt(1 - beta2^t) (computed in double, as torch does). grad_scale (device float, may be
 * NULL) multiplies the gradient first — clip_grad_norm_'s coefficient without a pass over
 * the gradient. The gradient is not modified. Async on `stream`. */
int gnnrec_adam_step_f32(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                         int64_t n, float step_size, double beta1, double beta2,
                         float bias_correction2_sqrt, float eps, float weight_decay,
                         const float* grad_scale, gnnrec_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* GNNREC_H_ */
