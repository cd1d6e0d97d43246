/*
 * twotower_hip.h -- C ABI of libtwotower_hip.so, the MI355X (gfx950) hot path of the
 * two-tower retrieval stack.
 *
 * The reference (HeikalPro/two-tower-model-v2) has no FFI of its own: its hot path is
 * Python that calls third-party numerics (faiss-cpu IndexFlatIP, sentence-transformers,
 * torch).  Every entry point below replaces one of those numeric calls; the reference
 * interface each replaces is cited (file:line under the reference root).  The Python
 * mirror of the reference classes (two-tower-model-v2_amd/twotower/) binds these with
 * ctypes; INTEGRATION.md shows the binding a maintainer of the reference would add.
 *
 * Conventions
 *   - All pointers are DEVICE pointers (hipMalloc / torch CUDA tensors), caller-owned,
 *     row-major, float32 unless stated.  `ld_*` = leading dimension (elements per row).
 *   - Every call is asynchronous on `stream` (a hipStream_t passed as void*); no call
 *     allocates device memory or synchronises.  Scratch comes from a caller workspace
 *     whose size is queried first.
 *   - Return value: TT_OK (0) or a negative TT_ERR_* code; tt_last_error() returns a
 *     thread-local message for the last failing call on the calling thread.
 *   - Numerics: every kernel follows a CANONICAL float32 evaluation order that the CPU
 *     oracle (oracle/tt_oracle.c) restates, so GPU and oracle agree bit-for-bit where
 *     the doc says "bit-exact".  See DESIGN.md "Canonical numerics".
 */
#ifndef TWOTOWER_HIP_H
#define TWOTOWER_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TT_OK 0
#define TT_ERR_INVALID (-1)     /* bad argument (shape, k, null pointer)              */
#define TT_ERR_LAUNCH (-2)      /* HIP launch / runtime error                         */
#define TT_ERR_UNSUPPORTED (-3) /* configuration outside what the kernels implement   */
#define TT_ERR_WORKSPACE (-4)   /* workspace too small                                */

#define TT_NORM_ADD_EPS 0 /* x / (||x|| + 1e-8)      vector_db.py:44-45,152-153,189-190 */
#define TT_NORM_MAX_EPS 1 /* x / max(||x||, 1e-12)   F.normalize: item_tower.py:209,
                                                     buyer_tower.py:66,99                */

/* Library version (major*10000 + minor*100 + patch) and last error (thread-local). */
int tt_version(void);
const char* tt_last_error(void);

/* ---------------------------------------------------------------------------------
 * Row L2 normalisation.  ||x|| is numpy's np.linalg.norm(axis=1) on float32, i.e.
 * sqrtf(pairwise_sum(x*x)) with numpy's 8-way-unrolled pairwise tree (bit-exact).
 *   mode TT_NORM_ADD_EPS replaces  VectorDatabase.build_index  src/inference/vector_db.py:43-45
 *                        and the query re-normalisation in retrieve / retrieve_batch
 *                        vector_db.py:151-153, 188-190.
 *   mode TT_NORM_MAX_EPS replaces  F.normalize(p=2, dim=1)  src/models/item_tower.py:209,
 *                        src/models/buyer_tower.py:66,99.
 * Also writes an optional bf16 copy (y_bf16 may be NULL; ld = ld_y).  In-place (x == y) is allowed.
 * --------------------------------------------------------------------------------- */
int tt_l2norm_rows_f32(const float* x, int64_t n, int32_t d, int64_t ld_x, float* y,
                       int64_t ld_y, uint16_t* y_bf16, int32_t mode, void* stream);

/* ---------------------------------------------------------------------------------
 * Exact inner-product top-k over a row-major catalog shard.
 * Replaces faiss.IndexFlatIP.search  (src/inference/vector_db.py:160 retrieve,
 * vector_db.py:197 retrieve_batch).  Scores are float32 dot products evaluated in the
 * canonical fma order (bit-exact vs the oracle); results sorted by score descending,
 * ties broken by LOWER global row (row_base + local row).  NaN scores are never
 * returned; if fewer than k finite scores exist the tail is (-inf, -1).
 *   db       [n, ld_db]  normalised catalog shard (ld_db >= d, multiple of 4, and the
 *                        padding columns d..ld_db-1 must be zero)
 *   q        [nq, ld_q]  normalised queries (ld_q >= d; same zero padding)
 *   out_*    [nq, k]     k <= n is the caller's job (reference clamps, vector_db.py:159,196)
 * workspace: size from tt_scan_workspace_bytes (same n, d, nq, k).
 * --------------------------------------------------------------------------------- */
int32_t tt_padded_dim(int32_t d); /* row length the scan reads: 64,128,256,384,512,768; -1 if d > 768 */
int tt_scan_workspace_bytes(int64_t n, int32_t d, int32_t nq, int32_t k, int64_t* bytes);
int tt_scan_topk_f32(const float* db, int64_t n, int32_t d, int64_t ld_db, int64_t row_base,
                     const float* q, int32_t nq, int64_t ld_q, int32_t k, float* out_score,
                     int64_t* out_idx, void* workspace, int64_t workspace_bytes,
                     void* stream);

/* Same as tt_scan_topk_f32, and records ev_start / ev_stop (hipEvent_t, may be NULL) on
 * `stream` immediately around the scan kernel (not the slab merge), so a benchmark can time
 * the dominant kernel alone. */
int tt_scan_topk_f32_timed(const float* db, int64_t n, int32_t d, int64_t ld_db,
                           int64_t row_base, const float* q, int32_t nq, int64_t ld_q, int32_t k,
                           float* out_score, int64_t* out_idx, void* workspace,
                           int64_t workspace_bytes, void* stream, void* ev_start,
                           void* ev_stop);

/* Exact scan of the queries listed on the device: slots 0 .. *qsel_n-1 read query qsel[slot]
 * and write row qsel[slot] of out_*.  Blocks beyond *qsel_n exit at once, so it can be
 * enqueued unconditionally as the fallback of tt_scan_topk_bf16f32 (no host sync). */
int tt_scan_topk_f32_select(const float* db, int64_t n, int32_t d, int64_t ld_db,
                            int64_t row_base, const float* q, int32_t nq, int64_t ld_q,
                            int32_t k, const int32_t* qsel, const int32_t* qsel_n,
                            float* out_score, int64_t* out_idx, void* workspace,
                            int64_t workspace_bytes, void* stream);

/* Same results as tt_scan_topk_f32 (bit-identical scores and order) for any 1 <= k <= 1024,
 * by scores-then-select: every canonical f32 score is written once (the scan's scoring loop)
 * and each query's k-th largest (score, ~row) key is found by a radix select over its score
 * row, then the k keys above it are sorted.  The large-k path (faiss.IndexFlatIP.search with
 * k up to 1000: server.py:46, vector_db.py:160,196): the scan's per-slab top-k lists cost
 * ~24-29 ms per search at k = 1000 over 1M rows.  Workspace: tt_select_workspace_bytes (the
 * score rows of up to 64 queries at a time: 256 MB at 1M rows). */
int tt_select_workspace_bytes(int64_t n, int32_t nq, int32_t k, int64_t* bytes);
int tt_scan_topk_select_f32(const float* db, int64_t n, int32_t d, int64_t ld_db,
                            int64_t row_base, const float* q, int32_t nq, int64_t ld_q,
                            int32_t k, float* out_score, int64_t* out_idx, void* workspace,
                            int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------
 * Same results as tt_scan_topk_f32 (bit-identical: canonical f32 scores, same order), found
 * through a bf16 MFMA filter over db_bf16 (the bf16 image of db, e.g. from tt_l2norm_rows_f32)
 * followed by an exact f32 re-rank of the candidates whose bf16 score lies within 2*eps_q of
 * the bf16 k-th best.  eps_q bounds |bf16 score - f32 score| for query q over every row; it
 * is derived on the device from x_norm_max >= max_r ||x_r|| and
 * x_resid_max >= max_r ||x_r - db_bf16_r|| (both from tt_bf16_image_bounds; larger values
 * stay exact but filter less).  Queries whose candidate lists overflow, or whose optimistic
 * sample threshold fails, are re-scanned exactly in a fallback launch.
 * k <= 128 (larger k: tt_scan_topk_f32).  Workspace: tt_filter_workspace_bytes.
 * ev_start/ev_stop (may be NULL) are recorded around the full-catalog filter kernel (the
 * dominant kernel; the sample levels, selection and re-rank are outside the bracket).
 * --------------------------------------------------------------------------------- */
int tt_filter_workspace_bytes(int64_t n, int32_t d, int32_t nq, int32_t k, int64_t* bytes);
/* Byte offset (in the workspace) of the int32 count of queries the last call served through
 * the exact fallback -- a diagnostic, read after the stream is synchronised. */
int tt_filter_fallback_offset(int64_t n, int32_t d, int32_t nq, int32_t k, int64_t* offset);
int tt_scan_topk_bf16f32(const float* db, const uint16_t* db_bf16, int64_t n, int32_t d,
                         int64_t ld_db, int64_t row_base, const float* q, int32_t nq,
                         int64_t ld_q, int32_t k, float x_norm_max, float x_resid_max,
                         float* out_score, int64_t* out_idx,
                         void* workspace, int64_t workspace_bytes, void* stream,
                         void* ev_start, void* ev_stop);
/* tt_scan_topk_bf16f32 for a catalog that also holds its int8 image (tt_i8_image; db_i8 may be
 * NULL): a large batch (> 2048 queries) at padded dim 384 runs its first, sampled level on the
 * int8 image (half the bytes, twice the MFMA rate).  That level only places the full level's
 * threshold, which the exact re-rank certifies, so the results are the same bits. */
int tt_scan_topk_bf16f32_i8s(const float* db, const uint16_t* db_bf16, const int8_t* db_i8,
                             const float* tile_scales, int64_t n, int32_t d, int64_t ld_db,
                             int64_t ld_i8, int64_t row_base, const float* q, int32_t nq,
                             int64_t ld_q, int32_t k, float x_norm_max, float x_resid_max,
                             float* out_score, int64_t* out_idx, void* workspace,
                             int64_t workspace_bytes, void* stream, void* ev_start,
                             void* ev_stop);

/* ---------------------------------------------------------------------------------
 * Same results as tt_scan_topk_f32 for the one-buyer serving call (nq <= 8, padded dim 384
 * or 768, k <= 128; src/api/server.py:241-244 -> vector_db.py:160 retrieve): one streaming pass
 * over an INT8 image of the catalog (tt_i8_image: half the bytes of the bf16 image), a
 * per-(query, slab) top-16 on v_mfma_i32_16x16x64_i8 with the exact f32 scores of the kept
 * rows, and a final that certifies the exact top k with a rigorous bound (a slab's dropped rows
 * score at most its 16th approximate score + eps, eps from x_norm_max, x_resid_max, s_max = the
 * image's bounds).  Uncertified queries take the exact f32 fallback in a following launch.
 * Workspace: tt_filter_workspace_bytes (same n, d, nq, k).  Returns TT_ERR_UNSUPPORTED outside
 * that shape (callers then use tt_scan_topk_bf16f32); tt_i8_single_pass_ok(n, d, nq, k, ld_i8)
 * answers 1 / 0 for a shape without a launch (the limits: nq <= 8, k <= 128, rows per CU
 * <= 65536 -- about 16.7M rows on 256 CUs -- and at most 256 CUs).
 * tt_debug_i8_force_unsupported(1) makes both report "unsupported" (test hook; 0 clears).
 * --------------------------------------------------------------------------------- */
int tt_i8_single_pass_ok(int64_t n, int32_t d, int32_t nq, int32_t k, int64_t ld_i8);
int tt_debug_i8_force_unsupported(int32_t on);
int tt_scan_topk_i8f32(const float* db, const int8_t* db_i8, const float* tile_scales,
                       int64_t n, int32_t d, int64_t ld_db, int64_t ld_i8, int64_t row_base,
                       const float* q, int32_t nq, int64_t ld_q, int32_t k, float x_norm_max,
                       float x_resid_max, float s_max, float* out_score, int64_t* out_idx,
                       void* workspace, int64_t workspace_bytes, void* stream, void* ev_start,
                       void* ev_stop);
/* The same search over the TILED int8 image (tt_i8_tile; padded dim 384 only), for nq <= 32:
 * each of a block's 8 waves streams its own 16-row blocks straight into MFMA operands (1 KB
 * contiguous per load instruction, no LDS staging, no block barrier), 9-32 queries as two
 * 16-query MFMA blocks per row block.  Same results bit for bit as tt_scan_topk_i8f32 and
 * tt_scan_topk_f32; same workspace (tt_filter_workspace_bytes), certification and fallback;
 * TT_ERR_UNSUPPORTED outside the shape tt_i8t_single_pass_ok(n, d, nq, k) accepts (callers
 * then take tt_scan_topk_i8f32 or tt_scan_topk_bf16f32). */
int tt_i8t_single_pass_ok(int64_t n, int32_t d, int32_t nq, int32_t k);
int tt_scan_topk_i8t_f32(const float* db, const int8_t* db_i8t, const float* tile_scales,
                         int64_t n, int32_t d, int64_t ld_db, int64_t row_base, const float* q,
                         int32_t nq, int64_t ld_q, int32_t k, float x_norm_max,
                         float x_resid_max, float s_max, float* out_score, int64_t* out_idx,
                         void* workspace, int64_t workspace_bytes, void* stream, void* ev_start,
                         void* ev_stop);

/* ---------------------------------------------------------------------------------
 * Row-sharded (multi-GPU) form of tt_scan_topk_bf16f32 (faiss IndexFlatIP.search,
 * vector_db.py:160,197, over a catalog split by rows across ranks).
 * Every rank holds its shard [row_base, row_base + n) in f32 and bf16, plus the GLOBAL
 * stride-TT_SHARD_SAMPLE_STRIDE sample of the bf16 image (rows 0, 16, 32, ... of the whole
 * catalog; 1/16 of a shard-set, built once with the index).  Per batch:
 *   1. tt_sharded_filter_begin (rank-local queries only, on the global sample):
 *      stats[q] = {theta_q, smax_q} = {a_J, max a} of the sample -- the threshold the
 *      single-catalog call derives, and the top of the probe range.
 *      -> caller: all-gather queries and stats (row order = query order)
 *   2. tt_sharded_filter_full (all W*B queries, on the shard):  bf16 filter with
 *      theta_q - 2 eps_q; probe_counts[q][i] = #shard rows with a >= t_i,
 *      t_i = theta_q + i (smax_q - theta_q) / TT_SHARD_PROBES.
 *      -> caller: all-reduce SUM of probe_counts [nq][TT_SHARD_PROBES] int32
 *   3. tt_sharded_filter_finish: a query with < k rows over all shards above theta_q takes the
 *      exact scan on every rank (identical decision everywhere); the rest re-rank the shard
 *      rows with a >= t* - 2 eps_q, t* = highest probe holding >= k rows (t* <= A_k).
 *      out = this shard's part of the global top-k (padded (-inf, -1)), merged across ranks
 *      with tt_topk_merge_f32 -- bit-identical to one search over the whole catalog.
 * x_norm_max / x_resid_max must bound the WHOLE catalog (all-reduce MAX of the shards'
 * tt_bf16_image_bounds).  Workspaces: begin -> tt_filter_workspace_bytes(n_sample, d, B, k);
 * full + finish (same buffer, kept between the calls) -> tt_sharded_workspace_bytes.
 * --------------------------------------------------------------------------------- */
#define TT_SHARD_PROBES 16
#define TT_SHARD_SAMPLE_STRIDE 16
int tt_sharded_workspace_bytes(int64_t n, int32_t d, int32_t nq, int32_t k, int64_t* bytes);
/* byte offset in the full/finish workspace of the int32 count of queries that took the
 * exact fallback on this shard (diagnostic) */
int tt_sharded_fallback_offset(int64_t n, int32_t d, int32_t nq, int32_t k, int64_t* offset);
/* Diagnostic (tests): byte offsets in a filter workspace of the band keys ([nq][offsets[4]]
 * uint64 (orderable score << 32 | ~row)), the band counts [nq] int32, the per-query fallback
 * flags [nq] int32 and the fallback count int32 (offsets[0..3]); offsets[4] = the band capacity
 * per query.  sharded = 0: tt_scan_topk_bf16f32's workspace; 1: the full/finish workspace. */
int tt_filter_workspace_layout(int64_t n, int32_t d, int32_t nq, int32_t k, int32_t sharded,
                               int64_t* offsets);
/* Test hook (fault injection for the bounds checks of decoded candidate rows): the NEXT
 * tt_scan_topk_bf16f32 call on this host thread corrupts query `query`'s best candidate key
 * on the device so that its row decodes to 0xffffffff -- where = 1: a band key between the
 * full level's selection and k_rerank (the large-batch path); where = 2: an exact key between
 * k_filter_topm and k_final_topm (the nq <= 4 single pass).  The kernels must then never read
 * that row and flag the query for the exact fallback.  where = 0 clears.  One-shot. */
int tt_debug_plant_bad_row(int32_t where, int32_t query);
/* 1 if this thread's last tt_scan_topk_bf16f32[_i8s] call ran its sample level on the int8
 * image (k_sample_i8), else 0 -- a test diagnostic. */
int tt_debug_last_sample_i8(void);
int tt_sharded_filter_begin(const uint16_t* sample_bf16, int64_t n_sample, int32_t d, int64_t ld,
                            const float* q, int32_t nq, int64_t ld_q, int32_t k, float* stats,
                            void* workspace, int64_t workspace_bytes, void* stream);
int tt_sharded_filter_full(const uint16_t* db_bf16, int64_t n, int32_t d, int64_t ld_db,
                           const float* q, int32_t nq, int64_t ld_q, int32_t k,
                           float x_norm_max, float x_resid_max, const float* stats,
                           int32_t* probe_counts, void* workspace, int64_t workspace_bytes,
                           void* stream, void* ev_start, void* ev_stop);
int tt_sharded_filter_finish(const float* db, const uint16_t* db_bf16, int64_t n, int32_t d,
                             int64_t ld_db, int64_t row_base, const float* q, int32_t nq,
                             int64_t ld_q, int32_t k, const float* stats,
                             const int32_t* probe_counts, float* out_score, int64_t* out_idx,
                             void* workspace, int64_t workspace_bytes, void* stream);

/* Bounds of a catalog shard and its bf16 image for tt_scan_topk_bf16f32: max-combines
 * (atomically, so successive add() batches accumulate; the caller zero-fills out2 once)
 * out2[0] >= max_r ||x_r|| and out2[1] >= max_r ||x_r - x_bf16_r||  (out2: 2 device floats).
 * NaN rows are skipped. */
/* The int8 image of a normalised catalog for tt_scan_topk_i8f32: per 64-row tile one scale
 * s = max |x| / 127 (tile_scales[ceil(n / 64)]), codes rint(x / s) in [-127, 127] into
 * codes [n, ld_codes] int8 (padding columns zero); out3 (device, 3 floats, max-combined like
 * tt_bf16_image_bounds; zero it first) >= (max ||x_r||, max ||x_r - s n_r||, max s ||n_r||). */
int tt_i8_image(const float* x, int64_t n, int32_t d, int64_t ld, int8_t* codes,
                int64_t ld_codes, float* tile_scales, float* out3, void* stream);
int tt_bf16_image_bounds(const float* x, const uint16_t* x_bf16, int64_t n, int32_t d,
                         int64_t ld, float* out2, void* stream);
/* The tiled int8 image for tt_scan_topk_i8t_f32, from tt_i8_image's codes [n, ld_codes]:
 * per 16-row block b, E / 64 pieces of 1 KB (E = tt_padded_dim(d)); piece s holds, at byte
 * 16 l (l = 16 g + col), row 16 b + col's codes 64 s + 16 g .. + 15 (rows past n zero).
 * tt_i8_tiled_bytes(n, d) = ceil(n / 16) * 16 * E (-1 when E % 64 != 0).  Buffers 16-B
 * aligned, ld_codes a multiple of 16.  The tile scales and bounds stay tt_i8_image's. */
int64_t tt_i8_tiled_bytes(int64_t n, int32_t d);
int tt_i8_tile(const int8_t* codes, int64_t ld_codes, int64_t n, int32_t d, int8_t* tiled,
               void* stream);

/* Merge n_lists per-shard top-k lists [n_lists, nq, k_in] (each sorted, global row ids)
 * into [nq, k]; same ordering rule.  Used after the RCCL all-gather of per-shard top-k
 * (multi-GPU row sharding). */
int tt_topk_merge_f32(const float* in_score, const int64_t* in_idx, int32_t n_lists,
                      int32_t nq, int32_t k_in, int32_t k, float* out_score,
                      int64_t* out_idx, void* stream);

/* ---------------------------------------------------------------------------------
 * Buyer tower.
 * tt_weighted_avg_l2_f32   replaces BuyerTower.weighted_average  src/models/buyer_tower.py:43-68
 *   items [b, s, d], w [b, s] -> out [b, ld_out]:  w/(sum w + 1e-8), sum_s x*w, F.normalize.
 * tt_gather_weighted_avg_l2_f32  same, with the history rows gathered from a resident
 *   item-embedding table by index (Mode B of EmbeddingEncoder.encode_buyer,
 *   src/inference/encoder.py:286-303): hist [b, s] int64 row ids into table [n_table, ld_table];
 *   an id < 0 marks padding (weight must be 0 there).
 * tt_attn_agg_l2_f32       replaces BuyerTower.attention_aggregation buyer_tower.py:70-101:
 *   a = W2.relu(W1.x + b1) + b2 ; softmax_s(a*w) ; sum_s alpha*x ; F.normalize.
 *   W1 [h, d] (nn.Linear weight layout), b1 [h], W2 [h] (Linear(h,1).weight), b2 [1].
 * --------------------------------------------------------------------------------- */
int tt_weighted_avg_l2_f32(const float* items, int64_t b, int32_t s, int32_t d,
                           const float* w, float* out, int64_t ld_out, void* stream);
int tt_gather_weighted_avg_l2_f32(const float* table, int64_t n_table, int64_t ld_table,
                                  int32_t d, const int64_t* hist, const float* w,
                                  int64_t b, int32_t s, float* out, int64_t ld_out,
                                  void* stream);
int tt_attn_agg_l2_f32(const float* items, int64_t b, int32_t s, int32_t d, const float* w,
                       const float* W1, const float* b1, int32_t h, const float* W2,
                       const float* b2, float* out, int64_t ld_out, void* stream);
/* Same results within 1e-6 (the first MLP layer's dot products in the f32 MFMA order instead of
 * a sequential chain) for batches: H = relu(x W1^T + b1) by tt_gemm_f32 into the workspace
 * (tt_attn_agg_workspace_bytes: b*s*h floats), then the per-buyer softmax / sum / F.normalize.
 * d % 32 != 0: runs tt_attn_agg_l2_f32 (no workspace used). */
int tt_attn_agg_workspace_bytes(int64_t b, int32_t s, int32_t h, int64_t* bytes);
int tt_attn_agg_l2_f32_ws(const float* items, int64_t b, int32_t s, int32_t d, const float* w,
                          const float* W1, const float* b1, int32_t h, const float* W2,
                          const float* b2, float* out, int64_t ld_out, void* workspace,
                          int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------
 * Item tower (tt_encoder.hip).
 *
 * The text encoder of ItemTower.encode_text (src/models/item_tower.py:100-124, which calls
 * SentenceTransformer("paraphrase-multilingual-MiniLM-L12-v2").encode: BertModel + mean
 * pooling, normalize_embeddings=False) over PACKED token sequences: ids[T] holds the n_seq
 * sequences back to back, cu_seqlens[n_seq+1] their offsets (every length >= 1, <= max_len).
 * Weights follow the Hugging Face BertModel state dict (nn.Linear [out, in] layout); Q, K, V
 * are concatenated row-wise into wqkv [3H, H] / bqkv [3H].  prec TT_PREC_F32 runs every GEMM
 * on v_mfma_f32_16x16x4_f32 (the parity path); TT_PREC_BF16 runs them on
 * v_mfma_f32_16x16x32_bf16 with f32 accumulation, f32 residual stream, LayerNorm, softmax and
 * pooling (the *_bf16 weight copies must be set); TT_PREC_X3 keeps the f32 path's operands and
 * splits them on the fly into bf16 hi + lo, each product as three bf16 MFMAs (hi.hi + lo.hi +
 * hi.lo, f32 accumulate: ~2^-16 relative per product instead of bf16's 2^-8) -- the f32 path's
 * precision class at bf16 MFMA rates.  out_pooled [n_seq, ld_out] f32.
 * --------------------------------------------------------------------------------- */
#define TT_PREC_F32 0
#define TT_PREC_BF16 1
#define TT_PREC_X3 2
#define TT_ACT_NONE 0
#define TT_ACT_GELU 1 /* exact erf GELU (hidden_act="gelu") */
#define TT_ACT_RELU 2

typedef struct tt_bert_layer {
  const float *wqkv, *bqkv;   /* [3H, H], [3H]   attention.self.{query,key,value} */
  const float *wo, *bo;       /* [H, H], [H]     attention.output.dense          */
  const float *ln1_g, *ln1_b; /* [H]             attention.output.LayerNorm      */
  const float *w1, *b1;       /* [I, H], [I]     intermediate.dense              */
  const float *w2, *b2;       /* [H, I], [H]     output.dense                    */
  const float *ln2_g, *ln2_b; /* [H]             output.LayerNorm                */
  const uint16_t *wqkv_bf16, *wo_bf16, *w1_bf16, *w2_bf16; /* bf16 images (TT_PREC_BF16) */
  /* TT_PREC_X3, optional: pre-split images [N, 2K] (tt_x3_split_weights); NULL -> the f32
   * weights are split on the fly */
  const uint16_t *wqkv_x3, *wo_x3, *w1_x3, *w2_x3;
  /* TT_PREC_X3 at H == 384 (head dim 32, I % 64 == 0), optional: x3i images W' [N, 2K] bf16
   * (tt_x3i_weights: per 32 k, 32 hi = bf16(W) then 32 lo = bf16(W - hi)).  When all four are
   * set the encoder takes the x3i form: every GEMM runs on the bf16 MFMA kernels with both
   * operands x3i interleaved -- per 32 k the three products hi.hi + lo.hi + hi.lo of
   * TT_PREC_X3, no split in the GEMM loop -- and every producer (embedding LayerNorm,
   * attention, the fused GEMM + LayerNorm, the QKV / FFN1 epilogues) writes its activation
   * x3i interleaved. */
  const uint16_t *wqkv_x3i, *wo_x3i, *w1_x3i, *w2_x3i;
} tt_bert_layer;

typedef struct tt_bert_model {
  int32_t vocab, hidden, heads, intermediate, layers, max_positions;
  float ln_eps;
  const float* word_emb;  /* [vocab, H] embeddings.word_embeddings     */
  const float* pos_emb;   /* [max_positions, H]                       */
  const float* type_emb;  /* [>=1, H] token_type_embeddings (row 0)   */
  const float *emb_ln_g, *emb_ln_b;
  const tt_bert_layer* layer; /* HOST array [layers] of device pointers */
} tt_bert_model;

int tt_bert_workspace_bytes(int64_t T, int32_t H, int32_t I, int32_t prec, int64_t* bytes);
int tt_bert_encode(const tt_bert_model* model, const int32_t* ids, const int32_t* cu_seqlens,
                   int32_t n_seq, int64_t T, int32_t max_len, int32_t prec, float* out_pooled,
                   int64_t ld_out, void* workspace, int64_t workspace_bytes, void* stream);

/* Building blocks of tt_bert_encode and of the projection head (ItemTower.projection,
 * item_tower.py:58-63: Linear -> ReLU -> Dropout(eval) -> Linear; then tt_l2norm_rows_f32
 * with TT_NORM_MAX_EPS for F.normalize, :209).
 * tt_gemm_*: C[M,N] = act(A[M,K] . W[N,K]^T + bias) + residual, f32 out (+ optional bf16
 *   copy C_bf16); K % 32 (f32) / K % 64 (bf16) == 0, any M, N; bias/residual may be NULL. */
int tt_gemm_f32(const float* A, int64_t lda, const float* W, int64_t ldw, const float* bias,
                const float* residual, int64_t ldr, float* C, int64_t ldc, uint16_t* C_bf16,
                int64_t ldc16, int32_t M, int32_t N, int32_t K, int32_t act, void* stream);
/* tt_gemm_x3: tt_gemm_f32's contract with the products on split-bf16 MFMA (TT_PREC_X3) */
int tt_gemm_x3(const float* A, int64_t lda, const float* W, int64_t ldw, const float* bias,
                const float* residual, int64_t ldr, float* C, int64_t ldc, uint16_t* C_bf16,
                int64_t ldc16, int32_t M, int32_t N, int32_t K, int32_t act, void* stream);
/* tt_x3_split_weights: W [N, K] f32 -> out [N, 2K] bf16, per 32-k block 32 hi then 32 lo in
 * the x3 GEMM's lane-slot order (K % 32 == 0).  tt_gemm_x3w: tt_gemm_x3 with W given as that
 * pre-split image (ld_wx3 in bf16 elements): the weights' split is done once, not per tile. */
int tt_x3_split_weights(const float* W, int64_t ldw, int32_t N, int32_t K, uint16_t* out,
                        int64_t ld_out, void* stream);
int tt_gemm_x3w(const float* A, int64_t lda, const uint16_t* Wx3, int64_t ld_wx3,
                const float* bias, const float* residual, int64_t ldr, float* C, int64_t ldc,
                uint16_t* C_bf16, int64_t ldc16, int32_t M, int32_t N, int32_t K, int32_t act,
                void* stream);
/* Split-bf16 interleaved rows ("x3i"): an f32 row v of length K (K % 32 == 0) as 2K bf16,
 * per 32 elements first hi = bf16(v) (round to nearest even) then lo = bf16(v - hi).
 * tt_x3i_weights: W [N, K] f32 -> out [N, 2K] x3i.  tt_gemm_x3i: the x3 product
 * act(A . W^T + bias) with A2 [M, 2K] and W2 [N, 2K] x3i rows (acc = A_hi.W_hi + A_hi.W_lo +
 * A_lo.W_hi on bf16 MFMA, f32 accumulation), written as x3i rows C2 [M, 2N] (N % 32 == 0).
 * tt_gemm_ln_x3i: tt_gemm_ln_bf16 in that form (A2 [M, 2K], W2 [384, 2K]) writing x f32 and
 * its x3i rows x2 [M, 768].  tt_attention_varlen_x3i: the encoder's attention over x3i QKV
 * rows qkv2 [T, >= 6H] (a head's Q / K / V = 32-blocks h / heads + h / 2 heads + h), every
 * product as three bf16 MFMAs, f32 softmax; context out2 [T, >= 2H] x3i (16-B aligned rows,
 * ld_out2 % 8 == 0).  Head dim 32. */
int tt_x3i_weights(const float* W, int64_t ldw, int32_t N, int32_t K, uint16_t* out,
                   int64_t ld_out, void* stream);
int tt_gemm_x3i(const uint16_t* A2, int64_t lda2, const uint16_t* W2, int64_t ldw2,
                const float* bias, uint16_t* C2, int64_t ldc2, int32_t M, int32_t N, int32_t K,
                int32_t act, void* stream);
int tt_gemm_ln_x3i(const uint16_t* A2, int64_t lda2, const uint16_t* W2, int64_t ldw2,
                   const float* bias, const float* gamma, const float* beta, float eps, float* x,
                   int64_t ldx, uint16_t* x2, int64_t ldx2, int32_t M, int32_t H, int32_t K,
                   void* stream);
int tt_attention_varlen_x3i(const uint16_t* qkv2, int64_t ld_qkv2, const int32_t* cu_seqlens,
                            int32_t n_seq, int32_t max_len, int32_t H, int32_t heads,
                            uint16_t* out2, int64_t ld_out2, void* stream);
int tt_gemm_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw,
                 const float* bias, const float* residual, int64_t ldr, float* C, int64_t ldc,
                 uint16_t* C_bf16, int64_t ldc16, int32_t M, int32_t N, int32_t K, int32_t act,
                 void* stream);
/* Fused BertSelfOutput / BertOutput (transformers BertModel, the encoder behind
 * SentenceTransformer.encode, item_tower.py:116-122): x = LayerNorm(A[M,K] . W[H,K]^T + bias + x)
 * in place over rows of x [M,H] f32, plus the bf16 copy x_bf16.  bf16 A/W, f32 accumulate and
 * LayerNorm (biased variance, eps).  H == 384 and K % 64 == 0 (TT_ERR_UNSUPPORTED otherwise);
 * x, bias, gamma, beta 16-B aligned.  Used by tt_bert_encode's bf16 path. */
int tt_gemm_ln_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw,
                    const float* bias, const float* gamma, const float* beta, float eps, float* x,
                    int64_t ldx, uint16_t* x_bf16, int64_t ldx16, int32_t M, int32_t H, int32_t K,
                    void* stream);
/* torch.nn.LayerNorm over rows of width H <= 1024 (BertLayer LayerNorms). */
int tt_layernorm_f32(const float* x, int64_t ldx, const float* gamma, const float* beta,
                     float eps, float* y, int64_t ldy, uint16_t* y_bf16, int64_t ldy16,
                     int64_t rows, int32_t H, void* stream);
/* BertSelfAttention over packed sequences: qkv [T, 3H] -> out [T, H].
 * tt_attention_varlen: MFMA kernel, head dim 32, prec TT_PREC_F32 (f32 MFMA) or TT_PREC_BF16
 *   (bf16 K/Q/V/P operands, f32 accumulation and softmax).
 * tt_attention_varlen_f32: scalar f32 kernel, head dim 32 or 64 (reference restatement). */
int tt_attention_varlen(const float* qkv, int64_t ld_qkv, const int32_t* cu_seqlens,
                        int32_t n_seq, int32_t max_len, int32_t H, int32_t heads, int32_t prec,
                        float* out, int64_t ld_out, uint16_t* out_bf16, void* stream);
/* Same (bf16 operands) reading a bf16 qkv [T, 3H]; out and/or out_bf16 may be NULL. */
int tt_attention_varlen_bf16(const uint16_t* qkv, int64_t ld_qkv, const int32_t* cu_seqlens,
                             int32_t n_seq, int32_t max_len, int32_t H, int32_t heads,
                             float* out, int64_t ld_out, uint16_t* out_bf16, void* stream);
int tt_attention_varlen_f32(const float* qkv, int64_t ld_qkv, const int32_t* cu_seqlens,
                            int32_t n_seq, int32_t max_len, int32_t H, int32_t heads,
                            float* out, int64_t ld_out, uint16_t* out_bf16, void* stream);
/* ItemTower.forward concat (item_tower.py:126-172,198): [pooled | brand_table[brand_ids] |
 * cat_table[cat_ids]]; a NULL table/ids or an id < 0 gives zeros (missing lists). */
int tt_item_concat(const float* pooled, int64_t ld_pooled, int32_t Ht, const int32_t* brand_ids,
                   const float* brand_table, const int32_t* cat_ids, const float* cat_table,
                   int32_t C, int64_t b, float* out, int64_t ld_out, uint16_t* out_bf16,
                   void* stream);

/* ---------------------------------------------------------------------------------
 * InfoNCE loss with in-batch negatives (tt_loss.hip), forward and backward in one call.
 * Replaces InfoNCELoss.forward (src/training/losses.py:20-79) + its autograd backward.
 * b [B, E] (ldb), p [B, E] (ldp), n [B, N, E] (row stride ldn_row, item stride ldn_item),
 * N <= 64, E % 32 == 0 (f32) / % 64 == 0 (bf16).  loss: ONE device float (mean over rows).
 * grad_b [B, E], grad_p [B, E], grad_n [B, N, E] (contiguous) are d loss / d input; pass
 * NULL for all three to skip the backward.  prec selects f32 or bf16 MFMA for the three
 * B x B x E GEMMs (softmax and the rest in f32).  Workspace: tt_infonce_workspace_bytes.
 * --------------------------------------------------------------------------------- */
int tt_infonce_workspace_bytes(int32_t B, int32_t N, int32_t E, int32_t prec,
                               int32_t with_grads, int64_t* bytes);
int tt_infonce_f32(const float* b, int64_t ldb, const float* p, int64_t ldp, const float* n,
                   int64_t ldn_row, int64_t ldn_item, int32_t B, int32_t N, int32_t E,
                   float temperature, int32_t prec, float* loss, float* grad_b, float* grad_p,
                   float* grad_n, void* workspace, int64_t workspace_bytes, void* stream);

/* Round-to-nearest-even bf16 copy of an f32 matrix (GEMM operands of the bf16 paths). */
int tt_f32_to_bf16(const float* x, int64_t ldx, int32_t rows, int32_t cols, uint16_t* y,
                   int64_t ldy, void* stream);

/* ---------------------------------------------------------------------------------
 * Training-step pieces (tt_train.hip) for configs[4]: InfoNCE on the item-tower head and the
 * buyer-tower attention MLP (src/training/trainer.py:74-243; text encoder frozen,
 * item_tower.py:40-42), GEMMs via tt_gemm_*.
 * --------------------------------------------------------------------------------- */
/* F.normalize backward: dy = (dz - z (z.dz)) / ||y|| (||y|| > 1e-12), else dz / 1e-12. */
int tt_l2norm_backward_f32(const float* y, int64_t ldy, const float* z, int64_t ldz,
                           const float* dz, int64_t lddz, int64_t n, int32_t d, float* dy,
                           int64_t lddy, void* stream);
/* x [rows, cols] -> t [cols, ldt] (t[c][r] = x[r][c]; columns rows..ldt-1 zero). */
int tt_transpose_f32(const float* x, int64_t ldx, int32_t rows, int32_t cols, float* t,
                     int32_t ldt, void* stream);
/* out[c] (+)= sum_r x[r][c]  (bias gradients). */
int tt_col_sum_f32(const float* x, int64_t ldx, int64_t rows, int32_t cols, float* out,
                   int32_t accumulate, void* stream);
/* dh[i] = 0 where h[i] <= 0 (ReLU backward, in place). */
int tt_relu_backward_f32(float* dh, const float* h, int64_t n, void* stream);
/* nn.Dropout(p) of the item projection (item_tower.py:61; active in train mode,
 * trainer.py:167) with a caller-drawn keep mask: x[i] = keep[i] ? x[i]*scale : 0 in place,
 * scale = 1/(1-p).  Applied to the incoming gradient it is the backward. */
int tt_dropout_apply_f32(float* x, const uint8_t* keep, float scale, int64_t n, void* stream);
/* BuyerTower.attention_aggregation after H = relu(x W1^T + b1) (buyer_tower.py:85-99):
 * a = H.W2 + b2, c = a*w, alpha = softmax_S(c), o = sum alpha x, z = F.normalize(o).
 * H [B*S, Hd], x [B, S, E], w [B, S]; saves alpha [B, S], onorm [B]. S <= 128, E <= 1024. */
int tt_attn_pool_fwd_f32(const float* H, int32_t Hd, const float* W2, float b2, const float* w,
                         const float* x, int64_t B, int32_t S, int32_t E, float* alpha,
                         float* onorm, float* z, int64_t ldz, void* stream);
/* Its backward: dW2 [Hd], db2 [1], dH [B*S, Hd] (ReLU mask not applied); da_ws [B*S] scratch. */
int tt_attn_pool_bwd_f32(const float* dz, int64_t lddz, const float* z, int64_t ldz,
                         const float* onorm, const float* alpha, const float* w, const float* x,
                         int64_t B, int32_t S, int32_t E, const float* H, const float* W2,
                         int32_t Hd, float* dW2, float* db2, float* dH, float* da_ws,
                         void* stream);
/* nn.Embedding(padding_idx=0) backward: table_grad[ids[r]] += g[r] (ids <= 0 skipped). */
int tt_embedding_backward_f32(const float* g, int64_t ldg, const int32_t* ids, int64_t n,
                              int32_t C, float* table_grad, void* stream);
/* tt_attn_pool_fwd_f32 with the bias b2 read from device memory (a step captured in a HIP
 * graph replays without a host read of the parameter), plus a bf16 copy of z (may be NULL; ld
 * = ldz) for the bf16 InfoNCE GEMM. */
int tt_attn_pool_fwd_f32_dev(const float* H, int32_t Hd, const float* W2, const float* b2,
                             const float* w, const float* x, int64_t B, int32_t S, int32_t E,
                             float* alpha, float* onorm, float* z, int64_t ldz, uint16_t* z_bf16,
                             void* stream);
/* tt_attn_pool_bwd_f32 with the ReLU backward of H fused into dH (dH = 0 where H <= 0) and
 * dW2 / db2 from per-buyer parts summed in a fixed order by a second launch (deterministic, no
 * atomics, no memsets).  da_ws holds B*S + 64 + B*(Hd+1) floats (da, then the parts). */
int tt_attn_pool_bwd_relu_f32(const float* dz, int64_t lddz, const float* z, int64_t ldz,
                              const float* onorm, const float* alpha, const float* w,
                              const float* x, int64_t B, int32_t S, int32_t E, const float* H,
                              const float* W2, int32_t Hd, float* dW2, float* db2, float* dH,
                              float* da_ws, void* stream);
/* tt_attn_pool_bwd_relu_f32 without its second launch: the per-buyer dW2 / db2 parts stay in
 * da_ws (after the B*S da values, at a 64-float boundary) for tt_train_bwd_tail. */
int tt_attn_pool_bwd_relu_parts_f32(const float* dz, int64_t lddz, const float* z, int64_t ldz,
                                    const float* onorm, const float* alpha, const float* w,
                                    const float* x, int64_t B, int32_t S, int32_t E,
                                    const float* H, const float* W2, int32_t Hd, float* dH,
                                    float* da_ws, void* stream);
/* Weight gradients without transposed copies: C [N, K] = A^T B for row-major A [M, N] (dY),
 * B [M, K] (X), f32 in; prec TT_PREC_BF16 rounds the operands to bf16 (bf16 MFMA, f32
 * accumulate), TT_PREC_F32 keeps f32 (f32 MFMA).  db (may be NULL) = column sums of A (the bias
 * gradient, f32).  The rows are split over blocks (partial tiles in the workspace) and a
 * second launch sums the splits in a fixed order (deterministic).  Workspace:
 * tt_gemm_tn_workspace_bytes (0 when the rows are not split); one workspace may serve calls
 * of different shapes in stream order. */
int tt_gemm_tn_workspace_bytes(int64_t M, int32_t N, int32_t K, int64_t* bytes);
int tt_gemm_tn(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int32_t N,
               int32_t K, int32_t prec, float* C, int64_t ldc, float* db, void* workspace,
               int64_t workspace_bytes, void* stream);
/* tt_gemm_tn without its second launch: the split sums stay in `workspace` (which must not be
 * reused until they are reduced) and tt_gemm_tn_reduce_many sums up to 8 such GEMMs in ONE
 * launch, same order and bits as tt_gemm_tn.  A plan with one split writes C / db directly
 * (its job is then skipped).  The training step defers its weight-gradient reduces to one
 * launch and InfoNCE reduces its two products together. */
typedef struct tt_tn_pending {
  const void* workspace;  /* the workspace given to tt_gemm_tn_partial */
  int64_t M;
  int32_t N, K;
  float* C;
  int64_t ldc;
  float* db; /* may be NULL */
} tt_tn_pending;
int tt_gemm_tn_partial(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M,
                       int32_t N, int32_t K, int32_t prec, float* C, int64_t ldc, float* db,
                       void* workspace, int64_t workspace_bytes, void* stream);
int tt_gemm_tn_reduce_many(const tt_tn_pending* jobs, int32_t n, void* stream);
/* The training step's backward tail in ONE launch: the deferred weight-gradient reduces (as
 * tt_gemm_tn_reduce_many), the attention pooling's dW2 / db2 from the per-buyer parts that
 * tt_attn_pool_bwd_relu_parts_f32 left at attn_parts (same order and bits as
 * tt_attn_pool_bwd_relu_f32's second launch; attn_parts NULL: none), and the embedding-row
 * gradients of tt_embedding_backward2_f32 (g_emb NULL: none). */
int tt_train_bwd_tail(const tt_tn_pending* jobs, int32_t njobs, const float* attn_parts,
                      int64_t B, int32_t Hd, float* dW2, float* db2, const float* g_emb,
                      int64_t ldg, const int32_t* ids0, const int32_t* ids1, int64_t n_emb,
                      int32_t C, float* grad0, float* grad1, void* stream);
/* nn.Dropout forward with the keep mask drawn in the kernel: element i is kept iff
 * hash(seed, *counter, i) >= p 2^32 (splitmix64, counter-based: a graph-replayed step draws a
 * fresh mask when the caller advances *counter, a device int64), kept values scaled by
 * 1/(1-p); plus a bf16 copy (may be NULL).  No mask is stored (the backward is
 * tt_relu_dropout_backward_f32 on the post-dropout activation). */
int tt_dropout_rng_f32(float* x, int64_t n, float p, uint64_t seed, const int64_t* counter,
                       uint16_t* x_bf16, void* stream);
/* Both item-tower embedding tables' row gradients in one launch: grad0[ids0[r]] += g[r][0:C],
 * grad1[ids1[r]] += g[r][C:2C] (ids <= 0 skipped; a NULL id array skips its table). */
int tt_embedding_backward2_f32(const float* g, int64_t ldg, const int32_t* ids0,
                               const int32_t* ids1, int64_t n, int32_t C, float* grad0,
                               float* grad1, void* stream);
/* tt_infonce_f32 with the caller's bf16 copies of b and p (either may be NULL: converted
 * inside) for the prec = TT_PREC_BF16 logits GEMM. */
int tt_infonce_ex(const float* b, int64_t ldb, const float* p, int64_t ldp, const float* n,
                  int64_t ldn_row, int64_t ldn_item, int32_t B, int32_t N, int32_t E,
                  float temperature, int32_t prec, float* loss, float* grad_b, float* grad_p,
                  float* grad_n, void* workspace, int64_t workspace_bytes, const uint16_t* b_bf16,
                  int64_t ldb16, const uint16_t* p_bf16, int64_t ldp16, void* stream);
/* nn.Dropout forward with a keep mask (tt_dropout_apply_f32) plus a bf16 copy (may be NULL). */
int tt_dropout_apply_ex(float* x, const uint8_t* keep, float scale, int64_t n, uint16_t* x_bf16,
                        void* stream);
/* ReLU (+ Dropout) backward on the post-activation h: dh = h > 0 ? dh * scale : 0 (scale =
 * 1/(1-p) with dropout, 1 without), plus a bf16 copy (may be NULL).  counter_advance (may be
 * NULL): a tt_dropout_rng_f32 draw counter this launch increments by one (the step's last use
 * of the mask is its forward, so the next step draws a new one). */
int tt_relu_dropout_backward_f32(float* dh, const float* h, float scale, int64_t n,
                                 uint16_t* dh_bf16, int64_t* counter_advance, void* stream);
/* tt_l2norm_backward_f32 plus a bf16 copy of dy (may be NULL). */
int tt_l2norm_backward_ex(const float* y, int64_t ldy, const float* z, int64_t ldz,
                          const float* dz, int64_t lddz, int64_t n, int32_t d, float* dy,
                          int64_t lddy, uint16_t* dy_bf16, int64_t lddy16, void* stream);
/* Batched operand preparation, ONE launch: job j writes src [rows, cols] f32 to dst as f32 or
 * bf16 (to_bf16), transposed (dst [cols, ld_dst], columns rows..ld_dst-1 zero) or not; src
 * NULL zero-fills dst [rows, cols] (not transposed).  The training step's weight-derived GEMM
 * operands (bf16 weights, transposed weights), bf16 copies of its inputs and the zeroing of
 * its accumulated gradients, once per step.  row_ids (may be NULL; not with transpose): dst
 * row r takes src row row_ids[r], zeros for a negative id -- the [text | brand | cat]
 * concatenation of the item head's input as jobs of the same launch. */
#define TT_CONVERT_MAX_JOBS 16
typedef struct tt_convert_job {
  const float* src;
  int64_t ld_src;
  int32_t rows, cols;
  void* dst;
  int64_t ld_dst;
  int32_t transpose, to_bf16;
  const int32_t* row_ids;
} tt_convert_job;
int tt_convert_batch(const tt_convert_job* jobs, int32_t njobs, void* stream);
/* torch.optim.Adam step (weight_decay 0): step is the 1-based step count after increment. */
int tt_adam_f32(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                float beta2, float eps, int32_t step, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* TWOTOWER_HIP_H */
