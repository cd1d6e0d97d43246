// tt_scan.hip -- fused inner-product scan + top-k over a catalog shard (gfx950).
//
// Replaces faiss.IndexFlatIP.search as called by VectorDatabase.retrieve
// (src/inference/vector_db.py:160) and retrieve_batch (vector_db.py:197).
//
// Structure (DESIGN.md "Scan"):
//   grid = (query tiles of 64) x (catalog slabs).  A 256-thread block = 4 waves; wave w
//   owns 16 queries whose float32 vectors live in VGPRs as v_mfma_f32_16x16x4_f32
//   B-fragments.  All 4 waves stream the SAME slab rows (one HBM read, three L1/L2 hits)
//   straight from HBM into A-fragments, 32 rows per step, and accumulate exact f32
//   scores with MFMA.  Lane-group g (= lane>>4) holds dims 16t+4g..16t+4g+3, so the MFMA
//   chain evaluates the canonical fma order (t, i, g) -> d = 16t+4g+i (tt_common.hpp).
//   Selection: per query a threshold theta (k-th best seen so far in this slab) and an
//   LDS candidate buffer; a score >= theta is appended; a full buffer is compacted by a
//   wave-wide bitonic sort (keep top k, raise theta).  At the end of the slab each
//   query's sorted top-k goes to the workspace; k_merge_lists reduces slabs -> top-k.
#include "tt_common.hpp"

namespace tt {

constexpr int SC_QPW = 16;                  // queries per wave (MFMA N)
constexpr int SC_ROWS = 32;                 // rows per step (2 MFMA row blocks)
constexpr int SC_MAX_SLAB_ROWS = 65536;     // row offsets stored as uint16

// Two selection configurations (same scoring loop):
//   narrow: 4 waves x 16 queries, 192-entry buffers, 256-key sorts  -> k <= 128
//   wide:   1 wave  x 16 queries, 1280-entry buffers, 2048-key sorts -> k <= 1024
// A buffer is compacted when it may overflow within one step (count > CAND - SC_ROWS);
// compaction keeps k entries, so CAND - SC_ROWS - k >= 32 appends fit between compactions.
template <int NW, int CAND, int SORTN>
struct ScanCfg {
  static constexpr int kWaves = NW;
  static constexpr int kCand = CAND;
  static constexpr int kSortN = SORTN;
  static constexpr int kQPB = NW * SC_QPW;
  static constexpr int kKMax = CAND - SC_ROWS - 32;
  struct Smem {
    float score[NW][SC_QPW][CAND];
    uint16_t roff[NW][SC_QPW][CAND];
    int cnt[NW][SC_QPW];
    float theta[NW][SC_QPW];
  };
};
using CfgNarrow = ScanCfg<4, 192, 256>;
using CfgWide = ScanCfg<1, 1280, 2048>;

template <int PER>
__device__ __forceinline__ uint64_t pick(const uint64_t (&key)[PER], int r) {
  uint64_t v = key[0];
#pragma unroll
  for (int i = 1; i < PER; ++i) v = (r == i) ? key[i] : v;
  return v;
}

// Sort one query's candidate buffer (wave-wide).  If gout_* are non-null the sorted top-k
// is written there (global row = row0 + offset) instead of back into LDS.
template <int SORTN>
__device__ __noinline__ void compact_query(float* sc, uint16_t* ro, int* cntp, float* thp,
                                           int k, int lane, float* gout_s, int* gout_r,
                                           int* gout_c, int row0) {
  constexpr int PER = SORTN / 64;
  const int c = *cntp;
  uint64_t key[PER];
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const int e = lane * PER + r;
    key[r] = e < c ? make_key(sc[e], (uint32_t)ro[e]) : 0ull;
  }
  bitonic_desc<PER>(key, lane);
  const int nc = c < k ? c : k;
  wave_sync();
  if (gout_s) {
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      const int e = lane * PER + r;
      if (e < nc) {
        gout_s[e] = key_score(key[r]);
        gout_r[e] = row0 + (int)key_row(key[r]);
      }
    }
    if (lane == 0) *gout_c = nc;
  } else {
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      const int e = lane * PER + r;
      if (e < nc) {
        sc[e] = key_score(key[r]);
        ro[e] = (uint16_t)key_row(key[r]);
      }
    }
    if (c >= k) {
      const int src_lane = (k - 1) / PER, src_r = (k - 1) % PER;
      const uint64_t kk = pick<PER>(key, src_r);
      const uint32_t hi = __shfl((uint32_t)(kk >> 32), src_lane, 64);
      if (lane == 0) *thp = key_float(hi);
    }
    if (lane == 0) *cntp = nc;
  }
  wave_sync();
}

template <typename IdxT>
__device__ void merge_lists_block(uint64_t* buf, int& bcnt, uint32_t& th_key, int qid,
                                  const float* __restrict__ in_s, const IdxT* __restrict__ in_i,
                                  const int* __restrict__ in_c, int n_lists,
                                  int64_t list_stride_q, int64_t list_stride_l, int k_in, int k,
                                  int64_t row_base, float* out_s, int64_t* out_i,
                                  const int* qsel, uint32_t thk_min = 0u);
constexpr int MG_CAP = 8192;

// Scan one (query tile, row slab) work item: query slots [qbase, qbase + kQPB) of [0, nq)
// (qsel: slot -> query row), catalog rows [s0, s1).  Each query's sorted slab top-k goes to
// the lists at index (slot * n_slabs + slab).  A wave whose 16 slots are all past nq skips the
// scan (a handful of flagged fallback queries then costs one wave's MFMAs, not the tile's).
template <int EP, class Cfg>
__device__ __forceinline__ void scan_tile(const float* __restrict__ db, int64_t n, int64_t ld_db,
                                          const float* __restrict__ q, int nq, int64_t ld_q,
                                          int k, int64_t s0, int64_t s1, int n_slabs, int slab,
                                          int qbase, float* __restrict__ ws_score,
                                          int* __restrict__ ws_row, int* __restrict__ ws_cnt,
                                          const int* __restrict__ qsel, typename Cfg::Smem& sm) {
  constexpr int SC_CAND = Cfg::kCand;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ql = lane & 15, g = lane >> 4;
  const int wbase = qbase + w * SC_QPW;
  const int qi = wbase + ql;
  const bool qvalid = qi < nq;

  // query fragment: dims 16t + 4g .. +3 of query qi
  f32x4 qf[EP / 16];
  {
    const int qrow = qvalid ? (qsel ? qsel[qi] : qi) : 0;
    const float* qp = q + (int64_t)qrow * ld_q + 4 * g;
#pragma unroll
    for (int t = 0; t < EP / 16; ++t) {
      f32x4 v = *(const f32x4*)(qp + 16 * t);
      qf[t] = qvalid ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  if (lane < SC_QPW) {
    sm.cnt[w][lane] = 0;
    sm.theta[w][lane] = -__builtin_huge_valf();
  }
  wave_sync();
  float theta = -__builtin_huge_valf();

  float* my_sc = sm.score[w][ql];
  uint16_t* my_ro = sm.roff[w][ql];
  int* my_cnt = &sm.cnt[w][ql];

  const int64_t s_end = wbase < nq ? s1 : s0;  // idle wave: no rows
  for (int64_t rb = s0; rb < s_end; rb += SC_ROWS) {
    const int64_t ra = (rb + ql < n) ? rb + ql : n - 1;
    const int64_t rc = (rb + 16 + ql < n) ? rb + 16 + ql : n - 1;
    const float* pa = db + ra * ld_db + 4 * g;
    const float* pc = db + rc * ld_db + 4 * g;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < EP / 16; ++t) {
      const f32x4 a0 = *(const f32x4*)(pa + 16 * t);
      const f32x4 a1 = *(const f32x4*)(pc + 16 * t);
      const f32x4 b = qf[t];
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[0], b[0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[0], b[0], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[1], b[1], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[1], b[1], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[2], b[2], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[2], b[2], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[3], b[3], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[3], b[3], acc1, 0, 0, 0);
    }
    // D[row 4g+j][col ql]: acc0 -> rows rb+4g+j, acc1 -> rows rb+16+4g+j
    float sv[8];
    int rv[8];
    uint32_t pass = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sv[j] = j < 4 ? acc0[j] : acc1[j - 4];
      rv[j] = (int)(rb - s0) + (j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4));
      const bool ok = qvalid && (s0 + rv[j] < s1) && (sv[j] >= theta);
      pass |= ok ? (1u << j) : 0u;
    }
    if (__ballot(pass != 0) != 0ull) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (pass & (1u << j)) {
          const int slot = atomicAdd(my_cnt, 1);
          my_sc[slot] = sv[j];
          my_ro[slot] = (uint16_t)rv[j];
        }
      }
      wave_sync();
      const int c = *my_cnt;
      uint64_t need = __ballot(qvalid && c > SC_CAND - SC_ROWS) & 0xffffull;
      while (need) {
        const int qq = __builtin_ctzll(need);
        need &= need - 1;
        compact_query<Cfg::kSortN>(sm.score[w][qq], sm.roff[w][qq], &sm.cnt[w][qq],
                                   &sm.theta[w][qq], k, lane, nullptr, nullptr, nullptr, 0);
      }
      theta = sm.theta[w][ql];
    }
  }

  // flush: sorted top-k of every valid query of this wave -> lists [slot][n_slabs][k]
  for (int qq = 0; qq < SC_QPW; ++qq) {
    const int qg = wbase + qq;
    if (qg >= nq) break;
    const int64_t base = ((int64_t)qg * n_slabs + slab);
    compact_query<Cfg::kSortN>(sm.score[w][qq], sm.roff[w][qq], &sm.cnt[w][qq],
                               &sm.theta[w][qq], k, lane, ws_score + base * k,
                               ws_row + base * k, ws_cnt + base, (int)s0);
  }
}

template <int EP, class Cfg>
__global__ __launch_bounds__(64 * Cfg::kWaves, ((EP <= 384 && Cfg::kWaves > 1) ? 2 : 1)) void k_scan_topk_f32(
    const float* __restrict__ db, int64_t n, int64_t ld_db, const float* __restrict__ q,
    int nq, int64_t ld_q, int k, int rows_per_slab, int n_slabs,
    float* __restrict__ ws_score, int* __restrict__ ws_row, int* __restrict__ ws_cnt,
    const int* __restrict__ qsel, const int* __restrict__ qsel_n, int* __restrict__ done,
    int64_t row_base, float* __restrict__ out_s, int64_t* __restrict__ out_i) {
  constexpr int SC_QPB = Cfg::kQPB;
  static_assert(sizeof(typename Cfg::Smem) >= MG_CAP * 8, "merge buffer aliases the scan state");
  __shared__ __attribute__((aligned(16))) typename Cfg::Smem sm;
  const int qt = blockIdx.x, slab = blockIdx.y;
  if (qsel) nq = *qsel_n;  // fallback mode: slots 0..nq-1 map to queries qsel[slot]
  if (qt * SC_QPB >= nq) return;
  const int64_t s0 = (int64_t)slab * rows_per_slab;
  const int64_t s1 = (s0 + rows_per_slab < n) ? s0 + rows_per_slab : n;
  scan_tile<EP, Cfg>(db, n, ld_db, q, nq, ld_q, k, s0, s1, n_slabs, slab, qt * SC_QPB, ws_score,
                     ws_row, ws_cnt, qsel, sm);
  if (!done) return;
  // Fused merge (the filter's exact fallback of a one-tile batch, nq <= 64): the last slab
  // block to finish merges the tile's queries -- one launch instead of scan + k_merge_lists,
  // and with no query flagged (the common case) every block has already returned above.
  // done[0] is zeroed by the search's per-query init; agent-scope fences publish the slab
  // lists across XCDs (their L2s are not coherent with each other).
  __shared__ int last, bcnt;
  __shared__ uint32_t th_key;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(&done[qt], 1) == n_slabs - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
  uint64_t* buf = reinterpret_cast<uint64_t*>(&sm);  // the scan state is dead
  for (int qq = 0; qq < SC_QPB; ++qq) {
    const int qg = qt * SC_QPB + qq;
    if (qg >= nq) break;
    merge_lists_block<int>(buf, bcnt, th_key, qg, ws_score, ws_row, ws_cnt, n_slabs,
                           (int64_t)n_slabs * k, (int64_t)k, k, k, row_base, out_s, out_i, qsel);
  }
  if (threadIdx.x == 0) done[qt] = 0;
}

// ---------------------------------------------------------------------- adaptive fallback
// The bf16 filter's exact fallback for batches of more than one 64-query tile.  How many
// queries were flagged is known only on the device (*qsel_n), so the decomposition is chosen
// there: the flagged slots form tiles of 16 (one wave each, ScanCfg<1, ...>), and the fixed
// grid of FB_GRID one-wave blocks is spread over (tile, slab) items -- a few flagged queries
// get the whole chip (~FB_GRID slabs of >= 512 rows) instead of one 64-query tile's slabs on
// the batch plan (1.43-1.48 ms for 3 flagged queries of a 10k batch at 1M rows, round 2).
// Blocks walk the items grid-stride; k_merge_fallback merges each slot's slab lists.
constexpr int FB_GRID = 2048;  // one-wave blocks: 8 per CU (18.5 KB LDS each)
constexpr int FB_MERGE_GRID = 256;  // k_merge_fallback blocks
using CfgFb = ScanCfg<1, 192, 256>;
struct FbPlan {
  int tiles, spt, rows;
};
__host__ __device__ inline FbPlan fb_plan(int64_t n, int nflag) {
  FbPlan p;
  p.tiles = (nflag + SC_QPW - 1) / SC_QPW;
  const int64_t smin = (n + SC_MAX_SLAB_ROWS - 1) / SC_MAX_SLAB_ROWS;  // uint16 row offsets
  const int64_t smax = (n + 511) / 512;                                  // >= 512 rows per slab
  int64_t s = p.tiles > 0 ? FB_GRID / p.tiles : 1;
  if (s > smax) s = smax;
  if (s < smin) s = smin;
  if (s < 1) s = 1;
  int64_t r = (n + s - 1) / s;
  r = (r + SC_ROWS - 1) / SC_ROWS * SC_ROWS;
  p.rows = (int)r;
  p.spt = (int)((n + r - 1) / r);
  return p;
}
// the split merge's partial lists (FB_MERGE_GRID x k of (f32 score, i64 row)) + counters
static int64_t fb_merge_bytes(int k) {
  return (int64_t)FB_MERGE_GRID * k * 12 + FB_MERGE_GRID * 4 + 256;
}
// list entries (of k) the fallback of up to nq flagged queries may write
static int64_t fb_items_max(int64_t n, int nq) {
  const int64_t tmax = (nq + SC_QPW - 1) / SC_QPW;
  const int64_t smin = (n + SC_MAX_SLAB_ROWS - 1) / SC_MAX_SLAB_ROWS;
  const int64_t a = FB_GRID, b = tmax * (smin > 1 ? smin : 1);
  return (a > b ? a : b) + 1;
}

template <int EP>
__global__ __launch_bounds__(64, 2) void k_scan_fallback(
    const float* __restrict__ db, int64_t n, int64_t ld_db, const float* __restrict__ q,
    int64_t ld_q, int k, const int* __restrict__ qsel, const int* __restrict__ qsel_n,
    float* __restrict__ ws_score, int* __restrict__ ws_row, int* __restrict__ ws_cnt,
    int* __restrict__ mg_done) {
  __shared__ __attribute__((aligned(16))) typename CfgFb::Smem sm;
  const int nq = *qsel_n;
  if (nq == 0) return;
  if (blockIdx.x == 0)  // the merge's per-slot arrival counters (k_merge_fallback)
    for (int i = threadIdx.x; i < FB_MERGE_GRID; i += blockDim.x) mg_done[i] = 0;
  const FbPlan p = fb_plan(n, nq);
  const int items = p.tiles * p.spt;
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    const int tile = it / p.spt, slab = it % p.spt;
    const int64_t s0 = (int64_t)slab * p.rows;
    const int64_t s1 = (s0 + p.rows < n) ? s0 + p.rows : n;
    scan_tile<EP, CfgFb>(db, n, ld_db, q, nq, ld_q, k, s0, s1, p.spt, slab, tile * SC_QPW,
                         ws_score, ws_row, ws_cnt, qsel, sm);
  }
}

// ----------------------------------------------------------------------------- merge
// One 256-thread block per query.  Lists: n_lists x k_in sorted entries (score, row);
// list j has cnt[j] valid entries (cnt == nullptr: all k_in valid, entries with idx < 0
// ignored).  theta = max over FULL lists (cnt == k_in >= k) of the k-th entry is a
// lower bound of the global k-th best; entries below it are skipped.  Survivors are
// collected in LDS in rounds (sort + truncate when the buffer would overflow).
constexpr int MG_CHUNK = 4096;

__device__ void block_bitonic_desc(uint64_t* buf, int n_pow2) {
  for (int size = 2; size <= n_pow2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int i = threadIdx.x; i < n_pow2 / 2; i += blockDim.x) {
        const int lo = 2 * stride * (i / stride) + (i % stride);
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint64_t a = buf[lo], b = buf[hi];
        if ((a < b) == up) {
          buf[lo] = b;
          buf[hi] = a;
        }
      }
    }
  }
  __syncthreads();
}

__device__ __forceinline__ int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

// One query's merge by the whole block (any block size); buf = MG_CAP keys of LDS.
template <typename IdxT>
__device__ void merge_lists_block(uint64_t* buf, int& bcnt, uint32_t& th_key, int qid,
                                  const float* __restrict__ in_s, const IdxT* __restrict__ in_i,
                                  const int* __restrict__ in_c, int n_lists,
                                  int64_t list_stride_q, int64_t list_stride_l, int k_in, int k,
                                  int64_t row_base, float* out_s, int64_t* out_i,
                                  const int* qsel, uint32_t thk_min) {
  const int64_t orow = qsel ? qsel[qid] : qid;
  const float* qs = in_s + (int64_t)qid * list_stride_q;
  const IdxT* qix = in_i + (int64_t)qid * list_stride_q;
  const int* qc = in_c ? in_c + (int64_t)qid * n_lists : nullptr;

  if (threadIdx.x == 0) { bcnt = 0; th_key = thk_min; }
  __syncthreads();
  // threshold from full lists (or a caller's sound lower bound of the k-th best: thk_min)
  uint32_t tk = 0u;
  if (k <= k_in) {
    for (int j = threadIdx.x; j < n_lists; j += blockDim.x) {
      const int c = qc ? qc[j] : k_in;
      if (c >= k) {
        const IdxT ix = qix[(int64_t)j * list_stride_l + (k - 1)];
        if (ix >= 0) {
          const uint32_t fk = float_key(qs[(int64_t)j * list_stride_l + (k - 1)]);
          tk = fk > tk ? fk : tk;
        }
      }
    }
  }
  atomicMax(&th_key, tk);
  __syncthreads();
  const uint32_t thk = th_key;

  const int64_t total = (int64_t)n_lists * k_in;
  for (int64_t c0 = 0; c0 < total; c0 += MG_CHUNK) {
    const int64_t c1 = c0 + MG_CHUNK < total ? c0 + MG_CHUNK : total;
    for (int64_t e = c0 + threadIdx.x; e < c1; e += blockDim.x) {
      const int j = (int)(e / k_in), i = (int)(e % k_in);
      const int c = qc ? qc[j] : k_in;
      if (i >= c) continue;
      const int64_t off = (int64_t)j * list_stride_l + i;
      const IdxT ix = qix[off];
      if (ix < 0) continue;
      const float s = qs[off];
      const uint32_t fk = float_key(s);
      if (s != s || fk < thk) continue;
      const int pos = atomicAdd(&bcnt, 1);
      buf[pos] = ((uint64_t)fk << 32) | (uint64_t)(0xffffffffu - (uint32_t)ix);
    }
    __syncthreads();
    const int nb = bcnt;
    if (nb > MG_CAP - MG_CHUNK) {  // truncate to top k before the next chunk
      const int np = next_pow2(nb);
      for (int i = nb + threadIdx.x; i < np; i += blockDim.x) buf[i] = 0ull;
      block_bitonic_desc(buf, np);
      if (threadIdx.x == 0) bcnt = nb < k ? nb : k;
    }
    __syncthreads();  // every thread has read bcnt before the next chunk appends
  }
  __syncthreads();
  const int nb = bcnt;
  const int np = next_pow2(nb < 2 ? 2 : nb);
  for (int i = nb + threadIdx.x; i < np; i += blockDim.x) buf[i] = 0ull;
  block_bitonic_desc(buf, np);
  for (int i = threadIdx.x; i < k; i += blockDim.x) {
    float s = -__builtin_huge_valf();
    int64_t ix = -1;
    if (i < nb) {
      s = key_score(buf[i]);
      ix = row_base + (int64_t)key_row(buf[i]);
    }
    out_s[orow * k + i] = s;
    out_i[orow * k + i] = ix;
  }
  __syncthreads();  // buf / bcnt / th_key free for the block's next query
}

template <typename IdxT>
__global__ __launch_bounds__(256) void k_merge_lists(const float* __restrict__ in_s,
                                                     const IdxT* __restrict__ in_i,
                                                     const int* __restrict__ in_c,
                                                     int n_lists, int64_t list_stride_q,
                                                     int64_t list_stride_l, int k_in, int k,
                                                     int64_t row_base, float* out_s,
                                                     int64_t* out_i, const int* qsel,
                                                     const int* qsel_n) {
  __shared__ uint64_t buf[MG_CAP];
  __shared__ int bcnt;
  __shared__ uint32_t th_key;
  const int qid = blockIdx.x;
  if (qsel && qid >= *qsel_n) return;
  merge_lists_block<IdxT>(buf, bcnt, th_key, qid, in_s, in_i, in_c, n_lists, list_stride_q,
                          list_stride_l, k_in, k, row_base, out_s, out_i, qsel);
}

// Merge of the adaptive fallback's slab lists: block-strided over the flagged slots.
// Merge of the adaptive fallback's slab lists.  A few flagged queries get up to ~2000 slabs
// of k entries each (1953 x 100 at 1M rows): one block per query walked all ~195k entries
// (+1.17 ms on a 10k batch with 3 flagged queries).  With fewer slots than blocks, each slot
// gets bps = FB_MERGE_GRID / nq blocks, each merging a contiguous range of its slab lists into
// a partial top-k (p_s / p_i, global rows); the last block of the slot to arrive (agent-scope
// counter mg_done[slot], zeroed by k_scan_fallback) merges the bps partial lists.
__global__ __launch_bounds__(256) void k_merge_fallback(const float* __restrict__ ws_score,
                                                        const int* __restrict__ ws_row,
                                                        const int* __restrict__ ws_cnt, int64_t n,
                                                        int k, int64_t row_base, float* out_s,
                                                        int64_t* out_i, const int* qsel,
                                                        const int* qsel_n, float* p_s,
                                                        int64_t* p_i, int* mg_done) {
  __shared__ uint64_t buf[MG_CAP];
  __shared__ int bcnt;
  __shared__ uint32_t th_key;
  __shared__ int last;
  const int nq = *qsel_n;
  if (nq == 0) return;
  const int spt = fb_plan(n, nq).spt;
  const int bps = nq < (int)gridDim.x ? (int)gridDim.x / nq : 1;
  if (bps == 1) {
    for (int slot = blockIdx.x; slot < nq; slot += gridDim.x)
      merge_lists_block<int>(buf, bcnt, th_key, slot, ws_score, ws_row, ws_cnt, spt,
                             (int64_t)spt * k, (int64_t)k, k, k, row_base, out_s, out_i, qsel);
    return;
  }
  const int slot = blockIdx.x / bps, part = blockIdx.x % bps;
  if (slot >= nq) return;
  // the slot's threshold over ALL its full lists (the k-th entry of any full list bounds the
  // k-th best from below): each partial block then keeps only the few entries above it
  // (with the partial's own lists only, ~k survivors per block had to be sorted)
  __shared__ uint32_t thk_all;
  if (threadIdx.x == 0) thk_all = 0u;
  __syncthreads();
  {
    uint32_t tk = 0u;
    const float* qs = ws_score + (int64_t)slot * spt * k;
    const int* qr = ws_row + (int64_t)slot * spt * k;
    const int* qc = ws_cnt + (int64_t)slot * spt;
    for (int j = threadIdx.x; j < spt; j += blockDim.x)
      if (qc[j] >= k && qr[(int64_t)j * k + k - 1] >= 0) {
        const uint32_t fk = float_key(qs[(int64_t)j * k + k - 1]);
        tk = fk > tk ? fk : tk;
      }
    atomicMax(&thk_all, tk);
  }
  __syncthreads();
  const uint32_t thk = thk_all;
  const int j0 = (int)((int64_t)part * spt / bps), j1 = (int)((int64_t)(part + 1) * spt / bps);
  const int64_t qo = (int64_t)slot * spt * k + (int64_t)j0 * k;
  float* ps = p_s + ((int64_t)slot * bps + part) * k;
  int64_t* pi = p_i + ((int64_t)slot * bps + part) * k;
  merge_lists_block<int>(buf, bcnt, th_key, 0, ws_score + qo, ws_row + qo,
                         ws_cnt + (int64_t)slot * spt + j0, j1 - j0, 0, (int64_t)k, k, k, 0,
                         ps, pi, nullptr, thk);
  __threadfence();  // this block's partial list visible before it counts itself in
  if (threadIdx.x == 0) last = atomicAdd(&mg_done[slot], 1) == bps - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();  // the other blocks' partial lists
  merge_lists_block<int64_t>(buf, bcnt, th_key, slot, p_s + (int64_t)slot * bps * k,
                             p_i + (int64_t)slot * bps * k, nullptr, bps, 0, (int64_t)k, k, k,
                             row_base, out_s, out_i, qsel, thk);
}

// ----------------------------------------------------------------------------- host
struct ScanPlan {
  int qt, n_slabs, rows_per_slab;
};

static bool wide_k(int k) { return k > CfgNarrow::kKMax; }

static int qpb_of(int k) { return wide_k(k) ? CfgWide::kQPB : CfgNarrow::kQPB; }

static ScanPlan plan_scan(int64_t n, int nq, int k, int par = 512) {
  ScanPlan p;
  const int qpb = qpb_of(k);
  p.qt = (nq + qpb - 1) / qpb;
  // enough blocks to fill 256 CUs x 2 (par), slabs no longer than SC_MAX_SLAB_ROWS
  int64_t s_min = (n + SC_MAX_SLAB_ROWS - 1) / SC_MAX_SLAB_ROWS;
  int64_t s_par = (par + p.qt - 1) / p.qt;
  int64_t s_rows = (n + 511) / 512;  // do not go below ~512 rows per slab
  int64_t s = s_par < s_rows ? s_par : s_rows;
  if (s < s_min) s = s_min;
  if (s < 1) s = 1;
  int64_t r = (n + s - 1) / s;
  r = (r + SC_ROWS - 1) / SC_ROWS * SC_ROWS;
  if (r > SC_MAX_SLAB_ROWS) r = SC_MAX_SLAB_ROWS;
  p.rows_per_slab = (int)r;
  p.n_slabs = (int)((n + r - 1) / r);
  return p;
}

static int padded_dim(int d) {
  const int ep[] = {64, 128, 256, 384, 512, 768};
  for (int e : ep)
    if (d <= e) return e;
  return -1;
}

}  // namespace tt

using namespace tt;

extern "C" int32_t tt_padded_dim(int32_t d) { return d >= 1 ? padded_dim(d) : -1; }

extern "C" int tt_scan_workspace_bytes(int64_t n, int32_t d, int32_t nq, int32_t k,
                                       int64_t* bytes) {
  TT_REQUIRE(bytes != nullptr, "bytes == NULL");
  TT_REQUIRE(n >= 1 && nq >= 1 && k >= 1, "n, nq, k must be >= 1");
  (void)d;
  const ScanPlan p = plan_scan(n, nq, k);
  const int64_t entries = (int64_t)nq * p.n_slabs * k;
  int64_t b = entries * 8 + (int64_t)nq * p.n_slabs * 4;
  if (p.qt > 1 && k <= CfgFb::kKMax) {  // the adaptive fallback's lists (the same memory)
    const int64_t fb = fb_items_max(n, nq) * SC_QPW * (8 * (int64_t)k + 4) + fb_merge_bytes(k);
    b = b > fb ? b : fb;
  }
  *bytes = (b + 255) / 256 * 256;
  return TT_OK;
}

static int scan_f32_impl(const float* db, int64_t n, int32_t d, int64_t ld_db,
                         int64_t row_base, const float* q, int32_t nq, int64_t ld_q, int32_t k,
                         const int32_t* qsel, const int32_t* qsel_n, float* out_score,
                         int64_t* out_idx, void* workspace, int64_t workspace_bytes,
                         void* stream, void* ev_start, void* ev_stop, int* done = nullptr) {
  TT_REQUIRE(n >= 1, "empty catalog");
  TT_REQUIRE(n <= 0x7fffffffLL, "shard rows must fit int32");
  TT_REQUIRE(nq >= 0, "nq < 0");
  TT_REQUIRE(k >= 1 && k <= n, "need 1 <= k <= n");
  if (nq == 0) return TT_OK;
  const int ep = padded_dim(d);
  if (ep < 0) return fail(TT_ERR_UNSUPPORTED, "tt_scan_topk_f32: d > 768");
  if (k > CfgWide::kKMax) return fail(TT_ERR_UNSUPPORTED, "tt_scan_topk_f32: k > 1024");
  TT_REQUIRE(ld_db >= ep && ld_q >= ep, "ld must be >= tt_padded_dim(d) (zero padded)");
  TT_REQUIRE(ld_db % 4 == 0 && ld_q % 4 == 0, "ld must be a multiple of 4");
  TT_REQUIRE(((uintptr_t)db % 16) == 0 && ((uintptr_t)q % 16) == 0, "db/q must be 16-B aligned");
  int64_t need = 0;
  tt_scan_workspace_bytes(n, d, nq, k, &need);
  if (workspace_bytes < need || workspace == nullptr)
    return fail(TT_ERR_WORKSPACE, "tt_scan_topk_f32: workspace too small");
  // (the fused one-tile fallback launched on every small search, usually exiting at once: 256
  // or 128 instead of 512 slab blocks saved <= 2 us of that idle launch -- not adopted)
  const ScanPlan p = plan_scan(n, nq, k);
  const int64_t entries = (int64_t)nq * p.n_slabs * k;
  float* ws_s = (float*)workspace;
  int* ws_r = (int*)(ws_s + entries);
  int* ws_c = ws_r + entries;
  hipStream_t st = (hipStream_t)stream;
  const bool wide = wide_k(k);
  const dim3 block(wide ? 64 * CfgWide::kWaves : 64 * CfgNarrow::kWaves);
  if (done && p.qt > 1) {
    // The filter's exact fallback for a batch of more than one 64-query tile: the flagged
    // queries are compacted into slots 0 .. *qsel_n, and the adaptive kernel decides on the
    // device how to spread them over the chip; its merge follows.  Both launches exit at once
    // when nothing is flagged.
    TT_REQUIRE(k <= CfgFb::kKMax, "fallback: k > 128");
    float* fs = (float*)workspace;
    int* fr = (int*)(fs + fb_items_max(n, nq) * SC_QPW * k);
    int* fc = fr + fb_items_max(n, nq) * SC_QPW * k;
    // the split merge's partials after the lists' counts (8-B aligned), then its counters
    const int64_t fc_end = (int64_t)((char*)(fc + fb_items_max(n, nq) * SC_QPW) - (char*)workspace);
    int64_t* pi = (int64_t*)((char*)workspace + (fc_end + 15) / 16 * 16);
    float* ps = (float*)(pi + (int64_t)FB_MERGE_GRID * k);
    int* mg = (int*)(ps + (int64_t)FB_MERGE_GRID * k);
#define TT_FB_CASE(E)                                                                         \
  case E:                                                                                     \
    hipLaunchKernelGGL(k_scan_fallback<E>, dim3(FB_GRID), dim3(64), 0, st, db, n, ld_db, q,   \
                       ld_q, k, qsel, qsel_n, fs, fr, fc, mg);                                \
    break;
    switch (ep) {
      TT_FB_CASE(64)
      TT_FB_CASE(128)
      TT_FB_CASE(256)
      TT_FB_CASE(384)
      TT_FB_CASE(512)
      TT_FB_CASE(768)
      default:
        return fail(TT_ERR_UNSUPPORTED, "fallback: bad padded dim");
    }
#undef TT_FB_CASE
    int rc = check_launch("k_scan_fallback");
    if (rc) return rc;
    hipLaunchKernelGGL(k_merge_fallback, dim3(FB_MERGE_GRID), dim3(256), 0, st, fs, fr, fc, n, k,
                       row_base, out_score, out_idx, qsel, qsel_n, ps, pi, mg);
    return check_launch("k_merge_fallback");
  }
  const dim3 grid(p.qt, p.n_slabs);
#define TT_SCAN_CASE(E)                                                                       \
  case E:                                                                                     \
    if (wide)                                                                                 \
      hipLaunchKernelGGL((k_scan_topk_f32<E, CfgWide>), grid, block, 0, st, db, n, ld_db, q,  \
                         nq, ld_q, k, p.rows_per_slab, p.n_slabs, ws_s, ws_r, ws_c, qsel,     \
                         qsel_n, done, row_base, out_score, out_idx);                         \
    else                                                                                      \
      hipLaunchKernelGGL((k_scan_topk_f32<E, CfgNarrow>), grid, block, 0, st, db, n, ld_db,   \
                         q, nq, ld_q, k, p.rows_per_slab, p.n_slabs, ws_s, ws_r, ws_c, qsel,  \
                         qsel_n, done, row_base, out_score, out_idx);                         \
    break;
  if (ev_start && hipEventRecord((hipEvent_t)ev_start, st) != hipSuccess)
    return fail(TT_ERR_LAUNCH, "tt_scan_topk_f32_timed: hipEventRecord(start) failed");
  switch (ep) {
    TT_SCAN_CASE(64)
    TT_SCAN_CASE(128)
    TT_SCAN_CASE(256)
    TT_SCAN_CASE(384)
    TT_SCAN_CASE(512)
    TT_SCAN_CASE(768)
    default:
      return fail(TT_ERR_UNSUPPORTED, "tt_scan_topk_f32: bad padded dim");
  }
#undef TT_SCAN_CASE
  int rc = check_launch("k_scan_topk_f32");
  if (rc) return rc;
  if (ev_stop && hipEventRecord((hipEvent_t)ev_stop, st) != hipSuccess)
    return fail(TT_ERR_LAUNCH, "tt_scan_topk_f32_timed: hipEventRecord(stop) failed");
  if (done) return TT_OK;  // merged inside the scan launch
  hipLaunchKernelGGL(k_merge_lists<int>, dim3(nq), dim3(256), 0, st, ws_s, ws_r, ws_c,
                     p.n_slabs, (int64_t)p.n_slabs * k, (int64_t)k, k, k, row_base, out_score,
                     out_idx, qsel, qsel_n);
  return check_launch("k_merge_lists");
}

extern "C" int tt_scan_topk_f32_timed(const float* db, int64_t n, int32_t d, int64_t ld_db,
                                      int64_t row_base, const float* q, int32_t nq,
                                      int64_t ld_q, int32_t k, float* out_score,
                                      int64_t* out_idx, void* workspace,
                                      int64_t workspace_bytes, void* stream, void* ev_start,
                                      void* ev_stop) {
  return scan_f32_impl(db, n, d, ld_db, row_base, q, nq, ld_q, k, nullptr, nullptr, out_score,
                       out_idx, workspace, workspace_bytes, stream, ev_start, ev_stop);
}

extern "C" int tt_scan_topk_f32(const float* db, int64_t n, int32_t d, int64_t ld_db,
                                int64_t row_base, const float* q, int32_t nq, int64_t ld_q,
                                int32_t k, float* out_score, int64_t* out_idx, void* workspace,
                                int64_t workspace_bytes, void* stream) {
  return scan_f32_impl(db, n, d, ld_db, row_base, q, nq, ld_q, k, nullptr, nullptr, out_score,
                       out_idx, workspace, workspace_bytes, stream, nullptr, nullptr);
}

// Exact scan of the queries listed on the device (qsel[0 .. *qsel_n)); outputs go to the
// listed rows of out_*.  Launched for nq slots; blocks beyond *qsel_n exit immediately.
extern "C" int tt_scan_topk_f32_select(const float* db, int64_t n, int32_t d, int64_t ld_db,
                                       int64_t row_base, const float* q, int32_t nq,
                                       int64_t ld_q, int32_t k, const int32_t* qsel,
                                       const int32_t* qsel_n, float* out_score,
                                       int64_t* out_idx, void* workspace,
                                       int64_t workspace_bytes, void* stream) {
  TT_REQUIRE(qsel != nullptr && qsel_n != nullptr, "qsel / qsel_n must be device pointers");
  return scan_f32_impl(db, n, d, ld_db, row_base, q, nq, ld_q, k, qsel, qsel_n, out_score,
                       out_idx, workspace, workspace_bytes, stream, nullptr, nullptr);
}

namespace tt {
// The bf16 filter's exact fallback (tt_filter.hip): nq <= 64 -> the select-mode scan with the
// slab merge fused into the scan launch (done: ONE zeroed counter, done[0], reset by the last
// block); nq > 64 -> the adaptive fallback (k_scan_fallback + k_merge_fallback; done unused).
int scan_f32_select_fused(const float* db, int64_t n, int32_t d, int64_t ld_db, int64_t row_base,
                          const float* q, int32_t nq, int64_t ld_q, int32_t k,
                          const int32_t* qsel, const int32_t* qsel_n, int* done,
                          float* out_score, int64_t* out_idx, void* workspace,
                          int64_t workspace_bytes, void* stream) {
  TT_REQUIRE(qsel && qsel_n && done, "qsel / qsel_n / done must be device pointers");
  return scan_f32_impl(db, n, d, ld_db, row_base, q, nq, ld_q, k, qsel, qsel_n, out_score,
                       out_idx, workspace, workspace_bytes, stream, nullptr, nullptr, done);
}
}  // namespace tt

extern "C" int tt_topk_merge_f32(const float* in_score, const int64_t* in_idx, int32_t n_lists,
                                 int32_t nq, int32_t k_in, int32_t k, float* out_score,
                                 int64_t* out_idx, void* stream) {
  TT_REQUIRE(n_lists >= 1 && nq >= 0 && k_in >= 1 && k >= 1, "bad sizes");
  TT_REQUIRE(k <= 4096, "k > 4096");
  if (nq == 0) return TT_OK;
  // layout [n_lists][nq][k_in]: list stride nq*k_in, query stride k_in
  hipLaunchKernelGGL(k_merge_lists<int64_t>, dim3(nq), dim3(256), 0, (hipStream_t)stream,
                     in_score, in_idx, (const int*)nullptr, n_lists, (int64_t)k_in,
                     (int64_t)nq * k_in, k_in, k, (int64_t)0, out_score, out_idx,
                     (const int*)nullptr, (const int*)nullptr);
  return check_launch("tt_topk_merge_f32");
}
