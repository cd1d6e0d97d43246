// tt_select.hip -- exact top-k by scores-then-radix-select (gfx950): the large-k scan.
//
// Replaces faiss.IndexFlatIP.search for k in (128, 1024] (server.py:46 lets /retrieve ask for
// up to k = 1000; vector_db.py:160,196 pass k straight to the index).  tt_scan_topk_f32 keeps a
// sorted top-k list per (query, slab of a few thousand rows) and merges them: at k = 1000 a
// slab list holds a quarter of its slab, so the lists and their merge cost 24-29 ms per search
// of a 1M-row catalog.  Here every exact f32 score is written once (the scan's MFMA scoring
// loop: the canonical fma order, so the scores are the scan's bits) and each query's k-th
// largest 64-bit key -- float_key(score) << 32 | ~row, the scan's order: score descending,
// ties to the lower row, NaN last -- is located by an MSB-first radix select over its score row
// (11/11/10-bit digits of the score word, then of the row word): a digit ends the search once
// the keys at or above its bucket number at most SL_CAP (usually the second digit: a 22-bit
// bucket holds a handful of keys), and those keys -- the top k and the rest of the bucket --
// are collected and sorted by one wave.  Launches per query chunk: init, scores (+ the first
// histogram for a single query), 2 x (histogram, digit), the tail (digits 3-6 for heavy
// duplicates; exits at once otherwise), collect, sort.  Each histogram / collect pass re-reads
// the chunk's score rows (4 B per row and query, L2 / MALL resident at 1M rows); the catalog is
// read once per 64-query tile.
#include "tt_common.hpp"

namespace tt {

constexpr int SL_BINS = 2048;
constexpr int SL_KMAX = 1024;
constexpr int SL_CAP = 2048;                         // candidates collected and sorted per query
constexpr int SL_CHUNK = 8192;                       // score rows per histogram / collect block
constexpr int64_t SL_SCORE_BUDGET = 256ll << 20;     // bytes of score rows per query chunk
constexpr int SL_QT = 16;                            // queries per wave (MFMA N)
constexpr int SL_ROWS = 32;                          // slab rows: a multiple of this
__constant__ const int kSlShift[6] = {53, 42, 32, 21, 10, 0};
__constant__ const int kSlWidth[6] = {11, 11, 10, 11, 11, 10};

struct SelState {
  uint64_t prefix;  // digits fixed so far (MSB first)
  uint64_t thr;     // done: the selection threshold (keys >= thr are the top k)
  int krem;         // rank of the k-th key among the keys that share `prefix`
  int done;         // the k-th key's remaining digits need not be resolved
  int ncand;        // collect counter
  int pad;
};

__device__ __forceinline__ uint64_t sel_key(float s, int64_t row) {
  return ((uint64_t)float_key(s) << 32) | (uint64_t)(0xffffffffu - (uint32_t)row);
}

// ---------------------------------------------------------------------------- scores
// Exact f32 scores of query rows [qbase, qbase + 16 * (SHARE ? 4 : 1)) for catalog rows
// [s0, s1): the scan's scoring loop (tt_scan.hip scan_tile: query dims 16t + 4g .. + 3 in the
// MFMA B operand, the same MFMA sequence per accumulator), so score[q][r] has the scan's bits.  SHARE
// (more than 16 queries): the block's 4 waves own 16 queries each and stream the same rows;
// otherwise one 16-query tile whose rows the 4 waves split.
// Rows per wave step: one 16-row MFMA block when the waves split the rows (a step's 24 loads
// all in flight beside the 96 query VGPRs: 0.57 -> 0.43 ms per k = 1000 search at nq = 1, 1M
// rows), two when they share them (nq = 32: 1.09 vs 1.17 ms with one).
// H0 (one query, rows split): the first digit's histogram is counted here from the scores in
// registers (LDS, flushed once per block) instead of by a pass over the score row.
#ifndef TT_SEL_RMIN
#define TT_SEL_RMIN 1024  // smallest slab (rows) when one query tile's waves split the rows (2048: 0.39 ms per nq = 1 search, 1024: 0.35)
#endif
#ifndef TT_SEL_NT
#define TT_SEL_NT 0  // catalog row loads non-temporal
#endif
template <int EP, bool SHARE, bool H0 = false>
__global__ __launch_bounds__(256, EP <= 384 ? 2 : 1) void k_sel_scores(
    const float* __restrict__ db, int64_t n, int64_t ld_db, const float* __restrict__ q, int nq,
    int64_t ld_q, int rows_per_slab, float* __restrict__ scores, int64_t ld_s,
    uint32_t* __restrict__ hist0) {
  static_assert(!(H0 && SHARE), "H0: rows split over the waves, one query");
  constexpr int RB = SHARE ? 2 : 1, ROWS = 16 * RB;
  __shared__ uint32_t lh[H0 ? SL_BINS : 1];
  if constexpr (H0) {
    for (int b = threadIdx.x; b < SL_BINS; b += 256) lh[b] = 0u;
    __syncthreads();
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ql = lane & 15, g = lane >> 4;
  const int nw = blockDim.x >> 6;  // SHARE: one wave per 16 queries of the block's tile
  const int qbase = blockIdx.y * (SHARE ? nw * SL_QT : SL_QT) + (SHARE ? w * SL_QT : 0);
  if (qbase >= nq) return;  // whole wave idle (uniform)
  const int qi = qbase + ql;
  const bool qvalid = qi < nq;
  f32x4 qf[EP / 16];
  {
    const float* qp = q + (int64_t)(qvalid ? qi : 0) * ld_q + 4 * g;
#pragma unroll
    for (int t = 0; t < EP / 16; ++t) {
      const f32x4 v = *(const f32x4*)(qp + 16 * t);
      qf[t] = qvalid ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  const int64_t s0 = (int64_t)blockIdx.x * rows_per_slab;
  const int64_t s1 = s0 + rows_per_slab < n ? s0 + rows_per_slab : n;
  float* srow = scores + (int64_t)(qvalid ? qi : 0) * ld_s;
  const int64_t first = SHARE ? s0 : s0 + (int64_t)ROWS * w;
  const int64_t stride = SHARE ? ROWS : 4 * ROWS;
  for (int64_t rb = first; rb < s1; rb += stride) {
    const float* pa[RB];
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      const int64_t r = (rb + 16 * b + ql < n) ? rb + 16 * b + ql : n - 1;
      pa[b] = db + r * ld_db + 4 * g;
    }
    f32x4 acc[RB];
#pragma unroll
    for (int b = 0; b < RB; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < EP / 16; ++t) {
      f32x4 a[RB];
#pragma unroll
      for (int b = 0; b < RB; ++b)
        a[b] = TT_SEL_NT ? __builtin_nontemporal_load((const f32x4*)(pa[b] + 16 * t))
                         : *(const f32x4*)(pa[b] + 16 * t);
      const f32x4 bq = qf[t];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int b = 0; b < RB; ++b)
          acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[b][u], bq[u], acc[b], 0, 0, 0);
    }
    // D[row 4g + j][query ql] of block b -> score row rb + 16 b + 4g + j
    if (qvalid) {
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        const int64_t r0 = rb + 16 * b + 4 * g;
        if (r0 + 3 < s1) {
          *(f32x4*)(srow + r0) = acc[b];
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (r0 + j < s1) srow[r0 + j] = acc[b][j];
        }
        if constexpr (H0) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (r0 + j < s1) atomicAdd(&lh[float_key(acc[b][j]) >> 21], 1u);
        }
      }
    }
  }
  if constexpr (H0) {
    __syncthreads();
    for (int b = threadIdx.x; b < SL_BINS; b += 256)
      if (lh[b]) atomicAdd(&hist0[b], lh[b]);
  }
}

// ------------------------------------------------------------------------- radix select
__global__ __launch_bounds__(256) void k_sel_init(SelState* __restrict__ st,
                                                  uint32_t* __restrict__ hist, int k) {
  const int qq = blockIdx.x;
  for (int b = threadIdx.x; b < SL_BINS; b += 256) hist[(int64_t)qq * SL_BINS + b] = 0u;
  if (threadIdx.x == 0) {
    SelState s;
    s.prefix = 0ull;
    s.thr = 0ull;
    s.krem = k;
    s.done = 0;
    s.ncand = 0;
    s.pad = 0;
    st[qq] = s;
  }
}

// Pass p histogram of digit p over the keys that share the state's prefix: block = (chunk of
// SL_CHUNK rows, query); LDS counts, flushed by atomics into the query's global histogram.
__global__ __launch_bounds__(256) void k_sel_hist(const float* __restrict__ scores, int64_t ld_s,
                                                  int64_t n, int p, const SelState* __restrict__ st,
                                                  uint32_t* __restrict__ hist) {
  __shared__ uint32_t lh[SL_BINS];
  const int qq = blockIdx.y;
  const SelState s = st[qq];
  if (s.done) return;  // uniform
  for (int b = threadIdx.x; b < SL_BINS; b += 256) lh[b] = 0u;
  __syncthreads();
  const int shift = kSlShift[p], width = kSlWidth[p], hs = shift + width;
  const uint32_t mask = (1u << width) - 1u;
  const float* sr = scores + (int64_t)qq * ld_s;
  const int64_t r0 = (int64_t)blockIdx.x * SL_CHUNK;
  const int64_t r1 = r0 + SL_CHUNK < n ? r0 + SL_CHUNK : n;
#pragma unroll 8
  for (int64_t r = r0 + threadIdx.x; r < r1; r += 256) {
    const uint64_t key = sel_key(sr[r], r);
    if (hs >= 64 || (key >> hs) == s.prefix) atomicAdd(&lh[(uint32_t)(key >> shift) & mask], 1u);
  }
  __syncthreads();
  uint32_t* gh = hist + (int64_t)qq * SL_BINS;
  for (int b = threadIdx.x; b < SL_BINS; b += 256)
    if (lh[b]) atomicAdd(&gh[b], lh[b]);
}

// Pass p digit: the bin d holding the krem-th largest key among those sharing the prefix
// (bins above d hold fewer than krem keys, with d at least krem); the histogram is cleared for
// the next pass.  When the keys in bin d and above number at most SL_CAP -- (k - krem) of them
// above the bin -- they are all collected: done, threshold (prefix . d) << shift.
__device__ void sel_digit(int p, int k, const SelState& s, SelState* __restrict__ sto,
                          uint32_t* h8base, uint32_t* part) {
  const int t = threadIdx.x;
  uint32_t h[8];
  uint32_t sum = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    h[i] = h8base[8 * t + i];
    sum += h[i];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) h8base[8 * t + i] = 0u;
  part[t] = sum;
  __syncthreads();
  // keys in bins above this thread's: the threads t' > t (suffix sum; 256 adds, done once)
  uint32_t above = 0;
  for (int u = t + 1; u < 256; ++u) above += part[u];
  const uint32_t krem = (uint32_t)s.krem;
#pragma unroll
  for (int i = 7; i >= 0; --i) {
    if (above < krem && above + h[i] >= krem) {
      const int shift = kSlShift[p], width = kSlWidth[p];
      SelState o = s;
      o.prefix = (s.prefix << width) | (uint64_t)(8 * t + i);
      o.krem = (int)(krem - above);
      // stop when the keys to collect fit the sort of the next power of two >= k (first
      // digit on), or SL_CAP (from the second digit on: the tail only for heavy duplicates)
      const uint32_t tot = (uint32_t)(k - s.krem) + above + h[i];
      uint32_t kp = 64;
      while (kp < (uint32_t)k) kp <<= 1;
      if (tot <= kp || (p >= 1 && tot <= (uint32_t)SL_CAP) || p == 5) {
        o.done = 1;
        o.thr = o.prefix << shift;
      }
      *sto = o;
    }
    above += h[i];
  }
}

__global__ __launch_bounds__(256) void k_sel_digit(int p, int k, SelState* __restrict__ st,
                                                   uint32_t* __restrict__ hist) {
  __shared__ uint32_t part[256];
  const int qq = blockIdx.x;
  const SelState s = st[qq];
  if (s.done) return;  // uniform
  sel_digit(p, k, s, st + qq, hist + (int64_t)qq * SL_BINS, part);
}

// Passes 2 .. 5 for a query whose first two digits left more than SL_CAP keys at or above the
// k-th key's bucket (thousands of keys sharing 22 bits of the score: exact duplicates): one
// block per query histograms the whole score row per pass in LDS.  Exits at once otherwise.
__global__ __launch_bounds__(256) void k_sel_tail(const float* __restrict__ scores, int64_t ld_s,
                                                  int64_t n, int k, SelState* __restrict__ st) {
  __shared__ uint32_t lh[SL_BINS];
  __shared__ uint32_t part[256];
  const int qq = blockIdx.x;
  if (st[qq].done) return;  // uniform
  const float* sr = scores + (int64_t)qq * ld_s;
  for (int b = threadIdx.x; b < SL_BINS; b += 256) lh[b] = 0u;
  for (int p = 2; p < 6; ++p) {
    __syncthreads();
    const SelState s = st[qq];
    if (s.done) return;  // uniform
    const int shift = kSlShift[p], width = kSlWidth[p], hs = shift + width;
    const uint32_t mask = (1u << width) - 1u;
    for (int64_t r = threadIdx.x; r < n; r += 256) {
      const uint64_t key = sel_key(sr[r], r);
      if ((key >> hs) == s.prefix) atomicAdd(&lh[(uint32_t)(key >> shift) & mask], 1u);
    }
    __syncthreads();
    sel_digit(p, k, s, st + qq, lh, part);  // clears lh for the next pass
    __threadfence_block();
  }
}

// Keys >= thr (k .. SL_CAP of them) -> the query's candidate list: gathered per block in LDS,
// then one global atomic per block reserves its slots (an atomic per taking wave on the one
// counter serialised ~1k atomics from every CU: 19 us at k = 1000, 1M rows).
__global__ __launch_bounds__(256) void k_sel_collect(const float* __restrict__ scores,
                                                     int64_t ld_s, int64_t n,
                                                     SelState* __restrict__ st,
                                                     uint64_t* __restrict__ cand) {
  __shared__ uint64_t lbuf[SL_CAP];
  __shared__ int lcnt, lbase;
  const int qq = blockIdx.y;
  if (threadIdx.x == 0) lcnt = 0;
  __syncthreads();
  const uint64_t thr = st[qq].thr;
  const float* sr = scores + (int64_t)qq * ld_s;
  const int64_t r0 = (int64_t)blockIdx.x * SL_CHUNK;
  const int64_t r1 = r0 + SL_CHUNK < n ? r0 + SL_CHUNK : n;
#pragma unroll 8
  for (int64_t r = r0 + threadIdx.x; r < r1; r += 256) {
    const uint64_t key = sel_key(sr[r], r);
    if (key >= thr) {
      const int slot = atomicAdd(&lcnt, 1);
      if (slot < SL_CAP) lbuf[slot] = key;  // bounds: at most SL_CAP keys >= thr in all
    }
  }
  __syncthreads();
  const int c = lcnt < SL_CAP ? lcnt : SL_CAP;
  if (c == 0) return;  // uniform
  if (threadIdx.x == 0) lbase = atomicAdd(&st[qq].ncand, c);
  __syncthreads();
  uint64_t* cq = cand + (int64_t)qq * SL_CAP;
  for (int e = threadIdx.x; e < c; e += 256)
    if (lbase + e < SL_CAP) cq[lbase + e] = lbuf[e];
}

// One block per query: the candidate keys (k .. SL_CAP, unique) are cut into 4 runs, one per
// wave, each sorted descending in registers (bitonic_desc: DPP exchanges for most stages);
// a key's final position is its index in its run plus, for each other run, the number of
// keys above it there (binary search of that run in LDS) -- the first k positions are written
// as (score, row).  NaN scores (key word 0) read (-inf, -1), as in the scan.  (A bitonic
// network over all keys in LDS: 21 us at k = 1000; one wave sorting 2048 keys: 51 us.)
template <int PER>
__device__ __forceinline__ void sel_sort_runs(const uint64_t* __restrict__ cq, int c, int k,
                                              uint64_t* ks, int64_t row_base, float* os,
                                              int64_t* oi) {
  constexpr int R = 64 * PER;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  uint64_t key[PER];
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const int e = w * R + lane * PER + r;
    key[r] = e < c ? cq[e] : 0ull;
  }
  bitonic_desc<PER>(key, lane);
#pragma unroll
  for (int r = 0; r < PER; ++r) ks[w * R + lane * PER + r] = key[r];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const uint64_t x = key[r];
    if (x == 0ull) continue;  // padding (every real key is nonzero: its row word is ~row)
    int rank = lane * PER + r;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      if (v == w) continue;
      const uint64_t* run = ks + v * R;
      int lo = 0, hi = R;  // keys of run v above x: the first index holding a key < x
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (run[mid] > x) lo = mid + 1;
        else hi = mid;
      }
      rank += lo;
    }
    if (rank < k) {
      const uint32_t hi32 = (uint32_t)(x >> 32);
      os[rank] = hi32 != 0u ? key_float(hi32) : -__builtin_huge_valf();
      oi[rank] = hi32 != 0u ? row_base + (int64_t)key_row(x) : -1;
    }
  }
}

__global__ __launch_bounds__(256) void k_sel_sort(const SelState* __restrict__ st,
                                                  const uint64_t* __restrict__ cand, int k,
                                                  int64_t row_base, float* __restrict__ out_s,
                                                  int64_t* __restrict__ out_i, int64_t q0) {
  __shared__ uint64_t ks[SL_CAP];
  const int qq = blockIdx.x;
  int c = st[qq].ncand;
  c = c < SL_CAP ? c : SL_CAP;
  float* os = out_s + (q0 + qq) * (int64_t)k;
  int64_t* oi = out_i + (q0 + qq) * (int64_t)k;
  for (int e = c + threadIdx.x; e < k; e += 256) {  // never taken: the collect gathers >= k
    os[e] = -__builtin_huge_valf();
    oi[e] = -1;
  }
  const uint64_t* cq = cand + (int64_t)qq * SL_CAP;
  if (c <= 4 * 256) sel_sort_runs<4>(cq, c, k, ks, row_base, os, oi);
  else sel_sort_runs<8>(cq, c, k, ks, row_base, os, oi);
}

static int sel_pad_dim(int d) {
  const int ep[] = {64, 128, 256, 384, 512, 768};
  for (int e : ep)
    if (d <= e) return e;
  return -1;
}

struct SelPlan {
  int qc;         // queries per chunk
  int64_t ld_s;   // score row stride (floats)
};

static SelPlan plan_select(int64_t n, int nq) {
  SelPlan p;
  p.ld_s = (n + 3) / 4 * 4;
  int64_t qc = SL_SCORE_BUDGET / (p.ld_s * 4);
  qc = qc >= 64 ? qc / 64 * 64 : (qc >= 16 ? qc / 16 * 16 : 16);
  p.qc = (int)(qc < nq ? qc : nq);
  return p;
}

}  // namespace tt

using namespace tt;

extern "C" int tt_select_workspace_bytes(int64_t n, int32_t nq, int32_t k, int64_t* bytes) {
  TT_REQUIRE(bytes != nullptr, "bytes == NULL");
  TT_REQUIRE(n >= 1 && nq >= 1 && k >= 1, "n, nq, k must be >= 1");
  const SelPlan p = plan_select(n, nq);
  const int64_t b = (int64_t)p.qc * p.ld_s * 4 + (int64_t)p.qc * SL_BINS * 4 +
                    (int64_t)p.qc * (int64_t)sizeof(SelState) + (int64_t)p.qc * SL_CAP * 8;
  *bytes = (b + 4 * 256 + 255) / 256 * 256;
  return TT_OK;
}

extern "C" int tt_scan_topk_select_f32(const float* db, int64_t n, int32_t d, int64_t ld_db,
                                       int64_t row_base, const float* q, int32_t nq,
                                       int64_t ld_q, int32_t k, float* out_score,
                                       int64_t* out_idx, void* workspace,
                                       int64_t workspace_bytes, void* stream) {
  TT_REQUIRE(n >= 1, "empty catalog");
  TT_REQUIRE(n <= 0x7fffffffLL, "shard rows must fit int32");
  TT_REQUIRE(nq >= 0, "nq < 0");
  TT_REQUIRE(k >= 1 && k <= n, "need 1 <= k <= n");
  if (nq == 0) return TT_OK;
  if (k > SL_KMAX) return fail(TT_ERR_UNSUPPORTED, "tt_scan_topk_select_f32: k > 1024");
  const int ep = sel_pad_dim(d);
  if (ep < 0) return fail(TT_ERR_UNSUPPORTED, "tt_scan_topk_select_f32: d > 768");
  TT_REQUIRE(ld_db >= ep && ld_q >= ep, "ld must be >= tt_padded_dim(d) (zero padded)");
  TT_REQUIRE(ld_db % 4 == 0 && ld_q % 4 == 0, "ld must be a multiple of 4");
  TT_REQUIRE(((uintptr_t)db % 16) == 0 && ((uintptr_t)q % 16) == 0, "db/q must be 16-B aligned");
  TT_REQUIRE(out_score && out_idx, "null output");
  int64_t need = 0;
  tt_select_workspace_bytes(n, nq, k, &need);
  if (workspace == nullptr || workspace_bytes < need)
    return fail(TT_ERR_WORKSPACE, "tt_scan_topk_select_f32: workspace too small");
  const SelPlan p = plan_select(n, nq);
  char* wsb = (char*)(((uintptr_t)workspace + 255) / 256 * 256);
  float* scores = (float*)wsb;
  uint32_t* hist = (uint32_t*)(wsb + (int64_t)p.qc * p.ld_s * 4);
  SelState* st = (SelState*)(hist + (int64_t)p.qc * SL_BINS);
  uint64_t* cand = (uint64_t*)(st + p.qc);
  hipStream_t s = (hipStream_t)stream;
  const int nchunk = (int)((n + SL_CHUNK - 1) / SL_CHUNK);
  for (int q0 = 0; q0 < nq; q0 += p.qc) {
    const int qn = nq - q0 < p.qc ? nq - q0 : p.qc;
    const float* qp = q + (int64_t)q0 * ld_q;
    hipLaunchKernelGGL(k_sel_init, dim3(qn), dim3(256), 0, s, st, hist, k);
    int rc = check_launch("k_sel_init");
    if (rc) return rc;
    const bool share = qn > SL_QT;
    // SHARE: blocks of one wave per 16 queries (up to 4): a 32-query chunk runs 2-wave blocks,
    // more of them per CU, instead of 4-wave blocks with 2 waves idle
    const int swaves = share ? ((qn + SL_QT - 1) / SL_QT < 4 ? (qn + SL_QT - 1) / SL_QT : 4) : 4;
    const int qtiles = share ? (qn + swaves * SL_QT - 1) / (swaves * SL_QT) : 1;
    // row slabs: ~2k blocks' worth of waves over the query tiles; >= 512 rows per wave (split
    // waves: a 2048-row slab is 512 rows per wave; shared: every wave streams the whole slab)
    int64_t slabs = ((share ? 2048 : 1024) + qtiles - 1) / qtiles;
    int64_t rps = (n + slabs - 1) / slabs;
    const int64_t rmin = share ? 512 : TT_SEL_RMIN;
    rps = rps < rmin ? rmin : (rps + SL_ROWS - 1) / SL_ROWS * SL_ROWS;
    slabs = (n + rps - 1) / rps;
    const dim3 grid((unsigned)slabs, (unsigned)qtiles);
    const bool h0 = !share && qn == 1;
#define TT_SEL_CASE(E)                                                                          \
  case E:                                                                                       \
    if (share)                                                                                  \
      hipLaunchKernelGGL((k_sel_scores<E, true>), grid, dim3(64 * swaves), 0, s, db, n, ld_db,  \
                         qp, qn, ld_q, (int)rps, scores, p.ld_s, hist);                         \
    else if (h0)                                                                                \
      hipLaunchKernelGGL((k_sel_scores<E, false, true>), grid, dim3(256), 0, s, db, n, ld_db,   \
                         qp, qn, ld_q, (int)rps, scores, p.ld_s, hist);                         \
    else                                                                                        \
      hipLaunchKernelGGL((k_sel_scores<E, false>), grid, dim3(256), 0, s, db, n, ld_db, qp, qn, \
                         ld_q, (int)rps, scores, p.ld_s, hist);                                 \
    break;
    switch (ep) {
      TT_SEL_CASE(64)
      TT_SEL_CASE(128)
      TT_SEL_CASE(256)
      TT_SEL_CASE(384)
      TT_SEL_CASE(512)
      TT_SEL_CASE(768)
      default:
        return fail(TT_ERR_UNSUPPORTED, "tt_scan_topk_select_f32: bad padded dim");
    }
#undef TT_SEL_CASE
    rc = check_launch("k_sel_scores");
    if (rc) return rc;
    // two digits on the chip (the second almost always leaves <= SL_CAP keys at or above the
    // k-th key's bucket), the rest -- duplicates -- in the per-query tail
    for (int pass = 0; pass < 2; ++pass) {
      if (!(pass == 0 && h0)) {
        hipLaunchKernelGGL(k_sel_hist, dim3(nchunk, qn), dim3(256), 0, s, scores, p.ld_s, n,
                           pass, st, hist);
        rc = check_launch("k_sel_hist");
        if (rc) return rc;
      }
      hipLaunchKernelGGL(k_sel_digit, dim3(qn), dim3(256), 0, s, pass, k, st, hist);
      rc = check_launch("k_sel_digit");
      if (rc) return rc;
    }
    hipLaunchKernelGGL(k_sel_tail, dim3(qn), dim3(256), 0, s, scores, p.ld_s, n, k, st);
    rc = check_launch("k_sel_tail");
    if (rc) return rc;
    hipLaunchKernelGGL(k_sel_collect, dim3(nchunk, qn), dim3(256), 0, s, scores, p.ld_s, n, st,
                       cand);
    rc = check_launch("k_sel_collect");
    if (rc) return rc;
    hipLaunchKernelGGL(k_sel_sort, dim3(qn), dim3(256), 0, s, st, cand, k, row_base, out_score,
                       out_idx, (int64_t)q0);
    rc = check_launch("k_sel_sort");
    if (rc) return rc;
  }
  return TT_OK;
}
