// tt_select.hip -- exact top-k by scores-then-radix-select (gfx950): the large-k scan.
//
// Replaces faiss.IndexFlatIP.search for k in (128, 1024] (server.py:46 lets /retrieve ask for
// up to k = 1000; vector_db.py:160,196 pass k straight to the index).  tt_scan_topk_f32 keeps a
// sorted top-k list per (query, slab of a few thousand rows) and merges them: at k = 1000 a
// slab list holds a quarter of its slab, so the lists and their merge cost 24-29 ms per search
// of a 1M-row catalog.  Here every exact f32 score is written once (the scan's MFMA scoring
// loop: the canonical fma order, so the scores are the scan's bits) and each query's k-th
// largest 64-bit key -- float_key(score) << 32 | ~row, the scan's order: score descending,
// ties to the lower row, NaN last -- is found by an MSB-first radix select over its score row
// (11/11/10-bit digits of the score word, then of the row word only when the k-th score is
// tied and not all of its ties are needed).  The keys >= it are exactly the top k; one wave
// sorts them.  Launches per query chunk: init, scores, up to 6 x (histogram, digit), collect,
// sort -- each histogram / collect pass re-reads the chunk's score rows (4 B per row and
// query, L2 / MALL resident at 1M rows), the catalog is read once per 64-query tile.
#include "tt_common.hpp"

namespace tt {

constexpr int SL_BINS = 2048;
constexpr int SL_KMAX = 1024;
constexpr int SL_CHUNK = 8192;                       // score rows per histogram / collect block
constexpr int64_t SL_SCORE_BUDGET = 256ll << 20;     // bytes of score rows per query chunk
constexpr int SL_QT = 16;                            // queries per wave (MFMA N)
constexpr int SL_ROWS = 32;                          // rows per wave step
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
// MFMA B operand, two 16-row blocks per step), so score[q][r] has the scan's bits.  SHARE
// (more than 16 queries): the block's 4 waves own 16 queries each and stream the same rows;
// otherwise one 16-query tile whose rows the 4 waves split.
template <int EP, bool SHARE>
__global__ __launch_bounds__(256, EP <= 384 ? 2 : 1) void k_sel_scores(
    const float* __restrict__ db, int64_t n, int64_t ld_db, const float* __restrict__ q, int nq,
    int64_t ld_q, int rows_per_slab, float* __restrict__ scores, int64_t ld_s) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ql = lane & 15, g = lane >> 4;
  const int qbase = blockIdx.y * (SHARE ? 4 * SL_QT : SL_QT) + (SHARE ? w * SL_QT : 0);
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
  const int64_t first = SHARE ? s0 : s0 + (int64_t)SL_ROWS * w;
  const int64_t stride = SHARE ? SL_ROWS : 4 * SL_ROWS;
  for (int64_t rb = first; rb < s1; rb += stride) {
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
    // D[row 4g + j][query ql]: acc0 -> rows rb + 4g + j, acc1 -> rows rb + 16 + 4g + j
    if (qvalid) {
      const int64_t r0 = rb + 4 * g, r1 = rb + 16 + 4 * g;
      if (r1 + 3 < s1) {
        *(f32x4*)(srow + r0) = acc0;
        *(f32x4*)(srow + r1) = acc1;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (r0 + j < s1) srow[r0 + j] = acc0[j];
          if (r1 + j < s1) srow[r1 + j] = acc1[j];
        }
      }
    }
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
// the next pass.  When bin d holds exactly krem keys all of them are in the top k: done, and
// every key >= (prefix . d) << shift is selected.
__global__ __launch_bounds__(256) void k_sel_digit(int p, SelState* __restrict__ st,
                                                   uint32_t* __restrict__ hist) {
  __shared__ uint32_t part[256];
  const int qq = blockIdx.x, t = threadIdx.x;
  const SelState s = st[qq];
  if (s.done) return;  // uniform
  uint32_t* gh = hist + (int64_t)qq * SL_BINS;
  uint32_t h[8];
  uint32_t sum = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    h[i] = gh[8 * t + i];
    sum += h[i];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) gh[8 * t + i] = 0u;
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
      if (h[i] == krem - above || p == 5) {
        o.done = 1;
        o.thr = o.prefix << shift;
      }
      st[qq] = o;
    }
    above += h[i];
  }
}

// Keys >= thr (exactly k of them) -> the query's candidate list (wave-aggregated slots).
__global__ __launch_bounds__(256) void k_sel_collect(const float* __restrict__ scores,
                                                     int64_t ld_s, int64_t n,
                                                     SelState* __restrict__ st,
                                                     uint64_t* __restrict__ cand) {
  const int qq = blockIdx.y, lane = threadIdx.x & 63;
  const uint64_t thr = st[qq].thr;
  const float* sr = scores + (int64_t)qq * ld_s;
  const int64_t r0 = (int64_t)blockIdx.x * SL_CHUNK;
  const int64_t r1 = r0 + SL_CHUNK < n ? r0 + SL_CHUNK : n;
  uint64_t* cq = cand + (int64_t)qq * SL_KMAX;
  // every lane runs the same trip count (ballots need the whole wave)
  for (int64_t rw = r0 + (threadIdx.x & ~63); rw < r1; rw += 256) {
    const int64_t r = rw + lane;
    const uint64_t key = r < r1 ? sel_key(sr[r], r) : 0ull;
    const bool take = r < r1 && key >= thr;
    const uint64_t m = __ballot(take);
    if (m) {
      int base = 0;
      if (lane == 0) base = atomicAdd(&st[qq].ncand, __popcll(m));
      base = __shfl(base, 0, 64);
      if (take) {
        const int slot = base + __popcll(m & ((1ull << lane) - 1ull));
        if (slot < SL_KMAX) cq[slot] = key;  // bounds: never more than k by construction
      }
    }
  }
}

// One wave per query: sort the k candidate keys (descending) and write (score, row).  NaN
// scores (key word 0) read (-inf, -1), as in the scan.
__global__ __launch_bounds__(64) void k_sel_sort(const SelState* __restrict__ st,
                                                 const uint64_t* __restrict__ cand, int k,
                                                 int64_t row_base, float* __restrict__ out_s,
                                                 int64_t* __restrict__ out_i, int64_t q0) {
  constexpr int PER = SL_KMAX / 64;
  const int qq = blockIdx.x, lane = threadIdx.x;
  int c = st[qq].ncand;
  c = c < SL_KMAX ? c : SL_KMAX;
  const uint64_t* cq = cand + (int64_t)qq * SL_KMAX;
  uint64_t key[PER];
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const int e = lane * PER + r;
    key[r] = e < c ? cq[e] : 0ull;
  }
  bitonic_desc<PER>(key, lane);
  float* os = out_s + (q0 + qq) * (int64_t)k;
  int64_t* oi = out_i + (q0 + qq) * (int64_t)k;
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const int e = lane * PER + r;
    if (e < k) {
      const uint32_t hi = (uint32_t)(key[r] >> 32);
      const bool ok = hi != 0u && e < c;
      os[e] = ok ? key_float(hi) : -__builtin_huge_valf();
      oi[e] = ok ? row_base + (int64_t)key_row(key[r]) : -1;
    }
  }
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
                    (int64_t)p.qc * (int64_t)sizeof(SelState) + (int64_t)p.qc * SL_KMAX * 8;
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
    const int qtiles = share ? (qn + 4 * SL_QT - 1) / (4 * SL_QT) : 1;
    // row slabs: >= 2 blocks per CU over the query tiles, slabs of >= 2048 rows
    int64_t slabs = (1024 + qtiles - 1) / qtiles;
    int64_t rps = (n + slabs - 1) / slabs;
    rps = rps < 2048 ? 2048 : (rps + SL_ROWS - 1) / SL_ROWS * SL_ROWS;
    slabs = (n + rps - 1) / rps;
    const dim3 grid((unsigned)slabs, (unsigned)qtiles);
#define TT_SEL_CASE(E)                                                                          \
  case E:                                                                                       \
    if (share)                                                                                  \
      hipLaunchKernelGGL((k_sel_scores<E, true>), grid, dim3(256), 0, s, db, n, ld_db, qp, qn,  \
                         ld_q, (int)rps, scores, p.ld_s);                                       \
    else                                                                                        \
      hipLaunchKernelGGL((k_sel_scores<E, false>), grid, dim3(256), 0, s, db, n, ld_db, qp, qn, \
                         ld_q, (int)rps, scores, p.ld_s);                                       \
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
    for (int pass = 0; pass < 6; ++pass) {
      hipLaunchKernelGGL(k_sel_hist, dim3(nchunk, qn), dim3(256), 0, s, scores, p.ld_s, n, pass,
                         st, hist);
      rc = check_launch("k_sel_hist");
      if (rc) return rc;
      hipLaunchKernelGGL(k_sel_digit, dim3(qn), dim3(256), 0, s, pass, st, hist);
      rc = check_launch("k_sel_digit");
      if (rc) return rc;
    }
    hipLaunchKernelGGL(k_sel_collect, dim3(nchunk, qn), dim3(256), 0, s, scores, p.ld_s, n, st,
                       cand);
    rc = check_launch("k_sel_collect");
    if (rc) return rc;
    hipLaunchKernelGGL(k_sel_sort, dim3(qn), dim3(64), 0, s, st, cand, k, row_base, out_score,
                       out_idx, (int64_t)q0);
    rc = check_launch("k_sel_sort");
    if (rc) return rc;
  }
  return TT_OK;
}
