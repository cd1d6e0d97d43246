// tt_filter.hip -- exact top-k via a bf16 MFMA filter + exact float32 re-rank (gfx950).
//
// Same contract as tt_scan_topk_f32 (replaces faiss.IndexFlatIP.search,
// src/inference/vector_db.py:160,197): results are the top-k by the CANONICAL float32 score
// (tt_common.hpp), ties to the lower row -- bit-identical to the f32 scan.  The bf16 pass
// only decides WHICH rows need an exact score:
//
//   a(r) = bf16(x_r) . bf16(q) accumulated in f32 by v_mfma_f32_16x16x32_bf16.
//   |a(r) - s(r)| <= eps_q, computed per query by k_query_eps from the catalog bounds
//   X >= max||x_r||, R >= max||x_r - bf16(x_r)|| (tt_bf16_image_bounds):
//     x.q - x~.q~ = (x - x~).q + x~.(q - q~)          (Cauchy-Schwarz on both terms)
//     eps_q = R|q| + (X+R)|q - q~| + 2E 2^-23 (X+R)|q~| + E 2^-24 X|q|      (x 1.001)
//   The last two terms bound the f32 accumulation of a (any order, 2 roundings per add, each
//   faithful -- the MFMA's internal rounding mode is not specified, so 2^-23 not 2^-24) and of
//   the canonical fma chain s (round to nearest) over E = padded-dim terms.  Using the measured
//   rounding residuals instead of the worst case u = 2^-8 per operand keeps eps ~2x tighter
//   for real data while staying a bound.
//
// Pipeline per call (all on the stream, no host sync, DESIGN.md "Scan v2"):
//   1. levels L = coarse..fine over nested strided row samples (stride 16^L, last = 1).
//      k_filter_bf16 appends every sample row with a >= theta_q to per-(query, slab)
//      candidate lists; k_select sorts a query's candidates and sets theta for the next
//      level = k-th best a of this sample (a lower bound of the k-th best a of any superset).
//      The last level filters with theta = T - 2*eps, and k_select keeps the band
//      a >= A_k - 2*eps, where A_k = k-th best a over the whole catalog.  Every row of the
//      exact top-k has a >= s - eps >= s_k - eps >= A_k - 2*eps, so the band contains it.
//   2. k_rerank computes the canonical f32 score of every band row (gathered from the f32
//      catalog), sorts (score desc, row asc) and writes the top-k.
//   3. A query whose candidate lists overflow is flagged, appended to a device-side list, and
//      served by the exact f32 scan kernel (tt_scan.hip) in a fallback launch whose blocks
//      exit immediately when the list is empty.
#include "tt_common.hpp"

#include <type_traits>

namespace tt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int FL_WAVES = 4;
constexpr int FL_CAP = 256;     // entries per (query, slab) list
constexpr int SEL_CAP = 4096;   // candidates per query a level may produce
constexpr int BAND_CAP = 1024;  // rows per query in the final band
constexpr int FL_KMAX = 128;
constexpr int SH_P = TT_SHARD_PROBES;  // sharded: count probes per query

// Sharded probe thresholds t_i = theta + i (smax - theta) / SH_P, i < SH_P (t_0 = theta).
// Identical expression in the counting (k_select_wave mode 2) and cutting (k_probe_cut)
// kernels: the cut is sound only for a t_i whose counts were taken with the same float.
__device__ __forceinline__ float probe_t(float theta, float smax, int i) {
  const float span = smax - theta;
  const float step = (span > 0.0f && span < __builtin_huge_valf()) ? span * (1.0f / SH_P) : 0.0f;
  return fmaf((float)i, step, theta);
}

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f32_to_bf16_rne(lo) | ((uint32_t)f32_to_bf16_rne(hi) << 16);
}


// --------------------------------------------------------------------------- filter
// Block: FL_WAVES waves over the same slab rows; wave w owns QB*16 queries (B fragments of
// v_mfma_f32_16x16x32_bf16 in VGPRs).  A fragments (16 rows x 32 dims) are streamed straight
// from HBM: lane l loads 16 B of row (l&15) at dims 32s + 8(l>>4).
template <int EP, int QB>
__global__ __launch_bounds__(64 * FL_WAVES, 2) void k_filter_dense(
    const uint16_t* __restrict__ xb, int64_t n, int64_t ld, const float* __restrict__ q,
    int nq, int64_t ldq, const float* __restrict__ theta, int64_t stride, int64_t n_sample,
    int rows_per_slab, int n_slabs, int n_qt, uint64_t* __restrict__ lists,
    int* __restrict__ counts) {
  constexpr int KS = EP / 32;  // k-steps
  constexpr int QPW = 16 * QB;
  __shared__ int cnt[FL_WAVES][QPW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int slab = lb / n_qt, qt = lb % n_qt;
  const int qbase = qt * (FL_WAVES * QPW) + w * QPW;

  bf16x8 qf[QB][KS];
  float th[QB];
  bool qv[QB];
#pragma unroll
  for (int b = 0; b < QB; ++b) {
    const int qi = qbase + 16 * b + col;
    qv[b] = qi < nq;
    th[b] = qv[b] ? theta[qi] : __builtin_huge_valf();
    const float* qp = q + (int64_t)(qv[b] ? qi : 0) * ldq + 8 * g;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const f32x4 v0 = *(const f32x4*)(qp + 32 * s);
      const f32x4 v1 = *(const f32x4*)(qp + 32 * s + 4);
      u32x4 u = {pack_bf16x2(v0[0], v0[1]), pack_bf16x2(v0[2], v0[3]), pack_bf16x2(v1[0], v1[1]),
                 pack_bf16x2(v1[2], v1[3])};
      qf[b][s] = __builtin_bit_cast(bf16x8, u);
    }
  }
  if (lane < QPW) cnt[w][lane] = 0;
  wave_sync();

  const int64_t j0 = (int64_t)slab * rows_per_slab;
  const int64_t j1 = (j0 + rows_per_slab < n_sample) ? j0 + rows_per_slab : n_sample;
  if (j0 < j1) {
    auto row_ptr = [&](int64_t jb) {
      int64_t j = jb + col;
      j = j < j1 ? j : j1 - 1;
      return (const u32x4*)(xb + j * stride * ld) + g;  // 16 B = 8 bf16 at dims 8g..
    };
    // EP <= 512: the next 16-row block's A fragments are loaded before this block's MFMAs
    // (one block in flight per wave); EP = 768 has no VGPRs for that and relies on the
    // second wave per SIMD to cover the load latency.
    constexpr bool PREFETCH = EP <= 512;
    u32x4 cur[KS], nxt[PREFETCH ? KS : 1];
    {
      const u32x4* p = row_ptr(j0);
#pragma unroll
      for (int s = 0; s < KS; ++s) cur[s] = p[4 * s];
    }
    for (int64_t jb = j0; jb < j1; jb += 16) {
      const bool more = jb + 16 < j1;
      if constexpr (PREFETCH) {
        if (more) {
          const u32x4* p = row_ptr(jb + 16);
#pragma unroll
          for (int s = 0; s < KS; ++s) nxt[s] = p[4 * s];
        }
      }
      f32x4 acc[QB];
#pragma unroll
      for (int b = 0; b < QB; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const bf16x8 a = __builtin_bit_cast(bf16x8, cur[s]);
#pragma unroll
        for (int b = 0; b < QB; ++b)
          acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[b][s], acc[b], 0, 0, 0);
      }
      // lane holds a(row jb + 4g + jj, query qbase + 16b + col)
      uint32_t pass = 0;
#pragma unroll
      for (int b = 0; b < QB; ++b)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const bool ok = (jb + 4 * g + jj < j1) && (acc[b][jj] >= th[b]);
          pass |= ok ? (1u << (4 * b + jj)) : 0u;
        }
      if (__ballot(pass != 0) != 0ull) {
#pragma unroll
        for (int b = 0; b < QB; ++b) {
          const int qi = qbase + 16 * b + col;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            if (pass & (1u << (4 * b + jj))) {
              const int slot = atomicAdd(&cnt[w][16 * b + col], 1);
              if (slot < FL_CAP) {
                const int64_t r = (jb + 4 * g + jj) * stride;
                lists[((int64_t)qi * n_slabs + slab) * FL_CAP + slot] =
                    make_key(acc[b][jj], (uint32_t)r);
              }
            }
          }
        }
      }
      if (more) {
        if constexpr (PREFETCH) {
#pragma unroll
          for (int s = 0; s < KS; ++s) cur[s] = nxt[s];
        } else {
          const u32x4* p = row_ptr(jb + 16);
#pragma unroll
          for (int s = 0; s < KS; ++s) cur[s] = p[4 * s];
        }
      }
    }
  }
  wave_sync();
  if (lane < QPW) {
    const int qi = qbase + lane;
    if (qi < nq) counts[(int64_t)qi * n_slabs + slab] = cnt[w][lane];
  }
}


// --------------------------------------------------------------------------- ring filter
// The streaming filter for every level except the coarsest.  One 512-thread block (8 waves,
// one block per CU) owns 8*QPW queries and a slab of sample rows.  Catalog tiles of TR rows
// are DMA'd HBM -> LDS by all waves (global_load_lds_dwordx4, 1 KiB per wave-instruction)
// into a 4-slot ring, PD = 3 tiles ahead, waited with a counted vmcnt and a raw s_barrier
// (cdna_hip_programming.md section 5 "Pipelining across barriers").  Each wave reads the
// A fragments of a tile with ds_read_b128 (16-B chunks XOR-swizzled by row on the DMA SOURCE
// address, read with the same XOR: conflict-free) and runs RB x QB x KS MFMAs.  Candidates
// (a >= theta) go to an LDS pool that is flushed to the per-(query, slab) lists in HBM only
// when half full and at the end, so global stores almost never sit in the vmcnt queue in
// front of the ring's DMA.
template <int EP> struct RingCfg;
template <> struct RingCfg<64> { static constexpr int TR = 64, QB = 2; };
template <> struct RingCfg<128> { static constexpr int TR = 32, QB = 2; };
template <> struct RingCfg<256> { static constexpr int TR = 32, QB = 2; };
#ifndef TT_RING_HALF
#define TT_RING_HALF 0  // 4-wave blocks, 2 per CU (independent lockstep groups per CU)
#endif
#ifndef TT_RING_QB4
#define TT_RING_QB4 0  // 4-wave blocks, 1 per CU, 64 queries per wave (half the LDS reads/flop)
#endif
#ifndef TT_RING_W4QB
// One wave per SIMD (4-wave blocks, 1 per CU, up to 512 registers per lane): the batched full
// level at E = 384 keeps TT_RING_W4QB 16-query blocks per wave (the other instantiations twice
// their RingCfg blocks, so every level keeps its queries per block); 0 = two waves per SIMD.
#define TT_RING_W4QB 0
#endif
#ifndef TT_RING_ASM
// with TT_RING_W4QB: the <384, 1> MFMAs as inline asm with the query fragments (B) pinned in
// AGPRs (the compiler-scheduled form moves them between AGPRs and VGPRs around every MFMA)
#define TT_RING_ASM 0
#endif
template <> struct RingCfg<384> {
  static constexpr int TR = TT_RING_HALF ? 16 : 32, QB = TT_RING_QB4 ? 4 : 2;
};
template <> struct RingCfg<512> { static constexpr int TR = 16, QB = 1; };
template <> struct RingCfg<768> { static constexpr int TR = 16, QB = 1; };

// Experiment switches (timing-only builds, results WRONG when set): tools/exp_filter.sh
#ifndef TT_EXP_NOSEL
#define TT_EXP_NOSEL 0  // skip candidate selection
#endif
#ifndef TT_EXP_SEL_TIMING
#define TT_EXP_SEL_TIMING 0  // printf per-phase wall-clock ticks (100 MHz) of k_select_reg
#endif
#ifndef TT_EXP_SEL_STOP
#define TT_EXP_SEL_STOP 0  // timing only: k_select_reg stops after the gather (1) / search (2)
#endif
#ifndef TT_EXP_NOIDLE
#define TT_EXP_NOIDLE 0  // small batches: padding-only waves run the MFMA stream too (A/B)
#endif
#ifndef TT_EXP_FINAL_STOP
#define TT_EXP_FINAL_STOP 0  // timing only: k_final_topm returns after the collect (1) / select (2)
#endif
#ifndef TT_EXP_FINAL_TIMING
#define TT_EXP_FINAL_TIMING 0  // printf k_final_topm phase wall-clock ticks (100 MHz), block 0
#endif
#ifndef TT_EXP_TM_STATS
#define TT_EXP_TM_STATS 0  // printf per-block compaction / append counts and phase ticks (block 0, 100)
#endif
#ifndef TT_EXP_TM_SLOTS
#define TT_EXP_TM_SLOTS 4  // single-pass small batches: ring slots (A/B)
#endif
#ifndef TT_EXP_NOWRITE
#define TT_EXP_NOWRITE 0  // selection control flow without the LDS pool writes
#endif
#ifndef TT_EXP_PRIO
#define TT_EXP_PRIO 0  // s_setprio 1 for waves 4-7 (static priority for the younger half)
#endif
#ifndef TT_RING_EARLY
#define TT_RING_EARLY 1  // k_filter_ring: first ring DMAs before the query loads (0: after)
#endif
#ifndef TT_RING_NT
// Non-temporal (aux = 2) ring DMA.  1 (default): the small-batch full level (LVL 2: one query
// tile, so every catalog byte is read exactly once) -- one-buyer full level 0.139 -> 0.124 ms
// (5.6 -> 6.2 TB/s), batched level unchanged; 3 = every level: the batched full level, whose
// 40 query tiles re-read the catalog from L2/MALL, 6.85 -> 7.29 ms (A/B, same box).
#define TT_RING_NT 1
#endif
#ifndef TT_RR_STAGED
// k_rerank: 1 (default) = wave-cooperative 256-B row pieces through an LDS stage, 0 = each
// thread loads its own row (64 rows per wave-instruction): re-rank ~0.65 -> ~0.45 ms per 10k
// queries at 1M x 384 (search minus full level 1.34 -> 1.13-1.15 ms, A/B on two boxes)
#define TT_RR_STAGED 1
#endif
#ifndef TT_RR_PF
#define TT_RR_PF 1  // k_rerank staged: chunks loaded ahead (2: 128 more VGPRs, +0.28 ms)
#endif
#ifndef TT_RR_NT
#define TT_RR_NT 0  // k_rerank: band rows loaded non-temporal (A/B: re-rank 0.65 -> 1.75 ms)
#endif
#ifndef TT_RR_ONEPHASE
// k_rerank scores the whole band in one phase (default).  The two-phase form (0: P1 first, then
// only the rows of the rest that can still reach s1) gathers ~25% fewer rows but adds a
// dependent gather + barrier per query block: in-process A/B (tools/ab_inproc.py, 16 reps,
// configs[2]) search minus full level 1.108 -> 1.186 ms -- slower, kept as a switch.
#define TT_RR_ONEPHASE 1
#endif
#ifndef TT_EXP_MAXONLY
#define TT_EXP_MAXONLY 0  // per-block max + ballot only (no per-slot scan)
#endif
#ifndef TT_EXP_BLKTIME
// timing only: k_filter_ring<EP, 1> records per block (start, end wall clock, hardware id,
// XCC id, logical block) into g_blktime (tt_debug_blktimes): the launch's per-CU timeline
#define TT_EXP_BLKTIME 0
#endif
#ifndef TT_EXP_BLKTIME_LVL
#define TT_EXP_BLKTIME_LVL 1  // the k_filter_ring level (LVL) whose blocks TT_EXP_BLKTIME records
#endif
#if TT_EXP_BLKTIME
constexpr int BLKTIME_MAX = 8192;
__device__ unsigned long long g_blktime[BLKTIME_MAX * 4];
__device__ unsigned long long g_blkph[BLKTIME_MAX * 2];  // k_filter_ring: tile 0 landed, loop end
#endif
TT_CHECK_EXP(TT_EXP_NOSEL || TT_EXP_NOWRITE || TT_EXP_MAXONLY ||
                 TT_EXP_SEL_STOP || TT_EXP_SEL_TIMING || TT_EXP_FINAL_STOP ||
                 TT_EXP_FINAL_TIMING || TT_EXP_TM_STATS || TT_EXP_TM_SLOTS != 4 ||
                 TT_EXP_BLKTIME,
             "TT_EXP_* (results wrong / printf / untested schedule)");
// The batched full level at E = 512 / 768 (configs[4]'s k_filter_ring<768, 1>) keeps TWO
// 16-query blocks per wave (192 fragment registers at E = 768) with one k-step of fragment
// read-ahead: each A fragment read from LDS feeds 2 MFMAs instead of 1.  2M x 768 x 10k
// queries, A/B x2 on one box (tools/bench_ab.sh --dim 768): full level 28.95 / 29.18 ms (one
// block, 2 steps ahead) -> 26.13 / 26.50 (two blocks, 2 ahead) -> 23.23 / 23.32 ms (two
// blocks, 1 ahead) = 42% -> 53% of the bf16 peak; self-check bit-exact.  Two tiles in flight
// (3-slot ring) instead of three: 22.54 / 22.55 -> 22.27 / 22.44 ms.  The sample levels of a
// large batch (LVL 3) at E >= 512 keep two blocks as well (10M x 768 step 120.7 / 120.9 ->
// 118.1 / 118.1 ms, small batches unchanged; A/B x2 on one box).  Small batches (LVL 0 and 2, HBM-bound) keep ONE: with two, a 256-query
// batch read the catalog once instead of twice (2M x 768: 1.11 -> 0.91 ms), but batches of
// 16-64 ran 4-9% slower (one k-step of read-ahead leaves a lone live block's LDS latency
// exposed; two steps spill; interleaving the blocks over the waves did not help) -- so the
// levels have their own queries per block (ring_qpb_rt), and batches past one 128-query tile
// take the two-block full level (LVL 4) instead.
#ifndef TT_RING_QB_WIDE
#define TT_RING_QB_WIDE 2  // query blocks per wave of the batched full level at E = 512 / 768
#endif
#ifndef TT_RING_FD_WIDE
#define TT_RING_FD_WIDE 1  // its fragment read-ahead (0: the generic rule)
#endif
#ifndef TT_RING_PD_WIDE
#define TT_RING_PD_WIDE 2  // its ring tiles in flight (0: RG_PD)
#endif
TT_CHECK_EXP(TT_RING_HALF || TT_RING_QB4 || TT_RING_W4QB || TT_RING_ASM ||
                 TT_RING_QB_WIDE != 2 || TT_RING_FD_WIDE != 1 || TT_RING_PD_WIDE != 2 ||
                 TT_EXP_NOIDLE || TT_EXP_PRIO ||
                 TT_RING_NT != 1 || TT_RR_STAGED != 1 || TT_RR_PF != 1 || TT_RR_NT ||
                 !TT_RR_ONEPHASE,
             "a non-default ring/re-rank schedule (untested by the GPU suite)");
#ifndef TT_RING_PD
// ring tiles in flight; 4 (5 slots, the pool's flush mark lowered to fit LDS): 6.33 -> 6.49 ms
#define TT_RING_PD 3
#endif
TT_CHECK_EXP(TT_RING_PD != 3, "TT_RING_PD");
constexpr int RG_WAVES = (TT_RING_HALF || TT_RING_QB4 || TT_RING_W4QB) ? 4 : 8, RG_PD = TT_RING_PD,
              RG_SLOTS = RG_PD + 1;  // 3 in flight
// Pool entries per wave: a query block's scan appends at most 16 x TR <= 512 (16 x 32 rows, all
// passing); it starts with wn <= RG_WFLUSH, so its writes need no bounds check.
constexpr int RG_WFLUSH = TT_RING_PD > 3 ? 64 : 256;
constexpr int RG_WPOOL = RG_WFLUSH + (TT_RING_QB4 ? 1024 : 512);
constexpr int RG_POOL = RG_WPOOL * RG_WAVES;  // pool entries per block
constexpr int RG_BLOCKS_PER_CU = TT_RING_HALF ? 2 : 1;

// Per-instantiation shape (LVL: see k_filter_ring).  The batched full level at E = 384
// (bench.py's roofline kernel) keeps THREE 16-query blocks per wave (384 queries per block):
// each 24 KB catalog tile feeds 1.5x the MFMAs, so the per-tile DMA pieces, barrier and waits
// weigh 1/3 less and the A-fragment reads per MFMA drop from 1/2 to 1/3.  The query fragments
// (144 VGPRs) leave room for one k-step of fragment read-ahead and a 3-slot ring (2 tiles in
// flight: 1.5x the compute per tile covers the same lead time): 6.26-6.33 -> 5.99-6.02 ms
// (A/B x2, one box).  Small batches (LVL 2: one-buyer searches are HBM-bound and want 3 tiles
// in flight) and sample levels keep two blocks per wave.
#ifndef TT_RING_S3
#define TT_RING_S3 0  // 1: the large-batch sample level (LVL 3) at E = 384 with 3 query blocks too
#endif
TT_CHECK_EXP(TT_RING_S3, "TT_RING_S3");
template <int EP, int LVL>
struct RingK {
  static constexpr int QB = TT_RING_W4QB ? (EP == 384 && LVL == 1 ? TT_RING_W4QB
                                                                  : 2 * RingCfg<EP>::QB)
                            : (EP == 384 && (LVL == 1 || (LVL == 3 && TT_RING_S3)) &&
                               !TT_RING_HALF && !TT_RING_QB4)
                                ? 3
                            : (EP >= 512 && (LVL == 1 || LVL >= 3)) ? TT_RING_QB_WIDE
                                                                     : RingCfg<EP>::QB;
  static constexpr int PD = QB == 3 ? 2 : (EP >= 512 && LVL == 1 && TT_RING_PD_WIDE) ? TT_RING_PD_WIDE : RG_PD;
  static constexpr int SLOTS = PD + 1;
};
template <int EP, int LVL = 0>
constexpr int ring_qpb() { return RG_WAVES * 16 * RingK<EP, LVL>::QB; }
template <int EP, int LVL>
constexpr int ring_smem() {
  return RingK<EP, LVL>::SLOTS * RingCfg<EP>::TR * EP * 2 + RG_POOL * 8 +
         ring_qpb<EP, LVL>() * 4 + 16;
}

// queries per block of k_filter_ring<ep, lvl> (the host's plan must use the same shape), and
// the instantiation a ring level runs: sample levels 0 (small batch) / 3 (large batch), the
// full level 2 (small batch) / 1 (large batch, > RG_SMALL_NQ queries)
template <int LVL>
static int ring_qpb_ep(int ep) {
  return ep == 64 ? ring_qpb<64, LVL>() : ep == 128 ? ring_qpb<128, LVL>()
         : ep == 256 ? ring_qpb<256, LVL>() : ep == 384 ? ring_qpb<384, LVL>()
         : ep == 512 ? ring_qpb<512, LVL>() : ring_qpb<768, LVL>();
}
static int ring_qpb_rt(int ep, int lvl) {
  return lvl == 1 ? ring_qpb_ep<1>(ep) : lvl == 2 ? ring_qpb_ep<2>(ep)
         : lvl == 3 ? ring_qpb_ep<3>(ep) : lvl == 4 ? ring_qpb_ep<4>(ep) : ring_qpb_ep<0>(ep);
}
constexpr int RG_SMALL_NQ_H = 2048;  // = RG_SMALL_NQ (declared with the kernel below)
// 4 = the full level of a mid-size batch at E >= 512 (more than one 128-query tile of LVL 2)
static int ring_lvl(bool tmax, int nq, int ep) {
  if (tmax) return nq > RG_SMALL_NQ_H ? 3 : 0;
  return nq > RG_SMALL_NQ_H ? 1 : (ep >= 512 && nq > ring_qpb_ep<2>(ep)) ? 4 : 2;
}

// LDS ops of the ring kernel's append path, in inline asm: the compiler cannot prove they do
// not alias the in-flight global_load_lds and would otherwise precede each with vmcnt(0),
// draining the ring whenever a candidate is found.
__device__ __forceinline__ uint32_t lds_add_rtn(uint32_t addr, uint32_t v) {
  uint32_t r;
  asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(r) : "v"(addr), "v"(v) : "memory");
  return r;
}
__device__ __forceinline__ void lds_write64(uint32_t addr, uint64_t v) {
  asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_write32(uint32_t addr, uint32_t v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(addr), "v"(v) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// A-fragment reads issued by hand so that their lgkmcnt waits are counted: the compiler's own
// schedule drains lgkmcnt(0) after every pair of reads (serialising LDS latency into the MFMA
// stream).  lds_wait_tie<N> waits until at most N LDS operations are outstanding and ties the
// fragment registers through the wait, so no consumer can be scheduled above it.
template <int N, typename F, int I = 0>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, F, I + 1>(static_cast<F&&>(f));
  }
}


__device__ __forceinline__ void lds_barrier() {
  // LDS traffic retired + workgroup barrier, WITHOUT the vmcnt(0) that __syncthreads() adds
  // while a global_load_lds is in flight (it would drain the ring)
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// 2 eps_q from the query's squared norms |q|^2, |q~|^2, |q - q~|^2 (any summation order: the
// growth factor covers it).  The last two terms bound the f32 accumulations: E 2^-24 X|q| the
// canonical fma chain of s (v_fma_f32 / fmaf, round to nearest), 2E 2^-23 (X+R)|q~| the
// MFMA's accumulation of a, whose internal rounding is not specified: any faithful rounding
// (error < 1 ulp = 2^-23 relative, round-toward-zero included), two roundings per addition.
template <int EP>
__device__ __forceinline__ float query_eps2(float sq, float st, float sr, float X, float R) {
  const float grow = 1.0f + (float)(EP + 2) * 1.1920929e-07f, up = 1.0f + 2.4e-7f;
  const float nq_ = sqrtf(sq * grow) * up, nt = sqrtf(st * grow) * up, nr = sqrtf(sr * grow) * up;
  const float g24 = (float)EP * 5.9604645e-08f * 1.01f;  // E 2^-24 (first order + slack)
  const float g23 = 2.0f * g24;                           // E 2^-23
  const float e = R * nq_ + (X + R) * nr + 2.0f * g23 * (X + R) * nt + g24 * X * nq_;
  const float r = 2.0f * e * 1.001f;
  return r == r ? r : __builtin_huge_valf();  // a NaN query: widest band (never returned)
}

// 2 eps_q of one query, computed by one wave (every lane gets the value): the norms of q, of
// its bf16 image and of the residual (the ONE expression every path uses: k_query_eps, the
// single-pass small batches)
template <int EP>
__device__ __forceinline__ float query_eps2_wave(const float* __restrict__ qr, float X, float R,
                                                 int lane) {
  float sq = 0.0f, st = 0.0f, sr = 0.0f;
  for (int i = lane; i < EP; i += 64) {
    const float v = qr[i], vt = __uint_as_float((uint32_t)f32_to_bf16_rne(v) << 16);
    sq = fmaf(v, v, sq);
    st = fmaf(vt, vt, st);
    sr = fmaf(v - vt, v - vt, sr);
  }
  for (int o = 32; o > 0; o >>= 1) {
    sq += __shfl_xor(sq, o, 64);
    st += __shfl_xor(st, o, 64);
    sr += __shfl_xor(sr, o, 64);
  }
  return query_eps2<EP>(sq, st, sr, X, R);
}

// Threshold of the batched full level from the last sample level's a_J (= aref) and 2 eps:
// every row of the exact top k has a >= s_k - eps, so the level must keep {a >= s_k - eps}.
// It keeps {a >= aref - 1.25 eps} and k_rerank certifies afterwards, from exact scores, that
// s_k >= aref - eps / 8 (the k-th exact score of the band is a lower bound of s_k): then
// s_k - eps >= aref - 1.125 eps > theta (the eps / 8 gap dwarfs the f32 rounding of these
// expressions).  A query that does not certify takes the exact fallback.  In practice s_k is
// far above aref (aref ~ the 336th row, s_k the 100th), so nothing falls back, and the level
// keeps ~484 instead of ~592 candidates per query at 1M x 384 (aref - 2 eps until round 4;
// tools/band_analysis.py restates the count).
#ifndef TT_FULL_THETA_2EPS
#define TT_FULL_THETA_2EPS 0  // timing builds: the round-4 threshold aref - 2 eps (A/B)
#endif
TT_CHECK_EXP(TT_FULL_THETA_2EPS, "TT_FULL_THETA_2EPS");
__device__ __forceinline__ float full_theta(float aref, float eps2) {
  return aref - (TT_FULL_THETA_2EPS ? 1.0f : 0.625f) * eps2;
}
__device__ __forceinline__ float full_cert(float aref, float eps2) { return aref - 0.0625f * eps2; }

// Per-query filter state, initialised by the first level of a search (k_query_eps's work,
// folded into that launch): eps2 from the catalog bounds X, R; aref = -inf; flags = 0;
// *qsel_n = 0.  eps2 == nullptr: a later level (theta read from the previous selection).
struct QueryInit {
  float X, R;
  float* eps2;
  float* aref;
  int* flags;
  int* qsel_n;
};

// LVL: 0 = a sample level of a small batch, 3 = a sample level of a large batch, 1 = the
// full-catalog (last) level of a large query batch (> RG_SMALL_NQ queries), 2 = the full level
// of a small batch, 4 = that of a mid-size batch at E >= 512 (ring_lvl) -- separate
// instantiations of
// the same code so that profiles attribute the dominant launch (bench.py's roofline kernel,
// 10k queries) on its own, apart from e.g. Mode A's 256-query searches.
constexpr int RG_SMALL_NQ = 2048;
static_assert(RG_SMALL_NQ == RG_SMALL_NQ_H, "one batch threshold");
template <int EP, int LVL>
__global__ __launch_bounds__(64 * RG_WAVES, RG_BLOCKS_PER_CU) void k_filter_ring(
    const uint16_t* __restrict__ xb, int64_t ld, const float* __restrict__ q, int nq,
    int64_t ldq, const float* __restrict__ theta, int64_t stride, int64_t n_sample,
    int rows_per_slab, int n_slabs, int n_qt, uint64_t* __restrict__ lists,
    int* __restrict__ counts, QueryInit qinit, const uint16_t* __restrict__ q16,
    int n_slabs_p, int rows_p) {
  constexpr int TR = RingCfg<EP>::TR, QB = RingK<EP, LVL>::QB;
  constexpr int RG_PD = RingK<EP, LVL>::PD, RG_SLOTS = RingK<EP, LVL>::SLOTS;
  constexpr int KS = EP / 32, QPW = 16 * QB, QPB = RG_WAVES * QPW;
  constexpr int CPR = EP / 8;  // 16-B chunks per row
  constexpr int TILE_B = TR * EP * 2;
  constexpr int PIECES = TILE_B / 1024, PPW = PIECES / RG_WAVES;
  constexpr int FM = (CPR >= 16 ? 16 : CPR) - 1;
  constexpr int RB = TR / 16;
  constexpr bool AMF = TT_RING_W4QB && TT_RING_ASM && EP == 384 && LVL == 1;
  constexpr bool SAMPLE = LVL == 0 || LVL == 3;  // a strided sample level (tile-max appends)
  constexpr int QSH = QPW <= 16 ? 4 : QPW <= 32 ? 5 : QPW <= 64 ? 6 : 7;  // pool entry: query bits
  static_assert((1 << QSH) >= QPW, "queries per wave fit the pool entry's query bits");
  static_assert(PIECES % RG_WAVES == 0, "tile must split into whole 1-KiB pieces per wave");
  __shared__ __attribute__((aligned(16))) char smem[ring_smem<EP, LVL>()];
  char* ring = smem;
  uint64_t* pool_key = (uint64_t*)(smem + RG_SLOTS * TILE_B);
  int* qcnt = (int*)(pool_key + RG_POOL);

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (TT_EXP_PRIO && w >= RG_WAVES / 2) __builtin_amdgcn_s_setprio(1);  // younger half (guide)
  const int col = lane & 15, g = lane >> 4;
  // Block -> (slab, query tile).  Uniform plan: XCD-contiguous ranges of (slab, tile) units,
  // the n_qt tiles of a slab adjacent (they share the slab's rows in L2).  Balanced plan
  // (n_slabs_p > 0, plan_balance): the last query tile is partial (e.g. 10k queries = 26 x 384
  // + 16) and costs about half a full block per row, so it has its own, coarser slabs
  // (n_slabs_p of rows_p rows, sized so its blocks cost about what a full block costs) and the
  // launch is exactly whole rounds of blocks; each XCD runs its share of the full tiles' units
  // first, then its share of the partial tile's.
  int slab, qt;
  int64_t rps = rows_per_slab;
  if (n_slabs_p > 0) {
    const int nfull = (n_qt - 1) * n_slabs, nblk = (int)gridDim.x;
    const int x = (int)blockIdx.x % 8, local = (int)blockIdx.x / 8;
    const int qf = nfull / 8, rf = nfull % 8, qb8 = nblk / 8, rb8 = nblk % 8;
    const int fx0 = x * qf + (x < rf ? x : rf), nfx = qf + (x < rf ? 1 : 0);
    const int px0 = x * qb8 + (x < rb8 ? x : rb8) - fx0;  // partial units of the XCDs before x
    if (local < nfx) {
      slab = (fx0 + local) / (n_qt - 1);
      qt = (fx0 + local) % (n_qt - 1);
    } else {
      slab = px0 + (local - nfx);
      qt = n_qt - 1;
      rps = rows_p;
    }
  } else {
    const int lb0 = xcd_remap(blockIdx.x, gridDim.x);
    slab = lb0 / n_qt;
    qt = lb0 % n_qt;
  }
  [[maybe_unused]] const int lb = slab * n_qt + qt;
  const int qbase = qt * QPB + w * QPW;
#if TT_EXP_BLKTIME
  const unsigned long long blk_t0 = wall_clock64();
  struct BlkTimeEnd {  // end stamp when the block's last wave leaves (any return path)
    unsigned long long t0;
    int lb;
    unsigned long long ph[2];
    __device__ ~BlkTimeEnd() {
      if (LVL != TT_EXP_BLKTIME_LVL || blockIdx.x >= BLKTIME_MAX) return;
      __syncthreads();
      if (threadIdx.x == 0) {
        g_blkph[2 * blockIdx.x] = ph[0];
        g_blkph[2 * blockIdx.x + 1] = ph[1];
        unsigned long long* o = g_blktime + 4 * blockIdx.x;
        o[0] = t0;
        o[1] = wall_clock64();
        o[2] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
        o[3] = ((unsigned long long)(unsigned)lb << 32) |
               (unsigned)__builtin_amdgcn_s_getreg((3 << 11) | 20);            // XCC_ID
      }
    }
  } blk_end{blk_t0, lb, {0ull, 0ull}};
#endif

  bf16x8 qf[QB][KS];
  float th[QB];

  const int64_t j0 = (int64_t)slab * rps;
  const int64_t j1 = (j0 + rps < n_sample) ? j0 + rps : n_sample;
  const int n_tiles = j0 < j1 ? (int)((j1 - j0 + TR - 1) / TR) : 0;

  // DMA of tile t into ring slot t % RG_SLOTS: piece p of the tile = LDS bytes [1024p, +1024),
  // lane i writes 16-B chunk P = 64p + i = (row r, position pos); its source is chunk
  // pos ^ (r & FM) of that row, so row r's logical chunk c lives at position c ^ (r & FM).
  // Per lane the (row, column byte) of each piece is loop-invariant.
  // sample levels read every stride-th row; the full level (LVL 1, 2) is the catalog itself
  const int64_t strd = SAMPLE ? stride : 1;
  const int64_t row_bytes = strd * ld * 2;
  // source = wave-uniform tile base (SGPRs) + the lane's 32-bit offset within the tile
  uint32_t voff[PPW];
#pragma unroll
  for (int pp = 0; pp < PPW; ++pp) {
    const int P = (w + RG_WAVES * pp) * 64 + lane;
    const int r = P / CPR;
    voff[pp] = (uint32_t)(r * row_bytes) + 16u * (uint32_t)((P % CPR) ^ (r & FM));
  }
  const int64_t tile_bytes = row_bytes * TR;
  const char* slab_base = (const char*)xb + j0 * row_bytes;
  // clamp: only the last tile of a ragged slab reads past j1 -- a separate instantiation
  // behind a scalar branch, so the common path is a uniform base + per-lane 32-bit offset
  // (the compiler had if-converted both paths into ~48 VALU selects per tile)
  // Each tile is read through a buffer resource based at the tile (scalar registers, TR rows
  // of range): the per-lane offset is the 32-bit voffset, so a piece costs no 64-bit VALU
  // address add (buffer_load_dwordx4 ... offen lds).
  auto issue_t = [&](int t, auto clamp_) __attribute__((always_inline)) {
    constexpr bool clamp = decltype(clamp_)::value;
    char* slot = ring + (t % RG_SLOTS) * TILE_B;
    const int64_t jt = j0 + (int64_t)t * TR;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(slab_base + (int64_t)t * tile_bytes), 0, (int)tile_bytes, 0x00020000);
#pragma unroll
    for (int pp = 0; pp < PPW; ++pp) {
      uint32_t off;
      if constexpr (!clamp) {
        off = voff[pp];
      } else {  // recompute the lane's (row, column) of piece pp: rare path, no live registers
        const int P = (w + RG_WAVES * pp) * 64 + lane;
        const int r = P / CPR;
        int64_t j = jt + r;
        j = j < j1 ? j : j1 - 1;
        off = (uint32_t)((j - jt) * row_bytes) + 16u * (uint32_t)((P % CPR) ^ (r & FM));
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(slot + (w + RG_WAVES * pp) * 1024), 16,
          off, 0, 0, ((TT_RING_NT >= 1 && (LVL == 2 || LVL == 4)) || TT_RING_NT >= 3) ? 2 : 0);
    }
  };
  auto issue = [&](int t) __attribute__((always_inline)) {
    if (j0 + (int64_t)(t + 1) * TR > j1) issue_t(t, std::true_type{});
    else issue_t(t, std::false_type{});
  };
  // the ring's first tiles go out BEFORE the queries are loaded (TT_RING_EARLY): the query
  // loads' latency and the first tiles' DMA latency overlap instead of adding up per block
  if (TT_RING_EARLY)
    for (int t = 0; t < RG_PD && t < n_tiles; ++t) issue(t);
  // this wave's queries as bf16 B-fragments (+ the first level's per-query state)
  const bool init = qinit.eps2 != nullptr;  // first level: theta = -inf, query state set here
  if (q16 != nullptr && !init) {
    // the bf16 query image (k_query_eps wrote it with this conversion): half the bytes of the
    // f32 rows and no branch between the loads, so all QB x KS fragment loads are in flight at
    // once (the f32 path's per-step conversion + first-level branch serialised them)
#pragma unroll
    for (int b = 0; b < QB; ++b) {
      const int qi = qbase + 16 * b + col;
      const bool v = qi < nq;
      th[b] = !v ? __builtin_huge_valf() : theta[qi];
      const uint16_t* qp = q16 + (int64_t)(v ? qi : 0) * EP + 8 * g;
#pragma unroll
      for (int s = 0; s < KS; ++s) qf[b][s] = *(const bf16x8*)(qp + 32 * s);
    }
  } else
#pragma unroll
  for (int b = 0; b < QB; ++b) {
    const int qi = qbase + 16 * b + col;
    const bool v = qi < nq;
    th[b] = !v ? __builtin_huge_valf() : init ? -__builtin_huge_valf() : theta[qi];
    const float* qp = q + (int64_t)(v ? qi : 0) * ldq + 8 * g;
    float sq = 0.0f, st = 0.0f, sr = 0.0f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const f32x4 v0 = *(const f32x4*)(qp + 32 * s);
      const f32x4 v1 = *(const f32x4*)(qp + 32 * s + 4);
      u32x4 u = {pack_bf16x2(v0[0], v0[1]), pack_bf16x2(v0[2], v0[3]), pack_bf16x2(v1[0], v1[1]),
                 pack_bf16x2(v1[2], v1[3])};
      qf[b][s] = __builtin_bit_cast(bf16x8, u);
      if (init && slab == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float x = i < 4 ? v0[i] : v1[i - 4];
          const uint32_t h = (u[i >> 1] >> (16 * (i & 1))) & 0xffffu;
          const float xt = __uint_as_float(h << 16);
          sq = fmaf(x, x, sq);
          st = fmaf(xt, xt, st);
          sr = fmaf(x - xt, x - xt, sr);
        }
      }
    }
    if (init && slab == 0) {  // lanes col, col+16, col+32, col+48 hold the query's 4 parts
      sq += __shfl_xor(sq, 16, 64);
      st += __shfl_xor(st, 16, 64);
      sr += __shfl_xor(sr, 16, 64);
      sq += __shfl_xor(sq, 32, 64);
      st += __shfl_xor(st, 32, 64);
      sr += __shfl_xor(sr, 32, 64);
      if (v && g == 0) {
        qinit.eps2[qi] = query_eps2<EP>(sq, st, sr, qinit.X, qinit.R);
        qinit.aref[qi] = -__builtin_huge_valf();
        qinit.flags[qi] = 0;
        qinit.qsel_n[1 + qi] = 0;  // done[qi] (FilterWs layout)
        if (qi == 0) *qinit.qsel_n = 0;
      }
    }
  }
  for (int i = tid; i < QPB; i += 64 * RG_WAVES) qcnt[i] = 0;
  // Candidate pool: each wave owns RG_WPOOL 8-byte entries and the counters of its own queries,
  // so appends need no atomics and no cross-wave synchronisation; the pool position `wn` is a
  // wave-uniform (scalar) count.  Entry = (orderable score << 32) | (row offset in the slab's
  // sample << QSH) | (query within the wave): one ds_write_b64 per candidate (the separate
  // query word of the first version cost a second write and its address).  Flush (rare):
  // per-(query, slab) list slots are assigned by LDS atomics on the wave's own counters, the
  // global key (score, ~row) rebuilt.  In-order LDS within a wave orders everything.
  uint64_t* wkey = pool_key + w * RG_WPOOL;
  uint32_t wn = 0;
  auto flush = [&]() __attribute__((always_inline)) {
    const int n = wn < (uint32_t)RG_WPOOL ? (int)wn : RG_WPOOL;
    for (int i = lane; i < n; i += 64) {
      const uint64_t e = wkey[i];
      const uint32_t lo = (uint32_t)e;
      const uint32_t ql = (uint32_t)(w * QPW) + (lo & ((1u << QSH) - 1));
      const uint32_t slot_i = lds_add_rtn(lds_addr(&qcnt[ql]), 1u);
      const uint32_t row = (uint32_t)((j0 + (int64_t)(lo >> QSH)) * strd);
      if (slot_i < (uint32_t)FL_CAP)
        lists[((int64_t)(qt * QPB + (int)ql) * n_slabs + slab) * FL_CAP + slot_i] =
            (e & 0xffffffff00000000ull) | (uint64_t)(~row);
    }
    wn = 0;
  };
  // A-fragment read offsets: row r = 16rb + col, chunk c = 4s + g = 16(u) .. with s = 4u + v,
  // so c ^ f = 4(s ^ h) + (g ^ (f & 3)) with f = r & FM, h = f >> 2  ->  the lane-dependent
  // part depends on v only; u becomes an immediate (+256u bytes).
  uint32_t lrd[RB][4];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int r = 16 * rb + col, f = r & FM, h = f >> 2;
#pragma unroll
    for (int v = 0; v < 4; ++v) lrd[rb][v] = 16 * (r * CPR + (g ^ (f & 3))) + 64 * (v ^ h);
  }

  // Fast reject of a finished tile (lane: RB*4 scores per query block): per-block maxima.
  // NaN scores (the t = 0 placeholder, NaN rows) never pass a >= test.
  auto tile_max = [&](const f32x4 (&sc)[RB][QB], float (&mx)[QB]) __attribute__((always_inline)) {
#pragma unroll
    for (int b = 0; b < QB; ++b) {
      float m = sc[0][b][0];
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) m = fmaxf(m, sc[rb][b][jj]);
      mx[b] = m;
    }
  };
  // orderable 32-bit image of a passing (so not NaN) score; -0 -> +0
  auto okey = [](float v) __attribute__((always_inline)) {
    const uint32_t u = __float_as_uint(v + 0.0f);
    return u ^ ((uint32_t)((int32_t)u >> 31) | 0x80000000u);
  };
  // the lane's part of a pool entry's low word: row 4g (+16 rb + jj) of the tile, query col
  const uint32_t lo_lane = ((uint32_t)(4 * g) << QSH) | (uint32_t)col;
  // Append the passing scores of tile t (lane: rows jt + 16rb + 4g + jj, query 16b + col).
  // One v_cmp + scalar branch per candidate slot; the lanes of a non-empty slot write at
  // wn + (passing lanes below).  The pool is flushed first if this block's scan could overrun
  // it (rare), so the writes carry no bounds check.  Rows past the slab end were set to -inf
  // when the tile finished.
  auto append = [&](const f32x4 (&sc)[RB][QB], const float (&mx)[QB], int t, int b_lo,
                    int b_hi) __attribute__((always_inline)) {
    const uint32_t lo_tile = lo_lane + ((uint32_t)(t * TR) << QSH);
#pragma unroll
    for (int b = 0; b < QB; ++b) {
      if (b < b_lo || b >= b_hi) continue;
      if (__ballot(mx[b] >= th[b]) == 0ull) continue;
      if (TT_EXP_MAXONLY) {
        asm volatile("" ::: "memory");
        continue;
      }
      if (wn > (uint32_t)RG_WFLUSH) flush();
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float v = sc[rb][b][jj];
          const uint64_t bm = __ballot(v >= th[b]);
          if (bm != 0ull) {
            if (!TT_EXP_NOWRITE && v >= th[b]) {
              const uint32_t pos = __builtin_amdgcn_mbcnt_hi(
                  (uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, wn));
              const uint32_t lo = lo_tile + ((uint32_t)(16 * rb + jj) << QSH) + 16u * b;
              lds_write64(lds_addr(&wkey[pos]), ((uint64_t)okey(v) << 32) | lo);
            }
            wn += (uint32_t)__popcll(bm);
          }
        }
    }
  };
  // Sample levels (LVL 0) only need the J-th best score of the sample, and the J-th largest
  // of the per-tile maxima is a lower bound of it (the top-J tile maxima are J distinct rows),
  // i.e. a sound threshold for the next level that is equal to a_J unless two of the top J
  // rows share a 32-row tile.  So a sample level appends ONE key per (query, tile): its max
  // (row id unused by the mode-0 selection) -- two cross-lane max steps and one ballot per
  // query block instead of 8 ballot rounds; at the stride-16 level ~95% of (tile, block)
  // pairs held a candidate.
  auto append_tmax = [&](const float (&mx)[QB], int t, int b_lo, int b_hi) __attribute__((always_inline)) {
    const uint32_t lo_t = ((uint32_t)(t * TR) << QSH) | (uint32_t)col;
    if (wn > (uint32_t)RG_WFLUSH) flush();  // <= 16 entries per block follow
#pragma unroll
    for (int b = 0; b < QB; ++b) {
      if (b < b_lo || b >= b_hi) continue;
      float m = mx[b];  // rows past the slab end are clamped copies of a real row: no mask
      m = fmaxf(m, __shfl_xor(m, 16, 64));
      m = fmaxf(m, __shfl_xor(m, 32, 64));
      const bool in = g == 0 && m >= th[b];
      const uint64_t bm = __ballot(in);
      if (bm == 0ull) continue;
      const uint32_t pos = __builtin_amdgcn_mbcnt_hi(
          (uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, wn));
      if (in) lds_write64(lds_addr(&wkey[pos]), ((uint64_t)okey(m) << 32) | (lo_t + 16u * b));
      wn += (uint32_t)__popcll(bm);
    }
  };
  // wait until only `younger` tiles issued after the awaited one are still in flight
  auto wait_tiles = [&](int younger) __attribute__((always_inline)) {
    if (younger >= 3) wait_vm<3 * PPW>();
    else if (younger == 2) wait_vm<2 * PPW>();
    else if (younger == 1) wait_vm<PPW>();
    else wait_vm<0>();
  };

  // Continuous MFMA stream over the slab: A fragments are read FD k-steps ahead into a
  // static register ring that runs ACROSS tile boundaries (the first FD steps of tile t+1
  // are read during the last FD steps of tile t), with hand-counted lgkmcnt waits.  Once per
  // tile, at step S_MID (before the first cross-tile read), every wave waits for its DMA
  // pieces of tile t+1, the block barriers (tile t+1 visible; every wave done with tile t-1),
  // and the slot of tile t-1 is refilled with tile t+PD.  The selection of tile t-1 (per-block
  // max mid-tile, then the candidate scan) runs between tile t's MFMAs.
  // FD + 1 divides KS (the ring index is s % (FD + 1)); 2 steps ahead where registers are tight
  // (three query blocks per wave: 6 MFMAs per k-step already cover one step of read-ahead,
  // and the fragment registers of a second step would spill)
  constexpr int FD = (EP >= 512 && (LVL == 1 || LVL >= 3) && TT_RING_FD_WIDE) ? TT_RING_FD_WIDE
                     : QB >= 3 ? 1 : (EP >= 384 && KS % 3 == 0) ? 2 : (KS >= 4 ? 3 : 1);
  static_assert(RG_SLOTS >= 3, "ring depth");
  constexpr int S_MID = (KS - FD) / 2;
  // Candidate scan of tile t-1 in one piece per query block, spread between tile t's MFMAs:
  // block P at step S0 + P * KS / QB (batched full level 6.81 -> 6.65 ms against all blocks at
  // step 1; S0 = 2 vs 1: 6.72 -> 6.64 ms; finer pieces and other spacings measured slower).
  // Sample levels append their tile maxima at step 1.
  constexpr int SP = KS / QB > 0 ? KS / QB : 1;
  constexpr int S0 = SAMPLE ? 1
                     : (QB > 1 && 2 + (QB - 1) * SP < KS) ? 2
                     : (QB > 1 && 1 + (QB - 1) * SP < KS) ? 1 : -1;  // -1: every block at step 1
  static_assert(KS % (FD + 1) == 0 && S_MID < KS - FD, "fragment ring layout");
  if (!TT_RING_EARLY)
    for (int t = 0; t < RG_PD && t < n_tiles; ++t) issue(t);
  wait_tiles(n_tiles - 1 < RG_PD - 1 ? n_tiles - 1 : RG_PD - 1);
  lds_barrier();  // tile 0 landed; counters initialised
#if TT_EXP_BLKTIME
  blk_end.ph[0] = wall_clock64();
#endif
  // A wave without a single real query only moves its share of the ring DMA, in lockstep with
  // the block's one barrier per tile: small batches (LVL 2, e.g. one buyer: its MFMAs on
  // padding queries had made the one-buyer full level issue-bound, 8 waves x 48 MFMAs / tile)
  // and the last, partial query tile of a large batch (LVL 1: 10k queries = 26 tiles of 384 +
  // 16, so 7 of that tile's 8 waves; its lone computing wave then has its SIMD to itself).
  if (qbase >= nq && !TT_EXP_NOIDLE) {
    for (int t = 0; t < n_tiles; ++t) {
      if (t + 1 < n_tiles) wait_tiles(n_tiles - 2 - t < RG_PD - 2 ? n_tiles - 2 - t : RG_PD - 2);
      asm volatile("s_barrier" ::: "memory");
      if (t + RG_PD < n_tiles) issue(t + RG_PD);
    }
    wait_vm<0>();
    return;
  }
  const float qnan = __builtin_nanf("");
  f32x4 accp[RB][QB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int b = 0; b < QB; ++b) accp[rb][b] = f32x4{qnan, qnan, qnan, qnan};

  // Fragment addresses: the tile loop is unrolled by RG_SLOTS so the slot of every tile is a
  // compile-time constant: slots 0-2 address from lrd, slots 3-4 from lrd + 3 TILE_B, and the
  // slot and k-step offsets are ds_read immediates (no address arithmetic in the loop).
  static_assert(RG_SLOTS <= 6 && 2 * TILE_B + 256 * (KS / 4) < 65536, "ds_read offset range");
  uint32_t lrd2[RB][4];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lrd[rb][i] += lds_addr(ring);
      lrd2[rb][i] = lrd[rb][i] + 3 * TILE_B;
    }
  u32x4 fr[FD + 1][RB];
  auto read_step = [&](auto slot_, auto sc_) __attribute__((always_inline)) {
    constexpr int SL = decltype(slot_)::value, S = decltype(sc_)::value;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
      fr[S % (FD + 1)][rb] = lds_read128<(SL % 3) * TILE_B + 256 * (S >> 2)>(
          SL >= 3 ? lrd2[rb][S & 3] : lrd[rb][S & 3]);
  };
  if (n_tiles > 0)
    static_for<FD>([&](auto s_) __attribute__((always_inline)) {
      read_step(std::integral_constant<int, 0>{}, s_);
    });
  for (int t0 = 0; t0 < n_tiles; t0 += RG_SLOTS) {
    static_for<RG_SLOTS>([&](auto u_) __attribute__((always_inline)) {
      constexpr int U = decltype(u_)::value;  // t % RG_SLOTS
      const int t = t0 + U;
      if (t < n_tiles) {
        const bool has_next = t + 1 < n_tiles;
        f32x4 acc[RB][QB];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
          for (int b = 0; b < QB; ++b) acc[rb][b] = f32x4{0.f, 0.f, 0.f, 0.f};
        float mx[QB];
        static_for<KS>([&](auto s_) __attribute__((always_inline)) {
          constexpr int s = decltype(s_)::value;
          if constexpr (s + FD < KS) {
            read_step(std::integral_constant<int, U>{}, std::integral_constant<int, s + FD>{});
            lds_wait<FD * RB>();
          } else {
            if (has_next) {
              read_step(std::integral_constant<int, (U + 1) % RG_SLOTS>{},
                        std::integral_constant<int, s + FD - KS>{});
              lds_wait<FD * RB>();
            } else {
              lds_wait<(KS - 1 - s) * RB>();
            }
          }
#pragma unroll
          for (int rb = 0; rb < RB; ++rb) reg_tie(fr[s % (FD + 1)][rb]);
#pragma unroll
          for (int rb = 0; rb < RB; ++rb) {
            const bf16x8 a = __builtin_bit_cast(bf16x8, fr[s % (FD + 1)][rb]);
#pragma unroll
            for (int b = 0; b < QB; ++b) {
              if constexpr (AMF) {
                const u32x4 au = fr[s % (FD + 1)][rb];
                if constexpr (s == 0)
                  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0"
                               : "=&v"(acc[rb][b]) : "v"(au), "a"(qf[b][s]));
                else
                  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                               : "+v"(acc[rb][b]) : "v"(au), "a"(qf[b][s]));
              } else {
                acc[rb][b] =
                    __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[b][s], acc[rb][b], 0, 0, 0);
              }
            }
          }
          if constexpr (s == 0) tile_max(accp, mx);  // VALU between this tile's MFMAs
          if constexpr (s == S_MID) {
            if (has_next) {
              // tiles issued after t+1 and still in flight: t+2 .. t+PD-1
              const int younger = n_tiles - 2 - t < RG_PD - 2 ? n_tiles - 2 - t : RG_PD - 2;
              wait_tiles(younger);
            }
            asm volatile("s_barrier" ::: "memory");
            if (t + RG_PD < n_tiles) issue(t + RG_PD);
          }
          if constexpr (SAMPLE || S0 < 0) {
            if constexpr (s == 1) {  // early: tile t-1's scores die before the peak
              if constexpr (SAMPLE) {
                if (!TT_EXP_NOSEL) append_tmax(mx, t - 1, 0, QB);
              } else {
                if (!TT_EXP_NOSEL) append(accp, mx, t - 1, 0, QB);
              }
            }
          } else if constexpr (s >= S0 && (s - S0) % SP == 0 && (s - S0) / SP < QB) {
            constexpr int P = (s - S0) / SP;
            if (!TT_EXP_NOSEL) append(accp, mx, t - 1, P, P + 1);
          }
          if (TT_EXP_NOSEL && s == 1) {
#pragma unroll
            for (int b = 0; b < QB; ++b)
              if (mx[b] >= th[b]) asm volatile("" ::: "memory");
          }
        });
        // (inline-asm MFMAs: the compiler does not see their results' VALU-read hazard)
        if constexpr (AMF) asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
          for (int b = 0; b < QB; ++b) accp[rb][b] = acc[rb][b];
        // the slab's last tile (full level): rows past j1 are clamped DMA copies of row j1 - 1
        if (!SAMPLE && j0 + (int64_t)(t + 1) * TR > j1) {
          const int lim = (int)(j1 - (j0 + (int64_t)t * TR));
#pragma unroll
          for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
              if (16 * rb + 4 * g + jj >= lim)
#pragma unroll
                for (int b = 0; b < QB; ++b) accp[rb][b][jj] = -__builtin_huge_valf();
        }
      }
    });
  }
#if TT_EXP_BLKTIME
  blk_end.ph[1] = wall_clock64();
#endif
  if (n_tiles > 0 && !TT_EXP_NOSEL) {
    float mx[QB];
    tile_max(accp, mx);
    if constexpr (SAMPLE) append_tmax(mx, n_tiles - 1, 0, QB);
    else append(accp, mx, n_tiles - 1, 0, QB);
  }
  wait_vm<0>();
  flush();
  lds_wait<0>();
  for (int i = lane; i < QPW; i += 64) {
    const int qi = qbase + i;
    if (qi < nq) {
      const uint32_t c = (uint32_t)qcnt[w * QPW + i];
      counts[(int64_t)qi * n_slabs + slab] =
          c > (uint32_t)FL_CAP ? FL_CAP + 1 : (int)c;
      // balanced plan: the partial tile's queries have n_slabs_p slabs, their lists keep the
      // n_slabs stride -- the slots past n_slabs_p read as empty
      if (n_slabs_p > 0 && qt == n_qt - 1)
        for (int s2 = slab + n_slabs_p; s2 < n_slabs; s2 += n_slabs_p)
          counts[(int64_t)qi * n_slabs + s2] = 0;
    }
  }
}

// --------------------------------------------------------------------------- select
__device__ void block_sort_desc(uint64_t* buf, int n_pow2) {
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

__device__ __forceinline__ int pow2_at_least(int v) {
  int p = 2;
  while (p < v) p <<= 1;
  return p;
}

__device__ void flag_query(int qid, int* flags, int* qsel, int* qsel_n) {
  if (atomicExch(&flags[qid], 1) == 0) {
    const int pos = atomicAdd(qsel_n, 1);
    qsel[pos] = qid;
  }
}

// mode 0 (sample level): theta_out[q] = aref[q] = a_J, the J-th best a of the sample (its
//   candidates are a superset of the sample's top J because theta <= a_J of a subset).
// mode 1 (full catalog): A_k = k-th best a.  The level was filtered with theta = aref - eps2;
//   that captures every row with a >= A_k - eps2 iff aref <= A_k: checked here, else the
//   query is flagged for the exact fallback.  band[q] = candidates with a >= A_k - eps2.
__global__ __launch_bounds__(256) void k_select(const uint64_t* __restrict__ lists,
                                                const int* __restrict__ counts, int n_slabs,
                                                int k, int J, const float* __restrict__ eps2,
                                                int mode,
                                                float* __restrict__ theta_out,
                                                float* __restrict__ aref,
                                                uint64_t* __restrict__ band, int* band_n,
                                                int* flags, int* qsel, int* qsel_n) {
  __shared__ uint64_t buf[SEL_CAP];
  __shared__ int total, bad;
  const int qid = blockIdx.x;
  if (threadIdx.x == 0) { total = 0; bad = flags[qid]; }
  __syncthreads();
  if (bad) {
    if (threadIdx.x == 0 && mode == 0) theta_out[qid] = __builtin_huge_valf();
    return;
  }
  const int* qc = counts + (int64_t)qid * n_slabs;
  for (int s = threadIdx.x; s < n_slabs; s += blockDim.x) {
    const int c = qc[s];
    if (c > FL_CAP) bad = 1;  // benign race: every writer stores 1
    else atomicAdd(&total, c);
  }
  __syncthreads();
  if (!bad && total > SEL_CAP) bad = 1;
  __syncthreads();
  if (bad) {
    if (threadIdx.x == 0) {
      flag_query(qid, flags, qsel, qsel_n);
      if (mode == 0) theta_out[qid] = __builtin_huge_valf();
    }
    return;
  }
  // gather: slab lists are contiguous per query -> walk (slab, slot) pairs
  __shared__ int fill;
  if (threadIdx.x == 0) fill = 0;
  __syncthreads();
  const uint64_t* ql = lists + (int64_t)qid * n_slabs * FL_CAP;
  for (int64_t e = threadIdx.x; e < (int64_t)n_slabs * FL_CAP; e += blockDim.x) {
    const int s = (int)(e / FL_CAP), i = (int)(e % FL_CAP);
    if (i < qc[s]) buf[atomicAdd(&fill, 1)] = ql[e];
  }
  __syncthreads();
  const int nb = total;
  const int np = pow2_at_least(nb);
  for (int i = nb + threadIdx.x; i < np; i += blockDim.x) buf[i] = 0ull;
  block_sort_desc(buf, np);
  if (mode == 0) {
    const float aj = nb >= J ? key_float((uint32_t)(buf[J - 1] >> 32)) : -__builtin_huge_valf();
    if (threadIdx.x == 0) {
      theta_out[qid] = aj;
      aref[qid] = aj;
    }
    return;
  }
  const float ak = nb >= k ? key_float((uint32_t)(buf[k - 1] >> 32)) : -__builtin_huge_valf();
  if (!(ak >= aref[qid])) {  // optimistic threshold did not hold (or fewer than k rows)
    if (threadIdx.x == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  // band = prefix of the sorted list with a >= ak - eps2 (NaN never enters the lists)
  const float thr = ak - eps2[qid];
  __shared__ int bn;
  if (threadIdx.x == 0) bn = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    const float a = key_float((uint32_t)(buf[i] >> 32));
    const bool in = a >= thr;
    const bool next_in = (i + 1 < nb) && key_float((uint32_t)(buf[i + 1] >> 32)) >= thr;
    if (in && !next_in) bn = i + 1;
  }
  __syncthreads();
  const int nband = bn;
  if (nband > BAND_CAP) {
    if (threadIdx.x == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  for (int i = threadIdx.x; i < nband; i += blockDim.x) band[(int64_t)qid * BAND_CAP + i] = buf[i];
  if (threadIdx.x == 0) band_n[qid] = nband;
}

// Wave-per-query selection (replaces the block sort): the candidate keys of a query are
// gathered into a wave-private LDS buffer, the R-th largest score (R = J or k) is found by a
// 32-step bitwise search on the orderable score bits (count of keys >= candidate, reduced
// across the wave), and -- full level -- the band a >= A_k - eps2 is compacted with
// ballot/mbcnt (unordered: k_rerank sorts by the exact score).  Same outputs as k_select.
constexpr int SW_CAP = 2048;  // candidates per query (more: the query takes the exact fallback)
__global__ __launch_bounds__(256) void k_select_wave(const uint64_t* __restrict__ lists,
                                                     const int* __restrict__ counts, int n_slabs,
                                                     int k, int J, const float* __restrict__ eps2,
                                                     int mode, float* __restrict__ theta_out,
                                                     float* __restrict__ aref,
                                                     uint64_t* __restrict__ band,
                                                     int* __restrict__ band_n, int* __restrict__ band_p1,
                                                     int* __restrict__ flags, int* qsel,
                                                     int* qsel_n, int nq,
                                                     const float* __restrict__ stats,
                                                     int* __restrict__ pcount,
                                                     float* __restrict__ smax_out,
                                                     int fin) {
  __shared__ uint64_t buf[4][SW_CAP];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int qid = blockIdx.x * 4 + w;
  if (qid >= nq) return;  // the whole wave (no block-level barriers below)
  uint64_t* kb = buf[w];
  if (mode == 2 && lane < SH_P) pcount[(int64_t)qid * SH_P + lane] = 0;  // overflow: count 0
  if (flags[qid]) {
    if (lane == 0 && mode == 0) theta_out[qid] = __builtin_huge_valf();
    return;
  }
  const int* qc = counts + (int64_t)qid * n_slabs;
  const uint64_t* ql = lists + (int64_t)qid * n_slabs * FL_CAP;
  // gather: lane = slab (64 slabs per pass); a wave scan of the slab counts gives each
  // lane its offset, then every lane copies its own slab's entries -- all list loads of a
  // pass are independent (no per-slab load -> offset dependency chain)
  int total = 0;
  bool bad = false;
  for (int s0 = 0; s0 < n_slabs && !bad; s0 += 64) {
    const int c = s0 + lane < n_slabs ? qc[s0 + lane] : 0;
    int incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o, 64);
      incl += lane >= o ? y : 0;
    }
    const int chunk = __shfl(incl, 63, 64);
    if (__ballot(c > FL_CAP) != 0ull || total + chunk > SW_CAP) {
      bad = true;
      break;
    }
    int mx = c;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
    const uint64_t* src = ql + (int64_t)(s0 + lane) * FL_CAP;
    uint64_t* dst = kb + total + incl - c;
    for (int j = 0; j < mx; j += 4) {
      uint64_t v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = j + u < c ? src[j + u] : 0ull;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (j + u < c) dst[j + u] = v[u];
    }
    total += chunk;
  }
  if (bad) {
    if (lane == 0) {
      flag_query(qid, flags, qsel, qsel_n);
      if (mode == 0) theta_out[qid] = __builtin_huge_valf();
    }
    return;
  }
  wave_sync();
  if (mode == 2) {
    // sharded full level: every candidate (a >= theta_g - eps2) is band; report the shard's
    // count of candidates a >= t_i at the SH_P probes (all-reduced SUM by the caller)
    const float th = stats[2 * qid], sm = stats[2 * qid + 1];
    int cnt[SH_P];
#pragma unroll
    for (int i = 0; i < SH_P; ++i) cnt[i] = 0;
    int nb = 0;
    uint64_t* qb = band + (int64_t)qid * BAND_CAP;
    for (int j0 = 0; j0 < total; j0 += 64) {
      const int j = j0 + lane;
      const bool in = j < total;
      const uint64_t key = in ? kb[j] : 0ull;
      const float a = key_float((uint32_t)(key >> 32));
#pragma unroll
      for (int i = 0; i < SH_P; ++i) cnt[i] += __popcll(__ballot(in && a >= probe_t(th, sm, i)));
      const uint64_t bm = __ballot(in);
      const int pos = nb + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
      if (in && pos < BAND_CAP) qb[pos] = key;
      nb += __popcll(bm);
    }
#pragma unroll
    for (int i = 0; i < SH_P; ++i)
      if (lane == i) pcount[(int64_t)qid * SH_P + i] = cnt[i];
    if (lane == 0) {
      if (nb > BAND_CAP) flag_query(qid, flags, qsel, qsel_n);  // this shard: exact fallback
      else band_n[qid] = nb;
    }
    return;
  }
  const int R = mode == 0 ? J : k;
  if (total < R) {  // fewer than R candidates: a_J = -inf (sample) / cannot certify (full)
    if (lane == 0) {
      if (mode == 0) {
        theta_out[qid] = -__builtin_huge_valf();
        aref[qid] = -__builtin_huge_valf();
        if (smax_out) smax_out[qid] = -__builtin_huge_valf();  // probes all at theta = -inf
      } else {
        flag_query(qid, flags, qsel, qsel_n);
      }
    }
    return;
  }
  constexpr int PER = SW_CAP / 64;
  const int ni = __builtin_amdgcn_readfirstlane((total + 63) / 64);
  uint32_t hv[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = lane + 64 * i;
    hv[i] = (i < ni && j < total) ? (uint32_t)(kb[j] >> 32) : 0u;  // 0 = below every key
  }
  uint32_t T = 0;
  for (int bit = 31; bit >= 0; --bit) {
    const uint32_t cand = T | (1u << bit);
    // wave count by ballot + scalar popcount (a 6-step shuffle reduction per bit was a
    // ~100-cycle dependent LDS chain: 32 of them dominated a lone query's selection)
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (i < ni) cnt += __popcll(__ballot(hv[i] >= cand));
    if (cnt >= R) T = cand;
  }
  const float A = key_float(T);
  if (mode == 0) {
    if (smax_out) {  // sharded: the sample's best a (upper end of the probe range)
      uint32_t m = 0;
#pragma unroll
      for (int i = 0; i < PER; ++i)
        if (i < ni) m = max(m, hv[i]);
      for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
      if (lane == 0) smax_out[qid] = key_float(m);
    }
    if (lane == 0) {  // fin: the next level is the full one -> its threshold (full_theta)
      theta_out[qid] = fin ? full_theta(A, eps2[qid]) : A;
      aref[qid] = A;
    }
    return;
  }
  if (!(A >= aref[qid])) {  // the optimistic threshold did not hold
    if (lane == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  const float thr = A - eps2[qid];
  int nb = 0;
  uint64_t* qb = band + (int64_t)qid * BAND_CAP;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    if (i < ni) {
      const int j = lane + 64 * i;
      const bool in = j < total && key_float(hv[i]) >= thr;
      const uint64_t bm = __ballot(in);
      const int pos = nb + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
      if (in && pos < BAND_CAP) qb[pos] = kb[j];
      nb += __popcll(bm);
    }
  }
  if (lane == 0) {
    if (nb > BAND_CAP) flag_query(qid, flags, qsel, qsel_n);
    else band_n[qid] = nb;
    band_p1[qid] = -1;  // unordered band: k_rerank scores it in one phase
  }
}

// Register-resident variant of k_select_wave (n_slabs <= 64; GROUPED: <= 1024, the
// small-batch levels' up-to-4-blocks-per-CU slabs, lane s owning slabs [sG, sG + G) with
// G = ceil(n_slabs / 64)).  Item e of the query's candidate sequence lives in lane e % 64,
// register e / 64; every list load of the query is issued before the first use, and the
// selection runs on registers.  Same outputs as k_select_wave.
constexpr int SR_GMAX = 16;
#ifndef TT_SEL_BOUND
#define TT_SEL_BOUND 1  // k_select_reg: bound + compaction before the bitwise search (0: off)
#endif
TT_CHECK_EXP(TT_SEL_BOUND != 1, "TT_SEL_BOUND");
template <bool GROUPED>
__global__ __launch_bounds__(256) void k_select_reg(const uint64_t* __restrict__ lists,
                                                    const int* __restrict__ counts, int n_slabs,
                                                    int k, int J, const float* __restrict__ eps2,
                                                    int mode, float* __restrict__ theta_out,
                                                    float* __restrict__ aref,
                                                    uint64_t* __restrict__ band,
                                                    int* __restrict__ band_n, int* __restrict__ band_p1,
                                                    int* __restrict__ flags, int* qsel,
                                                    int* qsel_n, int nq,
                                                    const float* __restrict__ stats,
                                                    int* __restrict__ pcount,
                                                    float* __restrict__ smax_out,
                                                    int fin) {
  const int lane = threadIdx.x & 63;
  const int qid = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (qid >= nq) return;  // the whole wave (no block-level barriers below)
#if TT_EXP_SEL_TIMING
  uint64_t tstamp[8];
  int ntst = 0;
  tstamp[ntst++] = wall_clock64();
#endif
  if (mode == 2 && lane < SH_P) pcount[(int64_t)qid * SH_P + lane] = 0;  // overflow: count 0
  if (flags[qid]) {
    if (lane == 0 && mode == 0) theta_out[qid] = __builtin_huge_valf();
    return;
  }

#if TT_EXP_SEL_TIMING
  tstamp[ntst++] = wall_clock64();
#endif
  const int* qc = counts + (int64_t)qid * n_slabs;
  const uint64_t* ql = lists + (int64_t)qid * n_slabs * FL_CAP;
  constexpr int GM = GROUPED ? SR_GMAX : 1;
  const int G = GROUPED ? (n_slabs + 63) / 64 : 1;  // slabs per lane
  const int wv = threadIdx.x >> 6;
  __shared__ uint16_t tbl_s[4][SW_CAP];     // item -> slab
  __shared__ int soff_s[4][64 * GM];        // slab -> first item
  int cj[GM];
  int c = 0;
  bool over = false;
#pragma unroll
  for (int j = 0; j < GM; ++j) {
    const int sj = lane * G + j;
    cj[j] = j < G && sj < n_slabs ? qc[sj] : 0;
    c += cj[j];
    over |= cj[j] > FL_CAP;
  }
  int incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, 64);
    incl += lane >= o ? y : 0;
  }
  // wave-uniform in SGPRs: loop guards on ni become scalar branches (as a VGPR value the
  // compiler had turned them into exec-masked regions with a VGPR counter)
  const int total = __builtin_amdgcn_readfirstlane(__shfl(incl, 63, 64));
  if (__ballot(over) != 0ull || total > SW_CAP) {
    if (lane == 0) {
      flag_query(qid, flags, qsel, qsel_n);
      if (mode == 0) theta_out[qid] = __builtin_huge_valf();
    }
    return;
  }
  constexpr int PER = SW_CAP / 64;
  const int ni = __builtin_amdgcn_readfirstlane((total + 63) / 64);

#if TT_EXP_SEL_TIMING
  tstamp[ntst++] = wall_clock64();
#endif
  uint32_t hv[PER], lo[PER];
  // item e of the query's candidate sequence (slabs in order) lives in lane e % 64, register
  // e / 64.  Each lane writes the slab id of its slabs' items into a wave-private LDS table
  // (plus each slab's first item); an item then needs two independent-per-item LDS reads to
  // address its list entry, so all of the query's list loads are in flight at once.  (A
  // per-item binary search over the lanes' offsets -- 6 dependent bpermutes -- made a lone
  // query's selection latency-bound: ~30-40 us.)
  {
    int o = incl - c;
#pragma unroll
    for (int j = 0; j < GM; ++j) {
      const int sj = lane * G + j;
      if (j < G && sj < n_slabs) {
        soff_s[wv][sj] = o;
        for (int t = 0; t < cj[j]; ++t) tbl_s[wv][o + t] = (uint16_t)sj;
        o += cj[j];
      }
    }
  }
  wave_sync();

#if TT_EXP_SEL_TIMING
  tstamp[ntst++] = wall_clock64();
#endif
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    hv[i] = 0u;  // 0 = below every key
    lo[i] = 0u;
    if (i < ni) {
      const int e = lane + 64 * i;
      if (e < total) {
        const int sl = tbl_s[wv][e];
        const uint64_t key = ql[(int64_t)sl * FL_CAP + (e - soff_s[wv][sl])];
        hv[i] = (uint32_t)(key >> 32);
        lo[i] = (uint32_t)key;
      }
    }
  }

#if TT_EXP_SEL_TIMING
  tstamp[ntst++] = wall_clock64();
#endif
#if TT_EXP_SEL_TIMING
  { uint32_t m = 0;
    for (int i = 0; i < PER; ++i) m ^= hv[i];
    if (m == 0x1234567u) theta_out[qid] = 1.f; }
  tstamp[ntst++] = wall_clock64();
#endif
  if (TT_EXP_SEL_STOP == 1) {  // timing only: stop after the gather
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i) m ^= hv[i] ^ lo[i];
    if (m == 0x12345u) theta_out[qid] = 0.f;
    return;
  }
  if (mode == 2) {
    // sharded full level: every candidate (a >= theta_g - eps2) is band; the shard's count of
    // candidates a >= t_i at the SH_P probes (all-reduced SUM by the caller).  The probe loop
    // stays rolled (unrolling it over the PER registers spilled).
    const float th = stats[2 * qid], sm = stats[2 * qid + 1];
#pragma unroll 1
    for (int t = 0; t < SH_P; ++t) {
      const float pt = probe_t(th, sm, t);
      int c = 0;
#pragma unroll
      for (int i = 0; i < PER; ++i)
        if (i < ni) c += __popcll(__ballot(lane + 64 * i < total && key_float(hv[i]) >= pt));
      if (lane == 0) pcount[(int64_t)qid * SH_P + t] = c;
    }
    int nb = 0;
    uint64_t* qb = band + (int64_t)qid * BAND_CAP;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      if (i < ni) {
        const bool in = lane + 64 * i < total;
        const uint64_t bm = __ballot(in);
        const int pos = nb + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
        if (in && pos < BAND_CAP) qb[pos] = ((uint64_t)hv[i] << 32) | lo[i];
        nb += __popcll(bm);
      }
    }
    if (lane == 0) {
      if (nb > BAND_CAP) flag_query(qid, flags, qsel, qsel_n);  // this shard: exact fallback
      else band_n[qid] = nb;
    }
    return;
  }
  const int R = mode == 0 ? J : k;
  if (total < R) {  // fewer than R candidates: a_J = -inf (sample) / cannot certify (full)
    if (lane == 0) {
      if (mode == 0) {
        theta_out[qid] = -__builtin_huge_valf();
        aref[qid] = -__builtin_huge_valf();
        if (smax_out) smax_out[qid] = -__builtin_huge_valf();
      } else {
        flag_query(qid, flags, qsel, qsel_n);
      }
    }
    return;
  }
  uint32_t T = 0;
  // Bound first (TT_SEL_BOUND): the R-th largest of the lanes' top-1 (R <= 64) or top-2
  // (R <= 128) keys is a lower bound L of the R-th largest key (>= R distinct keys reach it).
  // The keys >= L (a few dozen above R) are compacted through LDS into <= 4 registers per lane,
  // and the 32-step search runs there: for cand <= L both sets count >= R, above L they count
  // alike, so T is the same.  (The search over all PER registers -- 32 x ni ballots -- was
  // most of the selection's time: the sample level's ~2k keys per query.)
  __shared__ uint32_t cmp_s[4][256];
  int nc = -1;  // compacted keys (-1: none)
  uint32_t ck[4] = {0u, 0u, 0u, 0u};
  if (TT_SEL_BOUND && R <= 128 && ni > 4) {
    uint32_t m1 = 0u, m2 = 0u;
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (i < ni) {
        m2 = max(m2, min(m1, hv[i]));
        m1 = max(m1, hv[i]);
      }
    uint32_t L = 0u;
    for (int bit = 31; bit >= 0; --bit) {
      const uint32_t cand = L | (1u << bit);
      int cnt = __popcll(__ballot(m1 >= cand));
      if (R > 64) cnt += __popcll(__ballot(m2 >= cand));
      if (cnt >= R) L = cand;
    }
    int c = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (i < ni) c += __popcll(__ballot(hv[i] >= L && hv[i] != 0u));
    if (c <= 256) {
      int base = 0;
#pragma unroll
      for (int i = 0; i < PER; ++i)
        if (i < ni) {
          const bool in = hv[i] >= L && hv[i] != 0u;
          const uint64_t bm = __ballot(in);
          const int pos = base + (int)__builtin_amdgcn_mbcnt_hi(
                                     (uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
          if (in) cmp_s[wv][pos] = hv[i];
          base += __popcll(bm);
        }
      wave_sync();
#pragma unroll
      for (int r = 0; r < 4; ++r) ck[r] = lane + 64 * r < c ? cmp_s[wv][lane + 64 * r] : 0u;
      nc = c;
    }
  }
  if (nc >= 0) {
    const int nr = __builtin_amdgcn_readfirstlane((nc + 63) / 64);
    for (int bit = 31; bit >= 0; --bit) {
      const uint32_t cand = T | (1u << bit);
      int cnt = __popcll(__ballot(ck[0] >= cand));
      if (nr > 1) cnt += __popcll(__ballot(ck[1] >= cand));
      if (nr > 2) cnt += __popcll(__ballot(ck[2] >= cand)) + __popcll(__ballot(ck[3] >= cand));
      if (cnt >= R) T = cand;
    }
  } else
  for (int bit = 31; bit >= 0; --bit) {
    const uint32_t cand = T | (1u << bit);
    // wave count by ballot + scalar popcount (a 6-step shuffle reduction per bit was a
    // ~100-cycle dependent LDS chain: 32 of them dominated a lone query's selection)
    int cnt = 0;
#pragma unroll
    for (int i0 = 0; i0 < PER; i0 += 4)  // one branch per 4 registers (unused ones hold 0)
      if (i0 < ni)
#pragma unroll
        for (int u = 0; u < 4; ++u) cnt += __popcll(__ballot(hv[i0 + u] >= cand));
    if (cnt >= R) T = cand;
  }
  if (TT_EXP_SEL_STOP == 2) {  // timing only: stop after the bitwise search
    if (lane == 0 && T == 0x12345u) theta_out[qid] = 0.f;
    return;
  }
  const float A = key_float(T);

#if TT_EXP_SEL_TIMING
  tstamp[ntst++] = wall_clock64();
#endif
  if (mode == 0) {
    if (smax_out) {  // sharded: the sample's best a (upper end of the probe range)
      uint32_t m = 0;
#pragma unroll
      for (int i = 0; i < PER; ++i)
        if (i < ni) m = max(m, hv[i]);
      for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
      if (lane == 0) smax_out[qid] = key_float(m);
    }
    if (lane == 0) {  // fin: the next level is the full one -> its threshold (full_theta)
      theta_out[qid] = fin ? full_theta(A, eps2[qid]) : A;
      aref[qid] = A;
    }
    return;
  }
  if (!(A >= aref[qid])) {  // the optimistic threshold did not hold
    if (lane == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  const float thr = A - eps2[qid];
  int nb = 0;
  uint64_t* qb = band + (int64_t)qid * BAND_CAP;
  // the band in two parts: first the rows with a >= A_k (the k largest a, plus ties: P1), then
  // the other rows with a >= A_k - 2 eps; k_rerank scores P1 first and keeps from the rest only
  // rows that can still reach the k-th exact score (two-phase re-rank)
#pragma unroll
  for (int part = 0; part < 2; ++part) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      if (i < ni) {
        const bool in = lane + 64 * i < total &&
                        (part == 0 ? hv[i] >= T : hv[i] < T && key_float(hv[i]) >= thr);
        const uint64_t bm = __ballot(in);
        const int pos = nb + (int)__builtin_amdgcn_mbcnt_hi(
                                 (uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
        if (in && pos < BAND_CAP) qb[pos] = ((uint64_t)hv[i] << 32) | lo[i];
        nb += __popcll(bm);
      }
    }
    if (part == 0 && lane == 0) band_p1[qid] = nb;
  }
#if TT_EXP_SEL_TIMING
  tstamp[ntst++] = wall_clock64();
  if (lane == 0 && qid == 0 && n_slabs > 64)
    printf("SELT mode=%d n_slabs=%d total=%d: %d %d %d %d %d %d %d\n", mode, n_slabs, total,
           (int)(tstamp[1] - tstamp[0]), (int)(tstamp[2] - tstamp[1]), (int)(tstamp[3] - tstamp[2]),
           (int)(tstamp[4] - tstamp[3]), (int)(tstamp[5] - tstamp[4]), (int)(tstamp[6] - tstamp[5]),
           ntst > 7 ? (int)(tstamp[7] - tstamp[6]) : -1);
#endif
  if (lane == 0) {
    if (nb > BAND_CAP) flag_query(qid, flags, qsel, qsel_n);
    else band_n[qid] = nb;
  }
}

// --------------------------------------------------------------------------- small batches
// Small query batches (nq <= SM_NQ: the one-buyer /retrieve call, Mode A's 256-buyer
// searches): one 1024-thread block per query instead of one wave.  A lone query's
// k_select_reg (one wave walking up to 2048 keys and 32 dependent ballot steps) and
// k_rerank (6 dependent 256-B chunk rounds per 64 band rows) were latency-bound: 16-25 us
// each.  Here the whole block gathers the candidate keys into LDS, a 4-pass 8-bit radix
// select finds the R-th largest score, and (last level) the band's exact scores come from
// the f32 MFMA in one round: a wave scores 16 band rows with v_mfma_f32_16x16x4_f32, lane
// group g holding dims 16t+4g..+3 -- the canonical fma order (t, i, g), bit-identical to
// the f32 scan and k_rerank -- all of its 16-B row loads in flight at once.
constexpr int SM_THREADS = 1024, SM_WAVES = SM_THREADS / 64;
constexpr int SM_NQ = 256;
constexpr int SM_CAP = SW_CAP;  // candidates per query the small path selects from
constexpr int SM_PER = SM_CAP / SM_THREADS;  // keys per thread in the radix select

template <int CAP>
struct SmallLdsT {
  uint64_t key[CAP];   // the query's candidate keys (orderable score << 32 | ~row)
  int wred[SM_WAVES];
  uint32_t wmax[SM_WAVES];
  // radix select: pass p counts into hist[p % 3] (one barrier per pass); 512 bins for the
  // windowed first pass, 256 for the byte passes
  __attribute__((aligned(16))) int hist[3][512];
};
using SmallLds = SmallLdsT<SM_CAP>;

// Gather the query's per-slab candidate lists into s.key (n_slabs <= SM_THREADS).  Returns
// the candidate count, or -1 when a list overflowed / the total exceeds SM_CAP.
__device__ int small_collect(const uint64_t* __restrict__ lists, const int* __restrict__ counts,
                             int n_slabs, int qid, SmallLds& s) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = tid < n_slabs ? counts[(int64_t)qid * n_slabs + tid] : 0;
  int incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, 64);
    incl += lane >= o ? y : 0;
  }
  if (lane == 63) s.wred[w] = incl;
  const int over = __syncthreads_or(c > FL_CAP);
  int base = 0, total = 0;
#pragma unroll
  for (int i = 0; i < SM_WAVES; ++i) {
    const int v = s.wred[i];
    base += i < w ? v : 0;
    total += v;
  }
  if (over || total > SM_CAP) return -1;
  const uint64_t* l = lists + ((int64_t)qid * n_slabs + tid) * FL_CAP;
  const int e0 = base + incl - c;
#pragma unroll 4
  for (int i = 0; i < c; ++i) s.key[e0 + i] = l[i];
  __syncthreads();
  return total;
}

// One radix pass of a block-wide select over NB bins (256 or 512): key j (act) is counted
// in bin (larger bin = larger key); every wave then scans the histogram itself (no pick
// broadcast): lane l owns the NB/64 bins from NB - 1 - (NB/64) l downwards, so the inclusive
// prefix over lanes (DPP) counts the keys in bins >= the lane's lowest, and F = the first
// lane reaching r.  Returns the bin holding the r-th largest key; r becomes its rank inside
// that bin.  `next` (the following pass's histogram, NB entries) is zeroed before the
// barrier.  The callers' bin maps spread the keys, so no wave aggregation of the atomics.
template <int PER, int NB, class BinF>
__device__ __forceinline__ int radix_pass(int* hist, int* next, BinF binof, int& r) {
  constexpr int BPL = NB / 64;  // bins per lane
  const int tid = threadIdx.x, lane = tid & 63;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    uint32_t bin;
    if (binof(j, bin)) atomicAdd(&hist[bin], 1);
  }
  if (next)
    for (int i = tid; i < NB; i += blockDim.x) next[i] = 0;
  __syncthreads();
  int c[BPL];  // c[i] = bin NB - 1 - BPL lane - i
  const int top = NB - 1 - BPL * lane;
#pragma unroll
  for (int i = 0; i < BPL; ++i) c[i] = hist[top - i];
  int mine = 0;
#pragma unroll
  for (int i = 0; i < BPL; ++i) mine += c[i];
  const int incl = wave_incl_sum(mine);
  const int F = __builtin_ctzll(__ballot(incl >= r));
  int above = __builtin_amdgcn_readlane(incl - mine, F);
  int bin = NB - BPL * (F + 1);  // the lane's lowest bin unless found earlier
#pragma unroll
  for (int i = 0; i < BPL - 1; ++i) {
    const int ci = __builtin_amdgcn_readlane(c[i], F);
    if (above + ci >= r) {
      bin = NB - 1 - BPL * F - i;
      break;
    }
    above += ci;
  }
  r -= above;
  return bin;
}

// R-th largest high word (orderable score) of the keys h (0 = no key), block-wide radix
// select.  Caller guarantees at least R nonzero keys.  ONE barrier per pass; pass p counts
// into hist[p % 3], zeroed during pass p - 1 (after barrier p - 2, which every reader of that
// buffer's previous use, pass p - 3, had passed).
// hmax != 0 (the max nonzero h): a first pass over 16-bit prefixes in a window of 511 below
// hmax's -- the candidates' scores cluster (a fixed top byte puts nearly every key in one or
// two bins, and serialised same-address atomics), while prefix steps (2^-7 relative each, 128
// per octave) spread them; 511 steps cover 4 octaves of score below the maximum (255 did not
// cover the bench's Mode B buyer whose best row scores 0.75 and its 100th 0.19: 256 steps,
// so its select ran the plain 4 passes after the window: 10.2 us; 1023 steps: 4.7 us; 511:
// 3.1 us, iid 2.9 us) -- then the low two bytes: 3 passes.  The r-th key outside the
// window (bin 0) -> the plain 4 passes of 8 bits.  (Four passes with wave-aggregated atomics
// and four barriers each: 5.4 us of the one-buyer final.)
template <int PER, int CAP>
__device__ uint32_t small_radix_select(const uint32_t (&h)[PER], int R, SmallLdsT<CAP>& s,
                                       uint32_t hmax = 0u) {
  const int tid = threadIdx.x;
  for (int i = tid; i < 512; i += blockDim.x) s.hist[0][i] = 0;
  __syncthreads();
  int r = R, pc = 0, shift = 24;
  uint32_t prefix = 0u, pmask = 0u;
  if (hmax != 0u) {
    const uint32_t top = hmax >> 16;
    const int b = radix_pass<PER, 512>(s.hist[0], s.hist[1], [&](int j, uint32_t& bin) {
      const uint32_t d = top - (h[j] >> 16);
      bin = 511u - (d < 511u ? d : 511u);
      return h[j] != 0u;
    }, r);
    pc = 1;
    if (b > 0) {
      prefix = (top - (uint32_t)(511 - b)) << 16;
      pmask = 0xffff0000u;
      shift = 8;
    } else {
      r = R;
    }
  }
#pragma unroll 1
  for (; shift >= 0; shift -= 8, ++pc) {
    const int b = radix_pass<PER, 256>(s.hist[pc % 3], shift > 0 ? s.hist[(pc + 1) % 3] : nullptr,
                                       [&](int j, uint32_t& bin) {
                                         bin = (h[j] >> shift) & 255u;
                                         return h[j] != 0u && (h[j] & pmask) == prefix;
                                       }, r);
    prefix |= (uint32_t)b << shift;
    pmask |= 0xffu << shift;
  }
  return prefix;
}

// Sample level of a small batch (mode 0 of k_select_reg): theta_out = a_J (fin: a_J - eps2).
__global__ __launch_bounds__(SM_THREADS) void k_select_small(
    const uint64_t* __restrict__ lists, const int* __restrict__ counts, int n_slabs, int J,
    const float* __restrict__ eps2, float* __restrict__ theta_out, float* __restrict__ aref,
    int* __restrict__ flags, int* qsel, int* qsel_n, int fin) {
  __shared__ SmallLds s;
  const int qid = blockIdx.x, tid = threadIdx.x;
  if (flags[qid]) {
    if (tid == 0) theta_out[qid] = __builtin_huge_valf();
    return;
  }
  const int total = small_collect(lists, counts, n_slabs, qid, s);
  if (total < 0) {
    if (tid == 0) {
      flag_query(qid, flags, qsel, qsel_n);
      theta_out[qid] = __builtin_huge_valf();
    }
    return;
  }
  if (total < J) {  // fewer than J candidates: a_J = -inf
    if (tid == 0) theta_out[qid] = aref[qid] = -__builtin_huge_valf();
    return;
  }
  uint32_t h[SM_PER];
#pragma unroll
  for (int j = 0; j < SM_PER; ++j) {
    const int e = tid + j * SM_THREADS;
    h[j] = e < total ? (uint32_t)(s.key[e] >> 32) : 0u;
  }
  const float A = key_float(small_radix_select(h, J, s));
  if (tid == 0) {
    theta_out[qid] = fin ? A - eps2[qid] : A;
    aref[qid] = A;
  }
}

// LDS of the band re-rank (exact scores of the band rows + output ranks), one query per block
template <int EP>
struct BandLds {
  uint32_t brow[BAND_CAP];
  uint64_t sbuf[BAND_CAP];
  __attribute__((aligned(16))) float qs[EP];
  int wcnt[SM_WAVES];
};

// Exact canonical f32 scores of 16 rows: lane (r, g) = (lane & 15, lane >> 4) names row `row`
// (one per r), loads its dims 16t + 4g .. +3 for every t (all loads in flight), and the chain
// runs on v_mfma_f32_16x16x4_f32 with the query (LDS, f32) in every column: the canonical order
// (t, i, g), bit-identical to the f32 scan.  D[row 4g + j][col 0] comes back in lane 16 g,
// element j.  (Per-row VALU fma chains after an LDS transpose: 0.182 vs 0.177 ms per one-buyer
// search, 0.292 vs 0.276 ms at 256 queries.)
template <int EP>
__device__ __forceinline__ f32x4 exact16(const float* __restrict__ db, int64_t ld, uint32_t row,
                                         const float* qs, int lane) {
  const int g = lane >> 4;
  constexpr int NT = EP / 16, TCH = NT <= 24 ? NT : 16;  // t-steps per load batch
  static_assert(NT % TCH == 0, "load batches must tile the row");
  const float* xr = db + (int64_t)row * ld + 4 * g;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int t0 = 0; t0 < NT; t0 += TCH) {
    f32x4 a[TCH];
#pragma unroll
    for (int t = 0; t < TCH; ++t) a[t] = *(const f32x4*)(xr + 16 * (t0 + t));
    // every load of the batch issued before the chain: left to itself the scheduler kept two
    // in flight (1024-thread blocks: a 128-register budget), i.e. ~TCH dependent round trips
    // per 16 rows -- most of k_final_small's time (tools/blktime_small.py)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < TCH; ++t) {
      const f32x4 b = *(const f32x4*)(qs + 16 * (t0 + t) + 4 * g);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][0], b[0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][1], b[1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][2], b[2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][3], b[3], acc, 0, 0, 0);
    }
  }
  return acc;
}

// Band positions: keys (h[j] = high word of key slot tid + j * SM_THREADS, 0 = none) with
// a >= thr get consecutive positions in a deterministic order (block-wide prefix count).
// Returns the band size nb; *pos0 = this thread's first position.
template <int EP, int PER>
__device__ int band_positions(const uint32_t (&h)[PER], float thr, BandLds<EP>& bl, int* pos0) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int mine = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) mine += (h[j] != 0u && key_float(h[j]) >= thr) ? 1 : 0;
  const int incl = wave_incl_sum(mine);
  if (lane == 63) bl.wcnt[w] = incl;
  __syncthreads();
  int base = 0, nb = 0;
#pragma unroll
  for (int i = 0; i < SM_WAVES; ++i) {
    base += i < w ? bl.wcnt[i] : 0;
    nb += bl.wcnt[i];
  }
  *pos0 = base + incl - mine;
  return nb;
}

// Output of a band whose exact keys bl.sbuf[0, nb) are known: slot = rank (score desc, row
// asc): rank(e) = #keys ahead of key e (keys of distinct rows are distinct; equal keys -- only
// NaN scores, key 0 -- are ordered by position), so every band entry knows its output slot
// without a sort: ~nb compares per entry, over 4 threads per entry when nb <= 256 (the bitonic
// sorts this replaces spent 36 dependent stages: 4.6 us in one wave, 7.5 us block-wide).
template <int EP>
__device__ void band_rank_out(BandLds<EP>& bl, int nb, int qid, int k, int64_t row_base,
                              float* __restrict__ out_s, int64_t* __restrict__ out_i) {
  const int tid = threadIdx.x;
  const int per = nb <= 256 ? 4 : 1;
  const int e = tid / per, part = tid % per;
  int rank = 0;
  uint64_t me = 0ull;
  if (e < nb) {
    me = bl.sbuf[e];
#pragma unroll 8
    for (int j = part; j < nb; j += per) {
      const uint64_t o = bl.sbuf[j];
      rank += (o > me || (o == me && j < e)) ? 1 : 0;
    }
  }
  if (per == 4) rank = quad_sum(rank);  // the 4 partial counts sit in one lane quad
  if (e < nb && part == 0 && rank < k) {
    float sc = -__builtin_huge_valf();
    int64_t ix = -1;
    if (me != 0ull) {  // NaN score: key 0 ranks last, reported as (-inf, -1)
      sc = key_score(me);
      ix = row_base + (int64_t)key_row(me);
    }
    out_s[(int64_t)qid * k + rank] = sc;
    out_i[(int64_t)qid * k + rank] = ix;
  }
}

// Band = keys with a >= thr (band_positions); exact canonical f32 scores of the band rows
// (exact16, 16 rows per wave pass); output by rank (band_rank_out).  A band past BAND_CAP, or
// a decoded row >= n_rows (a corrupted key: never read), flags the query for the exact
// fallback instead.  Every slot < k is written when the band holds >= k rows (callers
// guarantee it).
template <int EP, int PER, int CAP>
__device__ void band_rerank(const uint32_t (&h)[PER], SmallLdsT<CAP>& s, BandLds<EP>& bl,
                            float thr, int qid, int k, int* flags, int* qsel, int* qsel_n,
                            const float* __restrict__ db, int64_t ld, int64_t n_rows,
                            const float* __restrict__ q, int64_t ldq, int64_t row_base,
                            float* __restrict__ out_s, int64_t* __restrict__ out_i) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < EP; i += SM_THREADS) bl.qs[i] = q[(int64_t)qid * ldq + i];
  int pos;
  const int nb = band_positions<EP>(h, thr, bl, &pos);
  if (nb > BAND_CAP) {
    if (tid == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  bool bad_row = false;  // a decoded row >= n_rows is never read: exact fallback instead
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int e = tid + j * SM_THREADS;
    if (h[j] != 0u && key_float(h[j]) >= thr) {
      const uint32_t r = key_row(s.key[e]);
      bad_row |= (int64_t)r >= n_rows;
      bl.brow[pos++] = (int64_t)r < n_rows ? r : 0u;
    }
  }
  if (__syncthreads_or(bad_row)) {
    if (tid == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  // exact scores: wave w takes band rows [16 gr, 16 gr + 16), gr = w, w + SM_WAVES, ...
  {
    const int r16 = lane & 15, g = lane >> 4;
    for (int gr = w; 16 * gr < nb; gr += SM_WAVES) {
      const int e = 16 * gr + r16;
      const f32x4 acc = exact16<EP>(db, ld, bl.brow[e < nb ? e : nb - 1], bl.qs, lane);
      if (r16 == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ej = 16 * gr + 4 * g + j;
          if (ej < nb) bl.sbuf[ej] = acc[j] != acc[j] ? 0ull : make_key(acc[j], bl.brow[ej]);
        }
      }
    }
  }
  __syncthreads();
  band_rank_out<EP>(bl, nb, qid, k, row_base, out_s, out_i);
}

// Full level of a small batch: selection (mode 1 of k_select_reg) + exact re-rank (k_rerank)
// in one launch.  A_k = k-th best a; A_k < aref -> the optimistic threshold failed (flag);
// band = candidates with a >= A_k - eps2 (<= BAND_CAP, else flag); exact canonical f32
// scores of the band rows by f32 MFMA; sort (score desc, row asc); top-k out.
// The band's row gathers (~180 random 1.5 KB rows per query) are memory-latency bound on one
// CU: 9-14 us of the one-buyer search.  Measured and not adopted: splitting a query over 8
// blocks that meet through a global counter (25-30 us: the agent-scope release/acquire that
// makes one block's scores visible to another XCD writes back / invalidates L2), and the full
// level touching its candidates' f32 rows as it flushes them (no change).
template <int EP>
__global__ __launch_bounds__(SM_THREADS) void k_final_small(
    const uint64_t* __restrict__ lists, const int* __restrict__ counts, int n_slabs, int k,
    const float* __restrict__ eps2, const float* __restrict__ aref, int* __restrict__ flags,
    int* qsel, int* qsel_n, const float* __restrict__ db, int64_t ld, int64_t n_rows,
    const float* __restrict__ q, int64_t ldq, int64_t row_base, float* __restrict__ out_s,
    int64_t* __restrict__ out_i) {
  __shared__ SmallLds s;
  __shared__ BandLds<EP> bl;
  const int qid = blockIdx.x;
  const int tid = threadIdx.x;
#if TT_EXP_BLKTIME
  struct BlkTimeEnd {  // TT_EXP_BLKTIME_LVL 9: this kernel's blocks instead of a ring level's
    unsigned long long t0;
    unsigned long long ph[2];
    __device__ ~BlkTimeEnd() {
      if (TT_EXP_BLKTIME_LVL != 9 || blockIdx.x >= BLKTIME_MAX) return;
      __syncthreads();
      if (threadIdx.x == 0) {
        g_blkph[2 * blockIdx.x] = ph[0];
        g_blkph[2 * blockIdx.x + 1] = ph[1];
        unsigned long long* o = g_blktime + 4 * blockIdx.x;
        o[0] = t0;
        o[1] = wall_clock64();
        o[2] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);
        o[3] = ((unsigned long long)blockIdx.x << 32) |
               (unsigned)__builtin_amdgcn_s_getreg((3 << 11) | 20);
      }
    }
  } blk_end{(unsigned long long)wall_clock64(), {0ull, 0ull}};
#endif
  if (flags[qid]) return;  // served by the exact fallback
  const int total = small_collect(lists, counts, n_slabs, qid, s);
#if TT_EXP_BLKTIME
  blk_end.ph[0] = wall_clock64();
#endif
  if (total < k) {  // overflow (-1) or too few candidates to certify: exact fallback
    if (tid == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  uint32_t h[SM_PER];
#pragma unroll
  for (int j = 0; j < SM_PER; ++j) {
    const int e = tid + j * SM_THREADS;
    h[j] = e < total ? (uint32_t)(s.key[e] >> 32) : 0u;
  }
  const float A = key_float(small_radix_select(h, k, s));
#if TT_EXP_BLKTIME
  blk_end.ph[1] = wall_clock64();
#endif
  if (!(A >= aref[qid])) {
    if (tid == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  band_rerank<EP>(h, s, bl, A - eps2[qid], qid, k, flags, qsel, qsel_n, db, ld, n_rows, q, ldq,
                  row_base, out_s, out_i);
}

// ------------------------------------------------------------ single-pass small batches
// nq <= TM_NQ (the one-buyer /retrieve call, server.py:241-244 -> vector_db.py:160): ONE
// streaming pass instead of sample level -> selection -> full level.  One block per CU
// (G = #CUs, one round, no tail), each owning a contiguous slab; the bf16 image streams
// HBM -> LDS through the ring of k_filter_ring (buffer_load ... lds, non-temporal, 3 tiles in
// flight, one s_barrier per tile) and one wave per 16-row block of a tile scores it on bf16
// MFMA (a 16-query block).  Each such wave keeps, per query, the running top-TM_M of its rows'
// a in an LDS buffer (append a >= tau, its running TM_M-th best; compact by a wave bitonic sort
// when the buffer nears full: a streaming top-m, ~TM_M ln(rows / TM_M) appends per query); at
// the end the waves' lists merge into the slab's sorted top-TM_M, and the block computes the
// exact keys of those rows (exact16).
// k_final_topm then takes, per query, the union U of the G lists: A = k-th best a of U; a slab
// dropped only rows with a <= tau_b (its TM_M-th best), so if every full list has
// tau_b < A - 2 eps, U holds every row with a >= A - 2 eps (and A is the catalog's A_k):
// the band, re-ranked exactly as in k_final_small.  Otherwise the query is flagged for the
// exact fallback.  Bytes: the bf16 image once; no sample level, no per-level selections.
constexpr int TM_NQ = 16;     // queries per MFMA query block (the buffers' query capacity)
// queries per search that take this path: per-tile appends, tile-max bounds and compactions
// grow with the query count, and from 8 queries on the multi-level path is as fast (one-buyer
// latency, topm vs multi-level, ms: nq 1 0.139 / 0.181, 2 0.145 / 0.195, 4 0.158 / 0.184,
// 8 0.188 / 0.186, 16 0.225 / 0.189)
#ifndef TT_EXP_TM_NQ_RUN
#define TT_EXP_TM_NQ_RUN 4  // timing builds: the single passes for larger batches
#endif
TT_CHECK_EXP(TT_EXP_TM_NQ_RUN != 4, "TT_EXP_TM_NQ_RUN");
constexpr int TM_NQ_RUN = TT_EXP_TM_NQ_RUN;
// the int8 single pass (k_filter_topm_i8) runs up to 8 queries: its candidate buffers are laid
// out for 4 (nq <= 4) or 8 queries (the kernel's QB), and 5-8 queries still beat the multi-level bf16
// path (1M x 384, nq = 8: 0.128 vs 0.185 ms; 16: 0.249 vs 0.183, so 16 stays multi-level)
constexpr int TM_NQ_I8 = TM_NQ_RUN > 8 ? TM_NQ_RUN : 8;
constexpr int TM_M = 16;      // rows kept per (query, slab)
constexpr int TM_BUF = 256;   // candidate buffer per query, split over the compute waves
constexpr int TM_SLOTS = TT_EXP_TM_SLOTS, TM_PD = TM_SLOTS - 1;  // ring slots, tiles in flight
constexpr int TM_WAVES = 8;
#ifndef TT_TM_ANYB
#define TT_TM_ANYB 1  // 1: one ballot per tile skips a wave's appends when no row passes tau
#endif
TT_CHECK_EXP(TT_TM_ANYB != 1, "TT_TM_ANYB");
#ifndef TT_TM_BIGBUF16
#define TT_TM_BIGBUF16 0  // 1: k_filter_topm's buffers hold TM_NQ_RUN queries, as the int8 pass's
#endif
TT_CHECK_EXP(TT_TM_BIGBUF16 != 0, "TT_TM_BIGBUF16");
// queries the single passes' candidate buffers hold.  They run for nq <= TM_NQ_RUN only, so the
// TM_NQ x TM_BUF keys of LDS can give each of those queries 4x the buffer: the int8 pass (4
// compute waves, 64 keys each per query otherwise) then compacts ~0 instead of 2.5 (nq = 1) /
// 9.7 (nq = 4) times per wave and slab -- nq 1 / 2 / 4: 0.094 / 0.104 / 0.129 -> 0.092 / 0.093 /
// 0.094 ms per search; the bf16 pass (2 compute waves, 128 keys each) gains at nq = 4 (0.156 ->
// 0.150) but loses at nq = 1 (0.141 -> 0.145), so it keeps the 16-query layout
constexpr int tm_qb16() { return TT_TM_BIGBUF16 ? TM_NQ_RUN : TM_NQ; }
#ifndef TT_TM_PREFIX
#define TT_TM_PREFIX 1  // 1: appends place a lane's 4 rows by one column prefix (0: per-row ballots)
#endif
TT_CHECK_EXP(TT_TM_PREFIX != 1, "TT_TM_PREFIX");
#ifndef TT_TM_SHTAU
#define TT_TM_SHTAU 1  // 1: the compute waves of a block share their tau bounds (max)
#endif
TT_CHECK_EXP(TT_TM_SHTAU != 1, "TT_TM_SHTAU");
constexpr int TM_CAP = 4096;  // final: keys per query (G x TM_M, G <= 256)

template <int EP>
constexpr int topm_smem() {
  return TM_SLOTS * RingCfg<EP>::TR * EP * 2 + TM_NQ * TM_BUF * 8;
}

template <int EP>
__global__ __launch_bounds__(64 * TM_WAVES, 1) void k_filter_topm(
    const uint16_t* __restrict__ xb, int64_t ld, int64_t n, const float* __restrict__ q, int nq,
    int64_t ldq, int rows_per_blk, const float* __restrict__ db, float X, float R,
    float* __restrict__ eps2, uint64_t* __restrict__ lists, uint64_t* __restrict__ xkeys,
    int* __restrict__ counts, int* __restrict__ flags, int* __restrict__ qsel_n) {
  constexpr int TR = RingCfg<EP>::TR, KS = EP / 32, CPR = EP / 8, RB = TR / 16;
  constexpr int TILE_B = TR * EP * 2, PIECES = TILE_B / 1024, PPW = PIECES / TM_WAVES;
  constexpr int FM = (CPR >= 16 ? 16 : CPR) - 1;
  static_assert(PIECES % TM_WAVES == 0, "tile must split into whole 1-KiB pieces per wave");
  __shared__ __attribute__((aligned(16))) char smem[topm_smem<EP>()];
  __shared__ int ncs[TM_NQ];
  char* ring = smem;
  uint64_t* tbuf = (uint64_t*)(smem + TM_SLOTS * TILE_B);  // [TM_NQ][TM_BUF]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int G = gridDim.x, blk = blockIdx.x;
  if (blk == 0 && tid < nq) {  // per-query fallback state (FilterWs: flags, qsel, qsel_n, done)
    flags[tid] = 0;
    qsel_n[1 + tid] = 0;
    if (tid == 0) *qsel_n = 0;
  }
  const int64_t j0 = (int64_t)blk * rows_per_blk;
  const int64_t j1 = (j0 + rows_per_blk < n) ? j0 + rows_per_blk : n;
  const int n_tiles = j0 < j1 ? (int)((j1 - j0 + TR - 1) / TR) : 0;

  // compute waves w < CW (one per 16-row block of a tile: the scoring of a tile is split so
  // that no single wave's per-tile work -- fragment reads, MFMAs, appends -- paces the ring;
  // one wave scoring the whole tile: 131 vs 122 us for the same stream without that work).
  // Each holds the query fragments (bf16 B operands, 16 queries) and its own per-query top-m
  // buffers tbuf[w][c][TMB].
  constexpr int TM_QB = tm_qb16(), CW = RB, TMB = TM_NQ * TM_BUF / TM_QB / CW;
  constexpr int CPER = TMB / 64;
  static_assert(TMB % 64 == 0 && TMB >= 2 * TM_M && CW <= TM_WAVES, "top-m buffer shape");
  const bool cw = w < CW;
  uint64_t* wbuf = tbuf + (cw ? w : 0) * TM_QB * TMB;  // [TM_QB][TMB] per compute wave
  bf16x8 qf[KS];
  const bool qv = col < nq;
  // tau bounds shared by the block's compute waves: a row below ANY wave's tau (each a lower
  // bound of the 16th best of distinct rows of this slab) is below the slab's 16th best, so
  // every wave may drop it -- each wave's appends follow the block's max
  __shared__ __attribute__((aligned(16))) float tau_sh[TM_NQ_RUN][4];
  if (TT_TM_SHTAU && w < 4 && lane < TM_NQ_RUN) tau_sh[lane][w] = -__builtin_huge_valf();
  float tau = qv ? -__builtin_huge_valf() : __builtin_huge_valf();
  int cnt = 0;  // appended keys of query `col` (same in the 4 lanes of a column)
  // tile-max bound of tau (appends): the 16 largest of the set, ascending (tm[0] = the 16th)
  float tm[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) tm[i] = -__builtin_huge_valf();
  // insert m: clamp(m, tm[i], tm[i + 1]) per entry = the sorted 16 largest of the set plus m
  // (one v_med3 each, branch-free; a no-op when m <= tm[0]); NaN enters as -inf
  auto tm_insert = [&](float m) __attribute__((always_inline)) {
    m = m == m ? m : -__builtin_huge_valf();
#pragma unroll
    for (int i = 0; i < 15; ++i) tm[i] = __builtin_amdgcn_fmed3f(tm[i], m, tm[i + 1]);
    tm[15] = fmaxf(tm[15], m);
  };
  // the block's shared tau for this lane's query (issued before the tile's fragment reads:
  // LDS reads complete in order)
  auto read_shtau = [&]() __attribute__((always_inline)) {
    if (!TT_TM_SHTAU) return -__builtin_huge_valf();
    const f32x4 v = *(const f32x4*)&tau_sh[col < TM_NQ_RUN ? col : 0][0];
    return fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
  };
  int st_compact = 0;
  uint64_t st_t0 = TT_EXP_TM_STATS ? wall_clock64() : 0, st_t1 = 0, st_t2 = 0;
  if (cw) {
    const float* qp = q + (int64_t)(qv ? col : 0) * ldq + 8 * g;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const f32x4 v0 = *(const f32x4*)(qp + 32 * s);
      const f32x4 v1 = *(const f32x4*)(qp + 32 * s + 4);
      u32x4 u = {pack_bf16x2(v0[0], v0[1]), pack_bf16x2(v0[2], v0[3]), pack_bf16x2(v1[0], v1[1]),
                 pack_bf16x2(v1[2], v1[3])};
      qf[s] = __builtin_bit_cast(bf16x8, u);
    }
  }
  wait_vm<0>();  // the query loads / init stores retire before the ring's counted waits

  const int64_t tile_bytes = (int64_t)ld * 2 * TR;
  const char* slab_base = (const char*)xb + j0 * ld * 2;
  uint32_t voff[PPW];
#pragma unroll
  for (int pp = 0; pp < PPW; ++pp) {
    const int P = (w + TM_WAVES * pp) * 64 + lane;
    const int r = P / CPR;
    voff[pp] = (uint32_t)(r * ld * 2) + 16u * (uint32_t)((P % CPR) ^ (r & FM));
  }
  auto issue = [&](int t) __attribute__((always_inline)) {
    char* slot = ring + (t % TM_SLOTS) * TILE_B;
    const int64_t jt = j0 + (int64_t)t * TR;
    const bool clamp = jt + TR > j1;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(slab_base + (int64_t)t * tile_bytes), 0, (int)tile_bytes, 0x00020000);
#pragma unroll
    for (int pp = 0; pp < PPW; ++pp) {
      uint32_t off = voff[pp];
      if (clamp) {  // rows past the slab end read a copy of its last row (masked below)
        const int P = (w + TM_WAVES * pp) * 64 + lane;
        const int r = P / CPR;
        int64_t j = jt + r;
        j = j < j1 ? j : j1 - 1;
        off = (uint32_t)((j - jt) * ld * 2) + 16u * (uint32_t)((P % CPR) ^ (r & FM));
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(slot + (w + TM_WAVES * pp) * 1024), 16,
          off, 0, 0, 2);
    }
  };
  auto wait_tiles = [&](int younger) __attribute__((always_inline)) {
    static_assert(TM_PD <= 4, "wait_tiles covers up to 3 younger tiles");
    if (younger >= 3) wait_vm<3 * PPW>();
    else if (younger == 2) wait_vm<2 * PPW>();
    else if (younger == 1) wait_vm<PPW>();
    else wait_vm<0>();
  };
  // fragment read offsets of the wave's row block (rows 16 w + col of a tile)
  uint32_t lrd[4];
  {
    const int r = 16 * (cw ? w : 0) + col, f = r & FM, h = f >> 2;
#pragma unroll
    for (int v = 0; v < 4; ++v)
      lrd[v] = lds_addr(ring) + 16 * (r * CPR + (g ^ (f & 3))) + 64 * (v ^ h);
  }
  // compaction of query c's buffer to its sorted top TM_M (wave_top16: a bitwise select, not a
  // sort of the buffer); tau = the TM_M-th key's score
  static_assert(TM_M == 16, "wave_top16 keeps 16");
  auto compact = [&](int c) __attribute__((always_inline)) {
    uint64_t* b = wbuf + c * TMB;
    const int cc = __shfl(cnt, c, 64);
    uint64_t key[CPER];
#pragma unroll
    for (int r = 0; r < CPER; ++r) {
      const int e = lane * CPER + r;
      key[r] = e < cc ? b[e] : 0ull;
    }
    int nc;
    const uint64_t k = wave_top16<CPER>(key, lane, b, &nc);
    if (lane < nc) b[lane] = k;
    const uint32_t hk = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(k >> 32), TM_M - 1);
    if (col == c) {
      cnt = nc;
      if (nc == TM_M) tau = fmaxf(tau, key_float(hk));
    }
    wave_sync();
  };

  // appends of tile t's scores (lane: rows jt + 16 w + 4 g + jj of query col): a >= tau
  // (NaN never passes); positions within a column by ballot (no atomics): the 4 lanes of a
  // column hold cnt.  Then the compactions the buffers need.
  auto appends = [&](f32x4 acc, int t, float shtau) __attribute__((always_inline)) {
    const int64_t jt = j0 + (int64_t)t * TR + 16 * w;
    if (TT_TM_SHTAU && qv) tau = fmaxf(tau, shtau);
    const uint64_t colmask = 0x0001000100010001ull << col;
    const uint64_t below = (1ull << lane) - 1ull;
    if (jt + 16 > j1) {  // (wave-uniform) the slab's last tile: rows past its end score -inf
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        if (jt + 4 * g + jj >= j1) acc[jj] = -__builtin_huge_valf();
    }
    // late in the slab tau has risen past nearly every row: one ballot skips the four
    const bool any = fmaxf(fmaxf(acc[0], acc[1]), fmaxf(acc[2], acc[3])) >= tau;
    if (!TT_TM_ANYB || __ballot(any) != 0ull) {
      const int lr0 = t * TR + 16 * w + 4 * g, nloc = (int)(j1 - j0);  // slab-local rows
      if (TT_TM_PREFIX) {
        // one pass for the lane's 4 rows: its pass count, the exclusive prefix over the
        // column's 4 lanes (lane ^ 16, lane ^ 32 partners) and the column's total
        bool pass[4];
        int np = 0;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          pass[jj] = lr0 + jj < nloc && acc[jj] >= tau;
          np += pass[jj] ? 1 : 0;
        }
        const auto x16 = __builtin_amdgcn_permlane16_swap((uint32_t)np, (uint32_t)np, false,
                                                          false);
        const int b = (int)((g & 1) ? x16[0] : x16[1]);  // lane ^ 16
        const int s2 = np + b;
        const auto x32 = __builtin_amdgcn_permlane32_swap((uint32_t)s2, (uint32_t)s2, false,
                                                          false);
        const int s2x = (int)(lane < 32 ? x32[1] : x32[0]);  // lane ^ 32
        int pos = cnt + ((g & 1) ? b : 0) + ((g & 2) ? s2x : 0);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          if (pass[jj]) {
            lds_write64(lds_addr(wbuf + col * TMB + pos),
                        make_key(acc[jj], (uint32_t)(j0 + lr0 + jj)));
            ++pos;
          }
        cnt += s2 + s2x;
      } else {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float v = acc[jj];
          const bool pass = lr0 + jj < nloc && v >= tau;
          const uint64_t bm = __ballot(pass);
          if (bm != 0ull) {
            const uint64_t mc = bm & colmask;
            if (pass) {
              const int pos = cnt + __popcll(mc & below);
              lds_write64(lds_addr(wbuf + col * TMB + pos),
                          make_key(v, (uint32_t)(j0 + lr0 + jj)));
            }
            cnt += __popcll(mc);
          }
        }
      }
    }
    // tau between compactions: the TM_M-th largest of a set of scores of DISTINCT rows (tm[],
    // the same multiset in the 4 lanes of a column) is a lower bound of the running TM_M-th
    // best.  The set: the first tile's 16 rows, then each later tile's max (a row of that
    // tile: distinct); rows past the slab end and NaNs enter as -inf.  Without it an empty
    // buffer took ~TMB rows before its first compaction, and tau then lagged: 3-4 compactions
    // per query and wave, all queries in the same tiles (nq = 16: 206 us for the 124 us
    // stream).
    if (t == 0) {  // the first tile's 16 rows (every lane of the column gathers all 16)
      float v16[16];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        v16[jj] = acc[jj];
        const auto x16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[jj]),
                                                          __float_as_uint(acc[jj]), false, false);
        v16[4 + jj] = __uint_as_float((g & 1) ? x16[0] : x16[1]);  // lane ^ 16
      }
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const auto x32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v16[jj]),
                                                          __float_as_uint(v16[jj]), false, false);
        v16[8 + jj] = __uint_as_float(lane < 32 ? x32[1] : x32[0]);  // lane ^ 32
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) tm_insert(v16[i]);
    } else {
      float m = fmaxf(fmaxf(acc[0], acc[1]), fmaxf(acc[2], acc[3]));
      const auto x16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m),
                                                        false, false);
      m = fmaxf(__uint_as_float(x16[0]), __uint_as_float(x16[1]));
      const auto x32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m),
                                                        false, false);
      tm_insert(fmaxf(__uint_as_float(x32[0]), __uint_as_float(x32[1])));  // the tile max
    }
    tau = fmaxf(tau, qv ? tm[0] : tau);
    const uint64_t need = __ballot(lane < 16 && cnt > TMB - 16);
    if (need != 0ull) {
      lds_wait<0>();
      uint64_t nd = need;
      while (nd) {
        const int c = __builtin_ctzll(nd);
        nd &= nd - 1;
        compact(c);
        if (TT_EXP_TM_STATS) ++st_compact;
      }
    }
    if (TT_TM_SHTAU && qv && g == 0) tau_sh[col][w] = tau;  // published for the other waves
  };

  // compute wave, per tile t: issue all of its row block's fragment reads (KS x 16 B per
  // lane), run tile t-1's appends while they are in flight, one wait, then tile t's MFMA chain
  // (its scores are appended in the next iteration: the LDS latency hides behind the appends)
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t < TM_PD && t < n_tiles; ++t) issue(t);
  if (w == TM_WAVES - 1 && blk < nq) {  // 2 eps of query blk for the final (not a compute wave)
    const float e = query_eps2_wave<EP>(q + (int64_t)blk * ldq, X, R, lane);
    if (lane == 0) eps2[blk] = e;
  }
  for (int t = 0; t < n_tiles; ++t) {
    wait_tiles(n_tiles - 1 - t < TM_PD - 1 ? n_tiles - 1 - t : TM_PD - 1);
    lds_barrier();  // tile t landed (every wave's pieces); every wave is done with tile t-1
    if (t + TM_PD < n_tiles) issue(t + TM_PD);  // into the slot of tile t-1
    if (cw) {
      const float shtau = read_shtau();
      const uint32_t so = (uint32_t)((t % TM_SLOTS) * TILE_B);
      u32x4 fr[KS];
      static_for<KS>([&](auto s_) __attribute__((always_inline)) {
        constexpr int S = decltype(s_)::value;
        fr[S] = lds_read128<256 * (S / 4)>(lrd[S % 4] + so);
      });
      if (t > 0) appends(acc, t - 1, shtau);
      lds_wait<0>();
      acc = f32x4{0.f, 0.f, 0.f, 0.f};
      static_for<KS>([&](auto s_) __attribute__((always_inline)) {
        constexpr int S = decltype(s_)::value;
        reg_tie(fr[S]);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fr[S]), qf[S],
                                                      acc, 0, 0, 0);
      });
    }
  }
  if (cw && n_tiles > 0) appends(acc, n_tiles - 1, read_shtau());
  wait_vm<0>();
  if (TT_EXP_TM_STATS) st_t1 = wall_clock64();
  // end of the slab, per query (queries spread over the waves): the top TM_M of the CW
  // buffers' keys together (wave_top16) -> tbuf[0][c], the slab's sorted list
  __shared__ int ncw[CW][TM_NQ];
  if (cw && lane < nq && g == 0) ncw[w][lane] = cnt;  // lanes 0..15: col = lane
  lds_wait<0>();  // the appends' hand-issued LDS writes retire before the barrier
  __syncthreads();
  for (int c = w; c < nq; c += TM_WAVES) {
    uint64_t key[CW * CPER];
#pragma unroll
    for (int wb = 0; wb < CW; ++wb) {
      const int cc = ncw[wb][c];
#pragma unroll
      for (int r = 0; r < CPER; ++r) {
        const int e = lane * CPER + r;
        key[wb * CPER + r] = e < cc ? tbuf[(wb * TM_QB + c) * TMB + e] : 0ull;
      }
    }
    int nc;
    const uint64_t k = wave_top16<CW * CPER>(key, lane, tbuf + c * TMB, &nc);
    if (lane < nc) {
      tbuf[c * TMB + lane] = k;
      lists[((int64_t)c * G + blk) * TM_M + lane] = k;
    }
    if (lane == 0) {
      counts[(int64_t)c * G + blk] = nc;
      ncs[c] = nc;
    }
  }
  // exact keys of the kept rows (every block in parallel, one 16-row exact16 pass per query
  // over the 8 waves, the f32 query read from L2 alongside the rows): the final then ranks its
  // band without gathering f32 rows on one CU
  __syncthreads();  // the sorted lists (tbuf) and ncs visible to every wave
  for (int c = w; c < nq; c += TM_WAVES) {
    const int nc = ncs[c], r16 = lane & 15, g4 = 4 * (lane >> 4);
    if (nc == 0) continue;
    const uint64_t* tb = tbuf + c * TMB;
    const f32x4 acc =
        exact16<EP>(db, ld, key_row(tb[r16 < nc ? r16 : 0]), q + (int64_t)c * ldq, lane);
    if (r16 == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (g4 + j < nc)
          xkeys[((int64_t)c * G + blk) * TM_M + g4 + j] =
              acc[j] != acc[j] ? 0ull : make_key(acc[j], key_row(tb[g4 + j]));
    }
  }
  if (TT_EXP_TM_STATS) {
    __syncthreads();
    st_t2 = wall_clock64();
    if ((blk == 0 || blk == 100) && cw && lane == 0)
      printf("topm blk %d wave %d: compactions %d, stream %d ticks, tail %d ticks, cnt0 %d\n",
             blk, w, st_compact, (int)(st_t1 - st_t0), (int)(st_t2 - st_t1), ncw[w][0]);
  }
}

// Final of the single-pass path, one block per query: union U of the G slab lists, A = k-th
// best a of U; every full list's TM_M-th a (tau_b) must be < A - 2 eps (else the query takes
// the exact fallback: a slab may have dropped a band row); band = U's keys with a >= A - 2 eps,
// output in the order of their exact keys, which the streaming blocks computed for every kept
// row (no f32 row gathers here).  2 eps comes from the streaming kernel (query_eps2_wave).
// One block, latency-bound: ~15 us with shuffle (ds_bpermute) scans and four barriers per
// radix pass, DPP scans and one barrier per pass now.
template <int EP>
__global__ __launch_bounds__(SM_THREADS) void k_final_topm(
    const uint64_t* __restrict__ lists, const uint64_t* __restrict__ xkeys,
    const int* __restrict__ counts, int G, int k, const float* __restrict__ eps2,
    int* __restrict__ flags, int* qsel, int* qsel_n, int64_t n_rows, int64_t row_base,
    float* __restrict__ out_s, int64_t* __restrict__ out_i) {
  constexpr int PER = TM_CAP / SM_THREADS;
  __shared__ SmallLdsT<1> s;
  __shared__ BandLds<EP> bl;
  __shared__ float eps_s;
  const int qid = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#if TT_EXP_FINAL_TIMING
  uint64_t ts[8];
  int nts = 0;
#define TT_FTS() (ts[nts++] = wall_clock64())
#else
#define TT_FTS() ((void)0)
#endif
  TT_FTS();
  // collect: slot e = slab e / TM_M, entry e % TM_M (0 = no key: the radix select and the band
  // skip it); the count, approximate key and exact key of every slot loaded together, before
  // the query's eps loads (one round trip; a per-slab copy loop had serialised ~16 dependent
  // L2 round trips); slots past a list's count hold stale keys and are masked
  uint32_t h[PER];
  uint64_t xk[PER];
  {
    int cj[PER];
    uint64_t kk[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int e = tid + j * SM_THREADS, b = e / TM_M;
      const int64_t o = ((int64_t)qid * G + (b < G ? b : 0)) * TM_M + e % TM_M;
      cj[j] = b < G ? counts[(int64_t)qid * G + b] : 0;
      kk[j] = lists[o];
      xk[j] = xkeys[o];
    }
    int mine = 0;
    uint32_t tmax = 0u;  // max over full lists of their TM_M-th key (tau_b)
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = (tid + j * SM_THREADS) % TM_M;
      const bool ok = i < cj[j];
      h[j] = ok ? (uint32_t)(kk[j] >> 32) : 0u;
      if (!ok) xk[j] = 0ull;
      if (ok && i == TM_M - 1) tmax = tmax > h[j] ? tmax : h[j];
      mine += h[j] != 0u;
    }
    mine = wave_sum(mine);
    tmax = wave_max_u32(tmax);
    uint32_t hm = 0u;
#pragma unroll
    for (int j = 0; j < PER; ++j) hm = hm > h[j] ? hm : h[j];
    hm = wave_max_u32(hm);
    if (tid == 0) eps_s = eps2[qid];
    if (lane == 0) {
      s.wred[w] = mine;
      s.wmax[w] = hm;
      bl.wcnt[w] = (int)tmax;  // (orderable keys as int: only compared after the reinterpret)
    }
  }
  __syncthreads();
  uint32_t tau_max = 0u, hmax = 0u;
#pragma unroll
  for (int i = 0; i < SM_WAVES; ++i) {
    const uint32_t y = (uint32_t)bl.wcnt[i], z = s.wmax[i];
    tau_max = tau_max > y ? tau_max : y;
    hmax = hmax > z ? hmax : z;
  }
  TT_FTS();
  int n_keys = 0;
#pragma unroll
  for (int i = 0; i < SM_WAVES; ++i) n_keys += s.wred[i];
  if (n_keys < k) {  // (a NaN query: no finite score anywhere) -> exact fallback
    if (tid == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  if (TT_EXP_FINAL_STOP == 1) return;
  const float A = key_float(small_radix_select(h, k, s, hmax));
  TT_FTS();
  if (TT_EXP_FINAL_STOP == 2) return;
  const float thr = A - eps_s;
  if (tau_max != 0u && key_float(tau_max) >= thr) {  // a slab may have dropped a band row
    if (tid == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  // band = keys with a >= A - 2 eps; their exact keys came from the streaming kernel
  int pos;
  const int nb = band_positions<EP>(h, thr, bl, &pos);
  if (nb > BAND_CAP) {
    if (tid == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  bool bad_row = false;  // a decoded row >= n_rows (corrupted key): exact fallback instead
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (h[j] != 0u && key_float(h[j]) >= thr) {
      bad_row |= xk[j] != 0ull && (int64_t)key_row(xk[j]) >= n_rows;
      bl.sbuf[pos++] = xk[j];
    }
  if (__syncthreads_or(bad_row)) {
    if (tid == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  TT_FTS();
  band_rank_out<EP>(bl, nb, qid, k, row_base, out_s, out_i);
  TT_FTS();
#if TT_EXP_FINAL_TIMING
  if (qid == 0 && tid == 0)
    printf("final_topm ticks: collect %d select %d band %d rank %d (nb %d) max %.4f A %.4f n %d\n",
           (int)(ts[1] - ts[0]), (int)(ts[2] - ts[1]), (int)(ts[3] - ts[2]), (int)(ts[4] - ts[3]),
           nb, key_float(hmax), A, n_keys);
#endif
#undef TT_FTS
}

// ------------------------------------------------------ single pass on the int8 image (nq <= 8)
// The one-buyer search reads the whole catalog image once, so its time is that image's bytes
// (bf16: 768 MB at 1M x 384, ~124 us at 6.2 TB/s).  An int8 image (tt_i8_image: 64-row tiles
// of codes n and one scale s) halves them.  The bound is looser than bf16's but still a
// rigorous one: with the query coded per query as t m (t = max |q| / 127, m = rint(q / t)),
//   |x.q - s t (n.m)| <= ||x - s n|| ||q|| + s ||n|| ||q - t m||
// and a = fl(fl(n.m) fl(s t)) (n.m exact in i32 and in f32: |n.m| <= 384 * 127^2 < 2^24) adds
// at most 2^-23 s ||n|| t ||m||, the canonical f32 chain at most E 2^-24 X ||q||:
//   eps = 1.001 (R ||q|| + S ||q - t m|| + 2^-23 S (||q|| + ||q - t m||) + 1.01 E 2^-24 X ||q||)
// with X, R, S the image's bounds (max ||x||, max ||x - s n||, max s ||n||; ~1, 0.0136, 1.003 on
// unit rows): eps ~0.02 (bf16: ~0.004).
// The stream, the per-(query, slab) streaming top-16 and the exact keys of the kept rows are
// k_filter_topm's, on v_mfma_i32_16x16x64_i8 (64-row tiles: 24 KB, the bf16 ring's tile size).
// The final certifies with exact scores instead of a band: a row a slab dropped has a <= tau_b
// (the slab list's 16th approximate score), so its exact score s <= tau_b + eps.  If
// max_b tau_b + eps < S_k, the k-th best EXACT score among the kept rows, no dropped row can
// reach the top k, which is then the kept rows' exact top k.  Otherwise the query takes the
// exact fallback.  (One eps instead of the band's two: on iid and Mode B queries the margin
// S_k - max tau - eps is 0.015-0.03, tools/i8_sim in DESIGN 4.1c.)
constexpr int I8_MAXTILES = 1024;  // 64-row scale tiles per block (rows_per_blk <= 65536)
#ifndef TT_I8_SLOTS
#define TT_I8_SLOTS 4  // ring slots of the int8 single pass (tiles in flight + 1)
#endif
TT_CHECK_EXP(TT_I8_SLOTS != 4, "TT_I8_SLOTS");
#ifndef TT_I8_SWZ
#define TT_I8_SWZ 1  // 0: XOR swizzle by r & 7 (2-way bank conflicts at E = 384), 1: by (r >> 1) & 7
#endif
TT_CHECK_EXP(TT_I8_SWZ != 1, "TT_I8_SWZ");
#ifndef TT_I8_DMAW
#define TT_I8_DMAW 1  // 1: only the waves that run no MFMA issue the ring's DMA (0: all waves)
#endif
TT_CHECK_EXP(TT_I8_DMAW != 1, "TT_I8_DMAW");
#ifndef TT_I8_EXP_NOCOMP
#define TT_I8_EXP_NOCOMP 0  // timing only (results WRONG): the int8 stream without compute
#endif
TT_CHECK_EXP(TT_I8_EXP_NOCOMP, "TT_I8_EXP_NOCOMP");
#ifndef TT_I8_EXP_PART
#define TT_I8_EXP_PART 0  // timing only (results WRONG): 1 no appends, 2 no LDS reads, 3 no MFMA
#endif
TT_CHECK_EXP(TT_I8_EXP_PART, "TT_I8_EXP_PART");
#ifndef TT_I8_EXP_CLK
#define TT_I8_EXP_CLK 0  // timing only: per-wave cycle split of the int8 stream's tile loop
#endif
TT_CHECK_EXP(TT_I8_EXP_CLK, "TT_I8_EXP_CLK");
#if TT_I8_EXP_CLK
__device__ unsigned long long g_i8clk[256 * TM_WAVES * 8];
#define I8CLK(i)                                               \
  do {                                                         \
    const unsigned long long c1_ = __builtin_amdgcn_s_memtime(); \
    ck[i] += c1_ - c0_;                                        \
    c0_ = c1_;                                                 \
  } while (0)
#else
#define I8CLK(i) \
  do {           \
  } while (0)
#endif
// 16-B chunk swizzle of an int8 tile row r (XOR of the chunk index within aligned groups of
// 8 / 16 chunks): the 16 rows a ds_read_b128 lane group reads must land in 16 different
// 16-B bank groups.  E = 384: 24 chunks per row, 24 = 8 mod 16, so rows r and r + 1 are 8
// bank groups apart -- XOR by (r >> 1) & 7 spreads each row pair over the other 8 (r & 7 put
// rows r and r + 8 on one bank group).  E = 768: 48 chunks = 0 mod 16: XOR by r & 15.
template <int EP>
__device__ __forceinline__ int i8_swz(int r) {
  return EP == 768 ? (r & 15) : TT_I8_SWZ ? ((r >> 1) & 7) : (r & 7);
}

template <int EP, int QB>
__global__ __launch_bounds__(64 * TM_WAVES, 1) void k_filter_topm_i8(
    const int8_t* __restrict__ xc, int64_t ldc, const float* __restrict__ scales, int64_t n,
    const float* __restrict__ q, int nq, int64_t ldq, int rows_per_blk,
    const float* __restrict__ db, int64_t ld, float X, float R, float S,
    float* __restrict__ eps1, uint64_t* __restrict__ lists, uint64_t* __restrict__ xkeys,
    int* __restrict__ counts, int* __restrict__ flags, int* __restrict__ qsel_n) {
  static_assert(EP == 384 || EP == 768, "int8 single pass: E = 384 or 768");
  constexpr int TR = 24576 / EP, KS = EP / 64, CPR = EP / 16, RB = TR / 16;
  // the ring's 1-KB DMA pieces per tile, issued by DW waves (PPW each): with TT_I8_DMAW the
  // TM_WAVES - RB waves that run no MFMA, so the compute waves' per-tile path carries no
  // address arithmetic or memory-pipe stalls and needs no vmcnt wait (the barrier after the
  // issuing waves' waits orders every piece)
  constexpr int DW = TT_I8_DMAW ? TM_WAVES - RB : TM_WAVES, DW0 = TM_WAVES - DW;
  constexpr int TILE_B = TR * EP, PIECES = TILE_B / 1024, PPW = PIECES / DW;
  constexpr int SLOTS = TT_I8_SLOTS, PD = SLOTS - 1;
  static_assert(PIECES % DW == 0 && CPR % 16 == 8 * (EP == 384), "tile layout");
  __shared__ __attribute__((aligned(16))) char smem[SLOTS * TILE_B + TM_NQ * TM_BUF * 8];
  __shared__ int ncs[TM_NQ];
  __shared__ float ssc[I8_MAXTILES];
  char* ring = smem;
  uint64_t* tbuf = (uint64_t*)(smem + SLOTS * TILE_B);  // [TM_NQ][TM_BUF]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int G = gridDim.x, blk = blockIdx.x;
  if (blk == 0 && tid < nq) {  // per-query fallback state (FilterWs: flags, qsel, qsel_n, done)
    flags[tid] = 0;
    qsel_n[1 + tid] = 0;
    if (tid == 0) *qsel_n = 0;
  }
  const int64_t j0 = (int64_t)blk * rows_per_blk;  // rows_per_blk: a multiple of 64
  const int64_t j1 = (j0 + rows_per_blk < n) ? j0 + rows_per_blk : n;
  const int n_tiles = j0 < j1 ? (int)((j1 - j0 + TR - 1) / TR) : 0;
  for (int i = tid; i < (rows_per_blk >> 6); i += 64 * TM_WAVES) {
    const int64_t st = (j0 >> 6) + i;
    ssc[i] = st < ((n + 63) >> 6) ? scales[st] : 0.0f;
  }

  constexpr int TM_QB = QB, CW = RB, TMB = TM_NQ * TM_BUF / TM_QB / CW;
  constexpr int CPER = TMB / 64;
  static_assert(TMB % 64 == 0 && TMB >= 2 * TM_M && CW <= TM_WAVES, "top-m buffer shape");
  const bool cw = w < CW && !TT_I8_EXP_NOCOMP;
  uint64_t* wbuf = tbuf + (cw ? w : 0) * TM_QB * TMB;  // [TM_QB][TMB] per compute wave
  u32x4 qf[KS];
  const bool qv = col < nq;
  // tau bounds shared by the block's compute waves: a row below ANY wave's tau (each a lower
  // bound of the 16th best of distinct rows of this slab) is below the slab's 16th best, so
  // every wave may drop it -- each wave's appends follow the block's max
  __shared__ __attribute__((aligned(16))) float tau_sh[QB][4];
  if (TT_TM_SHTAU && w < 4 && lane < QB) tau_sh[lane][w] = -__builtin_huge_valf();
  float tq = 0.0f;  // the query's code scale t
  float tau = qv ? -__builtin_huge_valf() : __builtin_huge_valf();
  int cnt = 0;
  // tile-max bound of tau (appends): the 16 largest of the set, ascending (tm[0] = the 16th)
  float tm[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) tm[i] = -__builtin_huge_valf();
  // insert m: clamp(m, tm[i], tm[i + 1]) per entry = the sorted 16 largest of the set plus m
  // (one v_med3 each, branch-free; a no-op when m <= tm[0]); NaN enters as -inf
  auto tm_insert = [&](float m) __attribute__((always_inline)) {
    m = m == m ? m : -__builtin_huge_valf();
#pragma unroll
    for (int i = 0; i < 15; ++i) tm[i] = __builtin_amdgcn_fmed3f(tm[i], m, tm[i + 1]);
    tm[15] = fmaxf(tm[15], m);
  };
  // the block's shared tau for this lane's query (issued before the tile's fragment reads:
  // LDS reads complete in order)
  auto read_shtau = [&]() __attribute__((always_inline)) {
    if (!TT_TM_SHTAU) return -__builtin_huge_valf();
    const f32x4 v = *(const f32x4*)&tau_sh[col < QB ? col : 0][0];
    return fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
  };
  if (cw) {
    // the query (column col) coded as t m: lanes (g, col) hold chunks 4s + g, i.e. dims
    // 64 s + 16 g .. + 15 -- the same chunk of every row the MFMA pairs them with
    const float* qp = q + (int64_t)(qv ? col : 0) * ldq + 16 * g;
    float mx = 0.0f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f32x4 v = *(const f32x4*)(qp + 64 * s + 4 * u);
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    tq = mx / 127.0f;
    double sq = 0.0, sd = 0.0;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      uint32_t wd[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f32x4 v = *(const f32x4*)(qp + 64 * s + 4 * u);
        uint32_t pk = 0u;
        // (selects, no branch: a branch per element kept these loads from being hoisted, so
        // they went out one at a time -- ~24 dependent round trips before the ring started)
        const float tdiv = tq > 0.0f ? tq : 1.0f;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          int c = (int)rintf(v[b] / tdiv);
          c = c > 127 ? 127 : c < -127 ? -127 : c;
          c = tq > 0.0f ? c : 0;
          const double e = (double)v[b] - (double)tq * (double)c;
          sq += (double)v[b] * (double)v[b];
          sd += e * e;
          pk |= ((uint32_t)(c & 0xff)) << (8 * b);
        }
        wd[u] = pk;
      }
      qf[s] = u32x4{wd[0], wd[1], wd[2], wd[3]};
    }
    sq += __shfl_xor(sq, 16, 64);
    sd += __shfl_xor(sd, 16, 64);
    sq += __shfl_xor(sq, 32, 64);
    sd += __shfl_xor(sd, 32, 64);
    if (blk == 0 && w == 0 && g == 0 && qv) {
      const double nq2 = sqrt(sq) * 1.000001, nd = sqrt(sd) * 1.000001;
      const double e = 1.001 * ((double)R * nq2 + (double)S * nd +
                                1.1920928955078125e-07 * (double)S * (nq2 + nd) +
                                1.01 * EP * 5.9604644775390625e-08 * (double)X * nq2);
      eps1[col] = e == e ? f64_up(e) : __builtin_huge_valf();
    }
  }
  wait_vm<0>();  // the query / scale loads and init stores retire before the ring's counted waits

  const int64_t tile_bytes = ldc * TR;
  const char* slab_base = (const char*)xc + j0 * ldc;
  const bool dmaw = w >= DW0;
  const int dw = dmaw ? w - DW0 : 0;
  uint32_t voff[PPW];
#pragma unroll
  for (int pp = 0; pp < PPW; ++pp) {
    const int P = (dw + DW * pp) * 64 + lane;
    const int r = P / CPR;
    voff[pp] = (uint32_t)(r * ldc) + 16u * (uint32_t)((P % CPR) ^ i8_swz<EP>(r));
  }
  auto issue = [&](int t) __attribute__((always_inline)) {
    if (!dmaw) return;
    char* slot = ring + (t % SLOTS) * TILE_B;
    const int64_t jt = j0 + (int64_t)t * TR;
    const bool clamp = jt + TR > j1;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(slab_base + (int64_t)t * tile_bytes), 0, (int)tile_bytes, 0x00020000);
#pragma unroll
    for (int pp = 0; pp < PPW; ++pp) {
      uint32_t off = voff[pp];
      if (clamp) {  // rows past the slab end read a copy of its last row (masked below)
        const int P = (dw + DW * pp) * 64 + lane;
        const int r = P / CPR;
        int64_t j = jt + r;
        j = j < j1 ? j : j1 - 1;
        off = (uint32_t)((j - jt) * ldc) + 16u * (uint32_t)((P % CPR) ^ i8_swz<EP>(r));
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(slot + (dw + DW * pp) * 1024), 16,
          off, 0, 0, 2);
    }
  };
  auto wait_tiles = [&](int younger) __attribute__((always_inline)) {
    static_assert(PD <= 4, "wait_tiles covers up to 3 younger tiles");
    if (!dmaw) return;  // issued nothing: the barrier after the issuing waves' waits orders it
    if (younger >= 3) wait_vm<3 * PPW>();
    else if (younger == 2) wait_vm<2 * PPW>();
    else if (younger == 1) wait_vm<PPW>();
    else wait_vm<0>();
  };
  uint32_t lrd[4];
  {
    const int r = 16 * (cw ? w : 0) + col, f = i8_swz<EP>(r), h = f >> 2;
#pragma unroll
    for (int v = 0; v < 4; ++v)
      lrd[v] = lds_addr(ring) + 16 * (r * CPR + (g ^ (f & 3))) + 64 * (v ^ h);
  }
  static_assert(TM_M == 16, "wave_top16 keeps 16");
#if TT_I8_EXP_CLK
  unsigned long long n_any = 0, n_cmp = 0;
#endif
  auto compact = [&](int c) __attribute__((always_inline)) {
    uint64_t* b = wbuf + c * TMB;
    const int cc = __shfl(cnt, c, 64);
    uint64_t key[CPER];
#pragma unroll
    for (int r = 0; r < CPER; ++r) {
      const int e = lane * CPER + r;
      key[r] = e < cc ? b[e] : 0ull;
    }
    int nc;
    const uint64_t k = wave_top16<CPER>(key, lane, b, &nc);
    if (lane < nc) b[lane] = k;
    const uint32_t hk = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(k >> 32), TM_M - 1);
    if (col == c) {
      cnt = nc;
      if (nc == TM_M) tau = fmaxf(tau, key_float(hk));
    }
    wave_sync();
  };
  // appends and the tile-max bound of tau: k_filter_topm's (the scores arrive as f32 here)
  auto appends = [&](f32x4 acc, int t, float shtau) __attribute__((always_inline)) {
    const int64_t jt = j0 + (int64_t)t * TR + 16 * w;
    if (TT_TM_SHTAU && qv) tau = fmaxf(tau, shtau);
    const uint64_t colmask = 0x0001000100010001ull << col;
    const uint64_t below = (1ull << lane) - 1ull;
    if (jt + 16 > j1) {  // (wave-uniform) the slab's last tile: rows past its end score -inf
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        if (jt + 4 * g + jj >= j1) acc[jj] = -__builtin_huge_valf();
    }
    // late in the slab tau has risen past nearly every row: one ballot skips the four
    const bool any = fmaxf(fmaxf(acc[0], acc[1]), fmaxf(acc[2], acc[3])) >= tau;
    if (!TT_TM_ANYB || __ballot(any) != 0ull) {
#if TT_I8_EXP_CLK
      ++n_any;
#endif
      const int lr0 = t * TR + 16 * w + 4 * g, nloc = (int)(j1 - j0);  // slab-local rows
      if (TT_TM_PREFIX) {
        // one pass for the lane's 4 rows: its pass count, the exclusive prefix over the
        // column's 4 lanes (lane ^ 16, lane ^ 32 partners) and the column's total
        bool pass[4];
        int np = 0;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          pass[jj] = lr0 + jj < nloc && acc[jj] >= tau;
          np += pass[jj] ? 1 : 0;
        }
        const auto x16 = __builtin_amdgcn_permlane16_swap((uint32_t)np, (uint32_t)np, false,
                                                          false);
        const int b = (int)((g & 1) ? x16[0] : x16[1]);  // lane ^ 16
        const int s2 = np + b;
        const auto x32 = __builtin_amdgcn_permlane32_swap((uint32_t)s2, (uint32_t)s2, false,
                                                          false);
        const int s2x = (int)(lane < 32 ? x32[1] : x32[0]);  // lane ^ 32
        int pos = cnt + ((g & 1) ? b : 0) + ((g & 2) ? s2x : 0);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          if (pass[jj]) {
            lds_write64(lds_addr(wbuf + col * TMB + pos),
                        make_key(acc[jj], (uint32_t)(j0 + lr0 + jj)));
            ++pos;
          }
        cnt += s2 + s2x;
      } else {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float v = acc[jj];
          const bool pass = lr0 + jj < nloc && v >= tau;
          const uint64_t bm = __ballot(pass);
          if (bm != 0ull) {
            const uint64_t mc = bm & colmask;
            if (pass) {
              const int pos = cnt + __popcll(mc & below);
              lds_write64(lds_addr(wbuf + col * TMB + pos),
                          make_key(v, (uint32_t)(j0 + lr0 + jj)));
            }
            cnt += __popcll(mc);
          }
        }
      }
    }
    if (t == 0) {  // the first tile's 16 rows (every lane of the column gathers all 16)
      float v16[16];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        v16[jj] = acc[jj];
        const auto x16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[jj]),
                                                          __float_as_uint(acc[jj]), false, false);
        v16[4 + jj] = __uint_as_float((g & 1) ? x16[0] : x16[1]);  // lane ^ 16
      }
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const auto x32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v16[jj]),
                                                          __float_as_uint(v16[jj]), false, false);
        v16[8 + jj] = __uint_as_float(lane < 32 ? x32[1] : x32[0]);  // lane ^ 32
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) tm_insert(v16[i]);
    } else {
      float m = fmaxf(fmaxf(acc[0], acc[1]), fmaxf(acc[2], acc[3]));
      const auto x16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m),
                                                        false, false);
      m = fmaxf(__uint_as_float(x16[0]), __uint_as_float(x16[1]));
      const auto x32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m),
                                                        false, false);
      tm_insert(fmaxf(__uint_as_float(x32[0]), __uint_as_float(x32[1])));  // the tile max
    }
    tau = fmaxf(tau, qv ? tm[0] : tau);
    const uint64_t need = __ballot(lane < 16 && cnt > TMB - 16);
    if (need != 0ull) {
      lds_wait<0>();
      uint64_t nd = need;
      while (nd) {
        const int c = __builtin_ctzll(nd);
        nd &= nd - 1;
        compact(c);
#if TT_I8_EXP_CLK
        ++n_cmp;
#endif
      }
    }
    if (TT_TM_SHTAU && qv && g == 0) tau_sh[col][w] = tau;  // published for the other waves
  };

  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#if TT_I8_EXP_CLK
  unsigned long long ck[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long c0_ = __builtin_amdgcn_s_memtime();
  const unsigned long long cstart = c0_;
#endif
  for (int t = 0; t < PD && t < n_tiles; ++t) issue(t);
  for (int t = 0; t < n_tiles; ++t) {
    wait_tiles(n_tiles - 1 - t < PD - 1 ? n_tiles - 1 - t : PD - 1);
    I8CLK(0);
    lds_barrier();  // tile t landed (every wave's pieces); every wave is done with tile t-1
    I8CLK(1);
    if (t + PD < n_tiles) issue(t + PD);
    I8CLK(2);
    if (cw) {
      const float shtau = read_shtau();
      const uint32_t so = (uint32_t)((t % SLOTS) * TILE_B);
      u32x4 fr[KS];
      static_for<KS>([&](auto s_) __attribute__((always_inline)) {
        constexpr int Sx = decltype(s_)::value;
        if (TT_I8_EXP_PART == 2)
          fr[Sx] = qf[Sx] ^ (uint32_t)t;
        else
          fr[Sx] = lds_read128<256 * (Sx / 4)>(lrd[Sx % 4] + so);
      });
      // the tile's scale (its 64-row scale tile) x the query's t: one product per lane
      const float st = ssc[(int)(((int64_t)t * TR) >> 6)] * tq;
      I8CLK(6);
      if (t > 0 && TT_I8_EXP_PART != 1) appends(acc, t - 1, shtau);
      I8CLK(3);
      lds_wait<0>();
      I8CLK(4);
      i32x4 ai = {0, 0, 0, 0};
      static_for<KS>([&](auto s_) __attribute__((always_inline)) {
        constexpr int Sx = decltype(s_)::value;
        reg_tie(fr[Sx]);
        if (TT_I8_EXP_PART == 3)
          ai += __builtin_bit_cast(i32x4, fr[Sx]);
        else
          ai = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, fr[Sx]),
                                                     __builtin_bit_cast(i32x4, qf[Sx]), ai, 0, 0,
                                                     0);
      });
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[jj] = (float)ai[jj] * st;
      I8CLK(5);
    }
  }
#if TT_I8_EXP_CLK
  if (lane == 0 && blk < 256) {
    ck[8] = __builtin_amdgcn_s_memtime() - cstart;
    ck[7] = (unsigned long long)n_tiles;
    ck[3] += ck[6] << 32;  // 3: appends (low word), reads (high word)
    ck[4] += n_any << 32;  // tiles whose appends ran / compactions (high words)
    ck[5] += n_cmp << 32;
    ck[6] = ck[8];
    for (int i = 0; i < 8; ++i) g_i8clk[(blk * TM_WAVES + w) * 8 + i] = ck[i];
  }
#endif
  if (cw && n_tiles > 0) appends(acc, n_tiles - 1, read_shtau());
  wait_vm<0>();
  __shared__ int ncw[CW][TM_NQ];
  if (w < CW && lane < nq && g == 0) ncw[w][lane] = cnt;  // (0 when TT_I8_EXP_NOCOMP)
  lds_wait<0>();
  __syncthreads();
  for (int c = w; c < nq; c += TM_WAVES) {
    uint64_t key[CW * CPER];
#pragma unroll
    for (int wb = 0; wb < CW; ++wb) {
      const int cc = ncw[wb][c];
#pragma unroll
      for (int r = 0; r < CPER; ++r) {
        const int e = lane * CPER + r;
        key[wb * CPER + r] = e < cc ? tbuf[(wb * TM_QB + c) * TMB + e] : 0ull;
      }
    }
    int nc;
    const uint64_t k = wave_top16<CW * CPER>(key, lane, tbuf + c * TMB, &nc);
    if (lane < nc) {
      tbuf[c * TMB + lane] = k;
      lists[((int64_t)c * G + blk) * TM_M + lane] = k;
    }
    if (lane == 0) {
      counts[(int64_t)c * G + blk] = nc;
      ncs[c] = nc;
    }
  }
  __syncthreads();
  for (int c = w; c < nq; c += TM_WAVES) {
    const int nc = ncs[c], r16 = lane & 15, g4 = 4 * (lane >> 4);
    if (nc == 0) continue;
    const uint64_t* tb = tbuf + c * TMB;
    const f32x4 ex =
        exact16<EP>(db, ld, key_row(tb[r16 < nc ? r16 : 0]), q + (int64_t)c * ldq, lane);
    if (r16 == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (g4 + j < nc)
          xkeys[((int64_t)c * G + blk) * TM_M + g4 + j] =
              ex[j] != ex[j] ? 0ull : make_key(ex[j], key_row(tb[g4 + j]));
    }
  }
}

// The int8 single pass over the TILED int8 image (round 6).  k_filter_topm_i8 stages 64-row
// tiles of the row-major image through an LDS ring with one block barrier per tile: every wave
// waits for the slowest wave's appends and the DMA waves' counted waits each tile, and the
// stream ran at 0.61 of 8 TB/s (its DMA-only floor: 0.78).  Here each of the 8 waves streams
// its OWN 16-row blocks (block b = w, w + 8, ... of the slab) straight into VGPRs, D blocks in
// flight, and runs the per-block work (KS i8 MFMAs, the tile scale, the appends and tile-max
// bound of the previous block) with no barrier in the loop: a slow block delays only its wave.
// Loads straight into MFMA operands need the tiled image (tt_i8_tile): a 16-row block is KS
// 1-KB pieces, piece s holding lane (g, col)'s 16 B = row col's bytes 64 s + 16 g .. + 15, so
// each load instruction reads 1 KB contiguous (tools/stream_probe.hip on MI355X: 7.0 TB/s into
// registers; the row-major image read in the same lane order: 5.5, and 2.5 TB/s with 96
// contiguous bytes per lane).  The query is coded in k_filter_topm_i8's chunk order.
// The loads are inline asm with explicit counted waits (vmcnt((D - 1) KS) before a block is
// consumed) so the compiler neither reorders nor flushes them; blocks past the slab read 0
// from the bounded buffer resource (rows past its end: masked).  Candidate buffers per (wave,
// query): TM_NQ TM_BUF / QB / 8 keys (128 at QB = 4).  The slab's merged top-16 and its exact
// keys are k_filter_topm_i8's, so k_final_topm_i8 is unchanged.
#ifndef TT_I8R_D
#define TT_I8R_D 4  // row blocks in flight per wave (timing builds: other depths)
#endif
TT_CHECK_EXP(TT_I8R_D != 4, "TT_I8R_D");
#ifndef TT_I8R_EXP
#define TT_I8R_EXP 0  // timing only (results WRONG): 1 no appends, 2 no appends and no MFMA
#endif
TT_CHECK_EXP(TT_I8R_EXP, "TT_I8R_EXP");
#ifndef TT_I8R_CLK
#define TT_I8R_CLK 0  // timing only: per-block phase stamps (s_memrealtime, 100 MHz) of the stream
#endif
TT_CHECK_EXP(TT_I8R_CLK, "TT_I8R_CLK");
#if TT_I8R_CLK
__device__ unsigned long long g_i8rclk[256 * 8];
__device__ unsigned long long g_i8fclk[8];  // k_final_topm_i8, query 0
extern "C" int tt_debug_i8r_clk(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_i8rclk), sizeof(g_i8rclk)) == hipSuccess &&
                 hipMemcpyFromSymbol(host + 256 * 8, HIP_SYMBOL(g_i8fclk), sizeof(g_i8fclk)) ==
                     hipSuccess
             ? 0
             : -2;
}
#define I8F_STAMP(i)                                                               \
  do {                                                                             \
    if (tid == 0 && qid == 0) g_i8fclk[i] = __builtin_amdgcn_s_memrealtime();      \
  } while (0)
#define I8R_STAMP(i)                                                               \
  do {                                                                             \
    if (tid == 0 && blk < 256) g_i8rclk[blk * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define I8R_STAMP(i) \
  do {               \
  } while (0)
#define I8F_STAMP(i) \
  do {               \
  } while (0)
#endif
template <int EP>
struct I8RegCfg {
  static constexpr int D = TT_I8R_D;  // row blocks in flight per wave (E = 384: 96 VGPRs)
  static_assert(EP == 384, "E = 768 would need 12 loads per block: D = 2 spills");
};
typedef int32_t i8r_v4i __attribute__((ext_vector_type(4)));

// Up to 32 queries (round 6): NQB = 2 runs two 16-query MFMA blocks on every row block (12
// MFMAs), each with its own tau / tile-max state and candidate lists; with no LDS ring the
// candidate buffers get 128 KB (QB = 16 / 32: 128 / 64 keys per wave and query), so 9-32
// queries stay off the multi-level ladder too.
constexpr int TM_NQ_I8T = 32;  // queries of the tiled int8 single pass
template <int QB>
constexpr int i8r_keys() {  // candidate-buffer keys of k_filter_topm_i8r
  return QB <= 8 ? TM_NQ * TM_BUF : 16384;
}
template <int EP, int QB, int NQB>
__global__ __launch_bounds__(64 * TM_WAVES, 1) void k_filter_topm_i8r(
    const int8_t* __restrict__ xt, int64_t /*unused*/, const float* __restrict__ scales,
    int64_t n, const float* __restrict__ q, int nq, int64_t ldq, int rows_per_blk,
    const float* __restrict__ db, int64_t ld, float X, float R, float S,
    float* __restrict__ eps1, uint64_t* __restrict__ lists, uint64_t* __restrict__ xkeys,
    int* __restrict__ counts, int* __restrict__ flags, int* __restrict__ qsel_n) {
  constexpr int KS = EP / 64, NW = TM_WAVES, D = I8RegCfg<EP>::D, BLK = 16 * EP;
  constexpr int TMB = i8r_keys<QB>() / QB / NW, CPER = TMB / 64, NQ16 = 16 * NQB;
  // a query's buffer every CS keys: the 2-key pad puts the 16 columns' appends (one ds_write
  // per row of the lane) on 16 different bank pairs instead of one bank (TMB * 8 B = 0 mod 256)
  constexpr int CS = TMB + 2;
  static_assert(TMB % 64 == 0 && TMB >= 2 * TM_M && QB <= NQ16 && NQ16 <= QB * 4,
                "top-m buffer shape");
  __shared__ __attribute__((aligned(16))) uint64_t tbuf[NW * QB * CS];  // [NW][QB][CS]
  __shared__ int ncs[QB];
  __shared__ int ncw[NW][QB];
  __shared__ float ssc[I8_MAXTILES];
  __shared__ __attribute__((aligned(16))) float tau_sh[QB][NW];
  __shared__ __attribute__((aligned(16))) float t2_sh[QB][NW];  // each wave's 2nd-largest tm
  __shared__ int next_blk;  // the next unclaimed 16-row block of the slab
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int G = gridDim.x, blk = blockIdx.x;
  I8R_STAMP(0);
  if (tid == 0) next_blk = NW * I8RegCfg<EP>::D;
  if (blk == 0 && tid < nq) {  // per-query fallback state (FilterWs: flags, qsel, qsel_n, done)
    flags[tid] = 0;
    qsel_n[1 + tid] = 0;
    if (tid == 0) *qsel_n = 0;
  }
  const int64_t j0 = (int64_t)blk * rows_per_blk;  // rows_per_blk: a multiple of 64
  const int64_t j1 = (j0 + rows_per_blk < n) ? j0 + rows_per_blk : n;
  const int nb = j0 < j1 ? (int)((j1 - j0 + 15) / 16) : 0;  // 16-row blocks of the slab
  // the slab's blocks as a bounded buffer resource (the tiled image pads the last block)
  const uint64_t sbase = (uint64_t)(uintptr_t)(xt + j0 * EP);
  i8r_v4i rs;
  rs[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)sbase);
  rs[1] = __builtin_amdgcn_readfirstlane((int)((uint32_t)(sbase >> 32) & 0xffffu));
  // (slabs past the catalog end -- j0 >= n at 1M rows over 256 CUs -- get 0 records: every load
  // of theirs reads 0 and touches no memory)
  rs[2] = __builtin_amdgcn_readfirstlane(nb * BLK);
  rs[3] = 0x00020000;
  u32x4 buf[D][KS];
  auto issue = [&](int slot, int b) __attribute__((always_inline)) {  // 16-row block b
    // (piece s at bo + 4096 (s / 4) + immediate 1024 (s % 4): the immediate is 12 bits)
    const uint32_t bo = (uint32_t)(b * BLK + 16 * lane), bo4 = bo + 4096u;
    static_assert(KS == 6, "six pieces per block");
#define TT_I8R_LD(S)                                                          \
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3 nt"         \
               : "=v"(buf[slot][S])                                           \
               : "v"((S) < 4 ? bo : bo4), "s"(rs), "n"(1024 * ((S) % 4))      \
               : "memory")
    TT_I8R_LD(0);
    TT_I8R_LD(1);
    TT_I8R_LD(2);
    TT_I8R_LD(3);
    TT_I8R_LD(4);
    TT_I8R_LD(5);
#undef TT_I8R_LD
  };

  for (int i = tid; i < (rows_per_blk >> 6); i += 64 * NW) {
    const int64_t st = (j0 >> 6) + i;
    ssc[i] = st < ((n + 63) >> 6) ? scales[st] : 0.0f;
  }
  if (lane < QB) {
    tau_sh[lane][w] = -__builtin_huge_valf();
    t2_sh[lane][w] = -__builtin_huge_valf();
  }
  uint64_t* wbuf = tbuf + w * QB * CS;  // [QB][CS] of this wave
  // per query block qb (queries 16 qb + col): validity, tau, count, the tile-max set
  bool qv[NQB];
  float tau[NQB];
  int cnt[NQB];
  float tm[NQB][16];  // the tile-max bound's sets, ascending (k_filter_topm_i8)
#pragma unroll
  for (int qb = 0; qb < NQB; ++qb) {
    qv[qb] = 16 * qb + col < nq;
    tau[qb] = qv[qb] ? -__builtin_huge_valf() : __builtin_huge_valf();
    cnt[qb] = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) tm[qb][i] = -__builtin_huge_valf();
  }
  auto tm_insert = [&](int qb, float m) __attribute__((always_inline)) {
    m = m == m ? m : -__builtin_huge_valf();
#pragma unroll
    for (int i = 0; i < 15; ++i) tm[qb][i] = __builtin_amdgcn_fmed3f(tm[qb][i], m, tm[qb][i + 1]);
    tm[qb][15] = fmaxf(tm[qb][15], m);
  };
  // The block's shared bound for query c: the largest of the waves' taus, and the smallest of
  // the waves' second-largest tile-max entries -- the 8 waves' two largest entries are the
  // scores of 16 distinct rows of the slab (disjoint blocks per wave, distinct rows within a
  // set), all >= that minimum, so the slab's 16th best is too.  (Each wave's own 16th of ~46
  // entries sat near the rows' 85th percentile: ~80 appends per wave and query, and at 32
  // queries 56 compactions per wave; TT_I8R_CLK.)
  static_assert(2 * NW == TM_M, "the waves' two largest entries make 16 rows");
  auto read_shtau = [&](int qb) __attribute__((always_inline)) {
    const int c = 16 * qb + col < QB ? 16 * qb + col : 0;
    const f32x4* p = (const f32x4*)&tau_sh[c][0];
    const f32x4 a = p[0], b = p[1];
    const f32x4* p2 = (const f32x4*)&t2_sh[c][0];
    const f32x4 a2 = p2[0], b2 = p2[1];
    return fmaxf(fmaxf(fmaxf(fmaxf(a[0], a[1]), fmaxf(a[2], a[3])),
                       fmaxf(fmaxf(b[0], b[1]), fmaxf(b[2], b[3]))),
                 fminf(fminf(fminf(a2[0], a2[1]), fminf(a2[2], a2[3])),
                       fminf(fminf(b2[0], b2[1]), fminf(b2[2], b2[3]))));
  };
  // the queries (column col of block qb) coded as t m, lane (g, col) holding dims 64 s + 16 g ..
  // + 15 for MFMA step s: the bytes the lane loads of every row (the tiled image's piece s).
  // The 24 16-B units su = 4 s + u of a lane are split over the 8 waves (3 each) and the codes
  // meet in LDS: the fully unrolled per-wave form (2,660 ISA lines before the first load) made
  // the prologue 10.7 of the 77 us launch (TT_I8R_CLK); this one is 2.5 us
  static_assert(KS * 4 == 3 * NW, "three 16-B query units per wave");
  __shared__ __attribute__((aligned(16))) float qmx[NQ16][NW];
  __shared__ double qsq[NQ16][NW], qsd[NQ16][NW];
  __shared__ uint32_t qcode[NQB][KS * 4][64];
  float tq[NQB];
  {
    f32x4 v[NQB][3];
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb) {
      const float* qp = q + (int64_t)(qv[qb] ? 16 * qb + col : 0) * ldq + 16 * g;
      float mx = 0.0f;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int su = 3 * w + j;
        v[qb][j] = *(const f32x4*)(qp + 64 * (su >> 2) + 4 * (su & 3));
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[qb][j][0]), fabsf(v[qb][j][1])),
                             fmaxf(fabsf(v[qb][j][2]), fabsf(v[qb][j][3]))));
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      if (g == 0) qmx[16 * qb + col][w] = mx;
    }
    __syncthreads();
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb) {
      const f32x4* p = (const f32x4*)&qmx[16 * qb + col][0];
      const f32x4 a = p[0], b = p[1];
      const float mx = fmaxf(fmaxf(fmaxf(a[0], a[1]), fmaxf(a[2], a[3])),
                             fmaxf(fmaxf(b[0], b[1]), fmaxf(b[2], b[3])));
      tq[qb] = mx / 127.0f;
      double sq = 0.0, sd = 0.0;
      const float tdiv = tq[qb] > 0.0f ? tq[qb] : 1.0f;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        uint32_t pk = 0u;
#pragma unroll
        for (int b = 0; b < 4; ++b) {  // (selects, no branch: see k_filter_topm_i8)
          const float x = v[qb][j][b];
          int c = (int)rintf(x / tdiv);
          c = c > 127 ? 127 : c < -127 ? -127 : c;
          c = tq[qb] > 0.0f ? c : 0;
          const double e = (double)x - (double)tq[qb] * (double)c;
          sq += (double)x * (double)x;
          sd += e * e;
          pk |= ((uint32_t)(c & 0xff)) << (8 * b);
        }
        qcode[qb][3 * w + j][lane] = pk;
      }
      sq += __shfl_xor(sq, 16, 64);
      sd += __shfl_xor(sd, 16, 64);
      sq += __shfl_xor(sq, 32, 64);
      sd += __shfl_xor(sd, 32, 64);
      if (g == 0) {
        qsq[16 * qb + col][w] = sq;
        qsd[16 * qb + col][w] = sd;
      }
    }
  }
  wait_vm<0>();     // every compiler-issued load retired: the loop's counted waits see only its own
  __syncthreads();  // ssc, tau_sh, the query codes
  u32x4 qf[NQB][KS];
#pragma unroll
  for (int qb = 0; qb < NQB; ++qb)
#pragma unroll
    for (int s = 0; s < KS; ++s)
      qf[qb][s] = u32x4{qcode[qb][4 * s][lane], qcode[qb][4 * s + 1][lane],
                        qcode[qb][4 * s + 2][lane], qcode[qb][4 * s + 3][lane]};
  if (blk == 0 && w < NQB && g == 0 && 16 * w + col < nq) {  // eps of query 16 w + col
    double sq = 0.0, sd = 0.0;
#pragma unroll
    for (int wb = 0; wb < NW; ++wb) {
      sq += qsq[16 * w + col][wb];
      sd += qsd[16 * w + col][wb];
    }
    const double nq2 = sqrt(sq) * 1.000001, nd = sqrt(sd) * 1.000001;
    const double e = 1.001 * ((double)R * nq2 + (double)S * nd +
                              1.1920928955078125e-07 * (double)S * (nq2 + nd) +
                              1.01 * EP * 5.9604644775390625e-08 * (double)X * nq2);
    eps1[16 * w + col] = e == e ? f64_up(e) : __builtin_huge_valf();
  }
  wait_vm<0>();  // (the eps stores retired: the loop's counted waits see only its own loads)
  I8R_STAMP(1);

  static_assert(TM_M == 16, "wave_top16 keeps 16");
  // compaction of query c's buffer (of this wave) to its top 16
#if TT_I8R_CLK
  unsigned long long n_cmp = 0, n_any = 0;
#endif
  auto compact = [&](int qb, int c16) __attribute__((always_inline)) {
#if TT_I8R_CLK
    ++n_cmp;
#endif
    const int c = 16 * qb + c16;
    uint64_t* b = wbuf + c * CS;
    const int cc = __shfl(cnt[qb], c16, 64);
    uint64_t key[CPER];
#pragma unroll
    for (int r = 0; r < CPER; ++r) {
      const int e = lane * CPER + r;
      key[r] = e < cc ? b[e] : 0ull;
    }
    int nc;
    const uint64_t k = wave_top16<CPER>(key, lane, b, &nc);
    if (lane < nc) b[lane] = k;
    const uint32_t hk = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(k >> 32), TM_M - 1);
    if (col == c16) {
      cnt[qb] = nc;
      if (nc == TM_M) tau[qb] = fmaxf(tau[qb], key_float(hk));
    }
    wave_sync();
  };
  // Cutting query c's buffer: first drop its keys below the query's current tau (a valid lower
  // bound of the slab's 16th best, so nothing it drops can be in the slab's top 16 -- early
  // appends fall below it once tau has risen): one ballot pass.  Only a buffer that is still
  // longer than lim is compacted to its top 16 (wave_top16, ~1 us).  (Compacting every full
  // buffer: 30 compactions per wave at 32 queries, ~1/4 of that launch; TT_I8R_CLK.)
  auto cut = [&](int qb, int c16, int lim) __attribute__((always_inline)) {
    const int c = 16 * qb + c16;
    uint64_t* bb = wbuf + c * CS;
    const int cc = __shfl(cnt[qb], c16, 64);
    const float tc = __shfl(tau[qb], c16, 64);
    uint64_t key[CPER];
#pragma unroll
    for (int r = 0; r < CPER; ++r) {
      const int e = lane * CPER + r;
      key[r] = e < cc ? bb[e] : 0ull;
    }
    wave_sync();
    int base = 0;
#pragma unroll
    for (int r = 0; r < CPER; ++r) {
      const bool keep = key[r] != 0ull && key_float((uint32_t)(key[r] >> 32)) >= tc;
      const uint64_t bm = __ballot(keep);
      const int pos = base + (int)__builtin_amdgcn_mbcnt_hi(
                                 (uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
      if (keep) bb[pos] = key[r];
      base += __popcll(bm);
    }
    wave_sync();
    if (col == c16) cnt[qb] = base;
    if (base > lim) compact(qb, c16);  // (wave-uniform)
  };
  auto compact_over = [&](int qb, int lim) __attribute__((always_inline)) {
    const uint64_t need = __ballot(lane < 16 && cnt[qb] > lim);
    if (need != 0ull) {
      lds_wait<0>();
      uint64_t nd = need;
      while (nd) {
        const int c16 = __builtin_ctzll(nd);
        nd &= nd - 1;
        cut(qb, c16, lim);
      }
    }
  };
  // appends of block bl for query block qb (first: the wave's first block) and the tile-max
  // bound: k_filter_topm_i8's
  auto appends = [&](int qb, f32x4 acc, int bl, bool first,
                     float shtau) __attribute__((always_inline)) {
    const int64_t jt = j0 + 16 * (int64_t)bl;
    const int c = 16 * qb + col;
    if (qv[qb]) tau[qb] = fmaxf(tau[qb], shtau);
    if (jt + 16 > j1) {  // (wave-uniform) the slab's last block: rows past its end score -inf
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        if (jt + 4 * g + jj >= j1) acc[jj] = -__builtin_huge_valf();
    }
    const bool any = fmaxf(fmaxf(acc[0], acc[1]), fmaxf(acc[2], acc[3])) >= tau[qb];
    if (__ballot(any) != 0ull) {
#if TT_I8R_CLK
      ++n_any;
#endif
      const int lr0 = 16 * bl + 4 * g, nloc = (int)(j1 - j0);  // slab-local rows
      bool pass[4];
      int np = 0;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        pass[jj] = lr0 + jj < nloc && acc[jj] >= tau[qb];
        np += pass[jj] ? 1 : 0;
      }
      const auto x16 = __builtin_amdgcn_permlane16_swap((uint32_t)np, (uint32_t)np, false, false);
      const int b = (int)((g & 1) ? x16[0] : x16[1]);  // lane ^ 16
      const int s2 = np + b;
      const auto x32 = __builtin_amdgcn_permlane32_swap((uint32_t)s2, (uint32_t)s2, false, false);
      const int s2x = (int)(lane < 32 ? x32[1] : x32[0]);  // lane ^ 32
      int pos = cnt[qb] + ((g & 1) ? b : 0) + ((g & 2) ? s2x : 0);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        if (pass[jj]) {
          lds_write64(lds_addr(wbuf + (c < QB ? c : 0) * CS + pos),
                      make_key(acc[jj], (uint32_t)(j0 + lr0 + jj)));
          ++pos;
        }
      cnt[qb] += s2 + s2x;
    }
    if (first) {  // the wave's first block: its 16 rows (every lane of the column gathers all 16)
      float v16[16];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        v16[jj] = acc[jj];
        const auto x16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[jj]),
                                                          __float_as_uint(acc[jj]), false, false);
        v16[4 + jj] = __uint_as_float((g & 1) ? x16[0] : x16[1]);
      }
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const auto x32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v16[jj]),
                                                          __float_as_uint(v16[jj]), false, false);
        v16[8 + jj] = __uint_as_float(lane < 32 ? x32[1] : x32[0]);
      }
#pragma unroll
      for (int k2 = 0; k2 < 16; ++k2) tm_insert(qb, v16[k2]);
    } else {
      float m = fmaxf(fmaxf(acc[0], acc[1]), fmaxf(acc[2], acc[3]));
      const auto x16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m),
                                                        false, false);
      m = fmaxf(__uint_as_float(x16[0]), __uint_as_float(x16[1]));
      const auto x32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m),
                                                        false, false);
      tm_insert(qb, fmaxf(__uint_as_float(x32[0]), __uint_as_float(x32[1])));  // the block max
    }
    tau[qb] = fmaxf(tau[qb], qv[qb] ? tm[qb][0] : tau[qb]);
    compact_over(qb, TMB - 16);
    if (qv[qb] && g == 0) {  // published for the other waves
      tau_sh[c][w] = tau[qb];
      t2_sh[c][w] = tm[qb][14];
    }
  };

  // Blocks are handed out dynamically: slot d of wave w starts on block w + NW d, and every
  // consumed slot claims the next block from a block-wide LDS counter, so a wave whose loads
  // come back early takes more of the slab and all 8 keep D blocks in flight to the end (with
  // the static round-robin split, wave 0 left the loop ~14 us before the block's last wave:
  // TT_I8R_CLK at 1M rows).  Claims are made in processing order and only grow, so the first
  // slot holding a block >= nb ends the wave's loop; its later slots hold larger blocks.
  // (Issuing the first blocks before the prologue, so their round trip overlaps the query's,
  // measured neutral: prologue 2.5 -> 7.7 us, loop 52.8 -> 47.8 us -- HBM-bound throughout.)
  f32x4 acc[NQB];
  int bid[D];
  static_for<D>([&](auto d_) __attribute__((always_inline)) {
    constexpr int d = decltype(d_)::value;
    bid[d] = w + NW * d;
    issue(d, bid[d]);
  });
  // The slot is a run-time (wave-uniform) index: only the per-slot pieces (the wait-and-MFMA
  // of a slot's registers, its next issue) are switched over, and the appends -- the bulk of
  // the loop's code -- appear once.  (Unrolling the loop over the D slots put D copies of them
  // in the loop: 10.5k instructions at 32 queries, and that build ran 0.27 ms per search.)
  int prev = -1;  // the block whose scores acc holds (its appends run one block later)
  bool first = true;
  for (int dcur = 0;;) {
    int b = 0;
    static_for<D>([&](auto d_) __attribute__((always_inline)) {
      if (dcur == decltype(d_)::value) b = bid[decltype(d_)::value];
    });
    const bool live = b < nb;  // (wave-uniform; the first slot at or past nb ends the loop)
    i32x4 ai[NQB];
    float sb = 0.0f;
    float shtau[NQB];
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb) shtau[qb] = read_shtau(qb);
    if (live) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * KS) : "memory");
      sb = ssc[b >> 2];  // the block's 64-row scale tile
      static_for<D>([&](auto d_) __attribute__((always_inline)) {
        constexpr int d = decltype(d_)::value;
        if (dcur == d) {
#pragma unroll
          for (int s = 0; s < KS; ++s) reg_tie(buf[d][s]);
#pragma unroll
          for (int qb = 0; qb < NQB; ++qb) {
            ai[qb] = i32x4{0, 0, 0, 0};
#pragma unroll
            for (int s = 0; s < KS; ++s) {
              if (TT_I8R_EXP == 2)
                ai[qb] += __builtin_bit_cast(i32x4, buf[d][s]);
              else
                ai[qb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
                    __builtin_bit_cast(i32x4, buf[d][s]), __builtin_bit_cast(i32x4, qf[qb][s]),
                    ai[qb], 0, 0, 0);
            }
          }
        }
      });
    }
    if (prev >= 0 && TT_I8R_EXP == 0) {
#pragma unroll
      for (int qb = 0; qb < NQB; ++qb) appends(qb, acc[qb], prev, first, shtau[qb]);
      first = false;
    }
    if (!live) break;
    if (TT_I8R_EXP && acc[0][0] == 1.2345f) tau_sh[0][w] = acc[0][1];  // keeps the work live
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[qb][jj] = (float)ai[qb][jj] * (sb * tq[qb]);
    prev = b;
    // the next block for this slot (past nb: reads 0 and ends the loop when reached); issued
    // after acc is converted, i.e. after the MFMAs that read the slot's registers completed
    int nx = 0;
    if (lane == 0) nx = __hip_atomic_fetch_add(&next_blk, 1, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
    nx = __builtin_amdgcn_readfirstlane(nx);
    __builtin_amdgcn_sched_barrier(0);
    static_for<D>([&](auto d_) __attribute__((always_inline)) {
      constexpr int d = decltype(d_)::value;
      if (dcur == d) {
        bid[d] = nx;
        issue(d, nx);
      }
    });
    __builtin_amdgcn_sched_barrier(0);
    dcur = dcur + 1 == D ? 0 : dcur + 1;
  }
  // every load retired before its registers are given back
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int d = 0; d < D; ++d)
#pragma unroll
    for (int s = 0; s < KS; ++s) reg_tie(buf[d][s]);
#if TT_I8R_CLK
  if (tid == 0 && blk < 256) {
    g_i8rclk[blk * 8 + 5] = n_cmp;
    g_i8rclk[blk * 8 + 6] = n_any;
  }
#endif
  // Each wave cuts its own lists for the merge (8 x at most 16 keys per query) by the block's
  // final shared bound (every wave's last tau and second-largest entry is published), which
  // leaves a few keys per wave and query; a list still longer than 16 is compacted.
  // (Compacting every list to 16 cost ~1 us per query and wave: 18.6 us of epilogue at 16
  // queries, 37 at 32.)
  lds_wait<0>();
  __syncthreads();
#pragma unroll
  for (int qb = 0; qb < NQB; ++qb) {
    const float bnd = read_shtau(qb);
    if (qv[qb]) tau[qb] = fmaxf(tau[qb], bnd);
    compact_over(qb, TM_M);
  }
  I8R_STAMP(2);
#pragma unroll
  for (int qb = 0; qb < NQB; ++qb)
    if (lane < 16 && 16 * qb + lane < nq) ncw[w][16 * qb + lane] = cnt[qb];
  lds_wait<0>();
  __syncthreads();
  I8R_STAMP(3);
  static_assert(NW * TM_M == 128, "the merge holds 2 keys per lane");
  for (int c = w; c < nq; c += NW) {
    uint64_t key[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {  // key e = 2 lane + r: wave e / 16's e % 16-th
      const int e = 2 * lane + r, wb = e >> 4, idx = e & 15;
      key[r] = idx < ncw[wb][c] ? tbuf[(wb * QB + c) * CS + idx] : 0ull;
    }
    int nc;
    const uint64_t k = wave_top16<2>(key, lane, tbuf + c * CS, &nc);
    if (lane < nc) {
      tbuf[c * CS + lane] = k;
      lists[((int64_t)c * G + blk) * TM_M + lane] = k;
    }
    if (lane == 0) {
      counts[(int64_t)c * G + blk] = nc;
      ncs[c] = nc;
    }
  }
  __syncthreads();
  I8R_STAMP(7);
  for (int c = w; c < nq; c += NW) {
    const int nc = ncs[c], r16 = lane & 15, g4 = 4 * (lane >> 4);
    if (nc == 0) continue;
    const uint64_t* tb = tbuf + c * CS;
    const f32x4 ex =
        exact16<EP>(db, ld, key_row(tb[r16 < nc ? r16 : 0]), q + (int64_t)c * ldq, lane);
    if (r16 == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (g4 + j < nc)
          xkeys[((int64_t)c * G + blk) * TM_M + g4 + j] =
              ex[j] != ex[j] ? 0ull : make_key(ex[j], key_row(tb[g4 + j]));
    }
  }
  I8R_STAMP(4);
}

// Final of the int8 single pass, one block per query: the union U of the G slab lists' exact
// keys; S_k = the k-th best exact score of U (radix select on the exact keys); certified when
// every full list's tau_b (its 16th approximate score) has tau_b + eps < S_k (see above);
// then U's keys with score >= S_k are ranked into the output (ties at S_k by row).
template <int EP>
__global__ __launch_bounds__(SM_THREADS) void k_final_topm_i8(
    const uint64_t* __restrict__ lists, const uint64_t* __restrict__ xkeys,
    const int* __restrict__ counts, int G, int k, const float* __restrict__ eps1,
    int* __restrict__ flags, int* qsel, int* qsel_n, int64_t n_rows, int64_t row_base,
    float* __restrict__ out_s, int64_t* __restrict__ out_i) {
  constexpr int PER = TM_CAP / SM_THREADS;
  __shared__ SmallLdsT<1> s;
  __shared__ BandLds<EP> bl;
  __shared__ uint32_t taus[SM_WAVES];
  const int qid = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  I8F_STAMP(0);
  uint32_t h[PER];
  uint64_t xk[PER];
  {
    int cj[PER];
    uint64_t kk[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int e = tid + j * SM_THREADS, b = e / TM_M;
      const int64_t o = ((int64_t)qid * G + (b < G ? b : 0)) * TM_M + e % TM_M;
      cj[j] = b < G ? counts[(int64_t)qid * G + b] : 0;
      kk[j] = lists[o];
      xk[j] = xkeys[o];
    }
    int mine = 0;
    uint32_t tmax = 0u, hm = 0u;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = (tid + j * SM_THREADS) % TM_M;
      const bool ok = i < cj[j];
      if (!ok) xk[j] = 0ull;
      h[j] = (uint32_t)(xk[j] >> 32);  // exact score (0: no key, or a NaN exact score)
      if (ok && i == TM_M - 1) tmax = tmax > (uint32_t)(kk[j] >> 32) ? tmax : (uint32_t)(kk[j] >> 32);
      mine += h[j] != 0u;
      hm = hm > h[j] ? hm : h[j];
    }
    mine = wave_sum(mine);
    tmax = wave_max_u32(tmax);
    hm = wave_max_u32(hm);
    if (lane == 0) {
      s.wred[w] = mine;
      s.wmax[w] = hm;
      taus[w] = tmax;
    }
  }
  __syncthreads();
  int n_keys = 0;
  uint32_t tau_max = 0u, hmax = 0u;
#pragma unroll
  for (int i = 0; i < SM_WAVES; ++i) {
    n_keys += s.wred[i];
    tau_max = tau_max > taus[i] ? tau_max : taus[i];
    hmax = hmax > s.wmax[i] ? hmax : s.wmax[i];
  }
  if (n_keys < k) {  // (NaN query / rows, or too few kept rows) -> exact fallback
    if (tid == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  I8F_STAMP(1);
  const float Sk = key_float(small_radix_select(h, k, s, hmax));
  I8F_STAMP(2);
  // certification: a row dropped by slab b has exact score <= tau_b + eps (strictly below S_k)
  if (tau_max != 0u && !(key_float(tau_max) + eps1[qid] < Sk)) {
    if (tid == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  int pos;
  const int nb = band_positions<EP>(h, Sk, bl, &pos);
  if (nb > BAND_CAP) {
    if (tid == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  bool bad_row = false;
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (h[j] != 0u && key_float(h[j]) >= Sk) {
      bad_row |= (int64_t)key_row(xk[j]) >= n_rows;
      bl.sbuf[pos++] = xk[j];
    }
  if (__syncthreads_or(bad_row)) {
    if (tid == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  I8F_STAMP(3);
  band_rank_out<EP>(bl, nb, qid, k, row_base, out_s, out_i);
  I8F_STAMP(4);
}

// ------------------------------------------ the batched sample level on the int8 image
// The first level of a large batch (a stride-16 sample, theta = -inf: every 32-row tile's
// maximum is a candidate, k_filter_ring<EP, 3>'s append_tmax) only has to PLACE the full
// level's threshold: its a_J becomes aref, the full level keeps a >= aref - 1.25 eps and the
// re-rank certifies from exact scores that s_k >= aref - eps / 8 (full_theta / full_cert), a
// query failing it takes the exact fallback.  So any estimate of a_J gives exact results; its
// quality only sets how many candidates the full level keeps.  Here the tile maxima come from
// the int8 image (tt_i8_image) at twice the bf16 MFMA rate and half the bytes: the coded
// query (k_query_eps: t m, t = max|q| / 127) against the rows' codes, times the rows' tile
// scale and t (positive, so they commute with the max).  Same lists / counts layout as the
// ring level (key = orderable max << 32 | ~first row of the tile); NaN maxima enter as -inf.
// E = 384, stride 16 (4 consecutive sample rows share one 64-row scale tile): 4 waves x 64
// queries per block, the slab's 64-row chunks through a 4-slot LDS ring (3 in flight,
// global_load_lds per lane: the sample rows are 16 catalog rows apart), per chunk and wave
// 4 row blocks x 4 query blocks x 6 k-steps of v_mfma_i32_16x16x64_i8.
#ifndef TT_SI_WAVES
#define TT_SI_WAVES 4  // waves (x 64 queries) per block of k_sample_i8: 4 (1 per SIMD) or 8
#endif
TT_CHECK_EXP(TT_SI_WAVES != 4, "TT_SI_WAVES");
#ifndef TT_SI_PIPE
#define TT_SI_PIPE 0  // 1: a chunk's epilogue runs between the next chunk's MFMAs (slower: A/B)
#endif
TT_CHECK_EXP(TT_SI_PIPE != 0, "TT_SI_PIPE");
#ifndef TT_SI_CH
#define TT_SI_CH 64  // sample rows per chunk (one barrier each): 64 (4-slot ring) or 128 (3 slots)
#endif
TT_CHECK_EXP(TT_SI_CH != 64, "TT_SI_CH");
#ifndef TT_SI_OCC2
#define TT_SI_OCC2 0  // 1: two 4-wave blocks per CU (3-slot rings, slabs <= 2048 sample rows)
#endif
TT_CHECK_EXP(TT_SI_OCC2 != 0, "TT_SI_OCC2");
#ifndef TT_SI_QBW
#define TT_SI_QBW 4  // 16-query blocks per wave of k_sample_i8 (4: 64 queries; 2: 32)
#endif
TT_CHECK_EXP(TT_SI_QBW != 4, "TT_SI_QBW");
constexpr int SI_NW = TT_SI_WAVES, SI_QBW = TT_SI_QBW, SI_QPB = 16 * SI_QBW * SI_NW;
constexpr int SI_CH = TT_SI_CH;
constexpr int SI_SLOTS = (SI_CH == 64 && !TT_SI_OCC2) ? 4 : 3, SI_RB = SI_CH / 16;
constexpr int SI_NT = SI_CH / 32, SI_BPC = TT_SI_OCC2 ? 2 : 1;
// sample rows per slab (the plan's FL_CAP tiles of 32; 2048 with two blocks per CU)
constexpr int SI_PD = SI_SLOTS - 1, SI_MAXROWS = TT_SI_OCC2 ? 2048 : 32 * FL_CAP;
template <int EP>
__global__ __launch_bounds__(64 * SI_NW, SI_BPC) void k_sample_i8(
    const int8_t* __restrict__ xc, int64_t ldc, const float* __restrict__ scales, int64_t n_rows,
    int64_t n_sample, int rows_per_slab, int n_slabs, const int8_t* __restrict__ q8,
    const float* __restrict__ tq8, int nq, uint64_t* __restrict__ lists,
    int* __restrict__ counts) {
  static_assert(EP == 384, "int8 sample level: E = 384");
  constexpr int KS = EP / 64, CPR = EP / 16, TILE_B = SI_CH * EP, PIECES = TILE_B / 1024;
  constexpr int PPW = PIECES / SI_NW, STRIDE = 16;
  static_assert(PIECES % SI_NW == 0 && CPR == 24, "chunk layout");
  __shared__ __attribute__((aligned(16))) char ring[SI_SLOTS * TILE_B];
  // the slab's row-group scales (4 sample rows = 64 catalog rows = one scale tile), staged once:
  // a global load per chunk in the epilogue stalled on its latency every chunk
  __shared__ float ssc[(SI_MAXROWS + SI_CH) / 4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int slab = (int)(blockIdx.x % (unsigned)n_slabs), qt = (int)(blockIdx.x / (unsigned)n_slabs);
  const int64_t j0 = (int64_t)slab * rows_per_slab;  // sample rows; rows_per_slab % 64 == 0
  const int64_t j1 = j0 + rows_per_slab < n_sample ? j0 + rows_per_slab : n_sample;
  if (j0 >= j1) return;
  const int n_ch = (int)((j1 - j0 + SI_CH - 1) / SI_CH);
  if (tid < SI_QPB) {
    const int qi = qt * SI_QPB + tid;
    if (qi < nq) counts[(int64_t)qi * n_slabs + slab] = (int)((j1 - j0 + 31) / 32);
  }
  // DMA: piece pp of a chunk = LDS bytes [1024 (w + 4 pp), +1024); lane chunk P = 64 (w + 4 pp)
  // + lane = (row r, position pos); its source is chunk pos ^ swz(r) of sample row r (clamped
  // to the slab's last row), so row r's logical chunk c sits at position c ^ swz(r)
  auto issue = [&](int c) __attribute__((always_inline)) {
    char* slot = ring + (c % SI_SLOTS) * TILE_B;
#pragma unroll
    for (int pp = 0; pp < PPW; ++pp) {
      const int P = (w + SI_NW * pp) * 64 + lane;
      const int r = P / CPR;
      int64_t i = j0 + (int64_t)c * SI_CH + r;
      i = i < j1 ? i : j1 - 1;
      const int8_t* src = xc + (i * STRIDE) * ldc + 16 * ((P % CPR) ^ i8_swz<EP>(r));
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)src,
          (__attribute__((address_space(3))) void*)(slot + (w + SI_NW * pp) * 1024), 16, 0, 0);
    }
  };
  for (int c = 0; c < SI_PD && c < n_ch; ++c) issue(c);
  for (int gi = tid; gi < n_ch * (SI_CH / 4); gi += 64 * SI_NW) {
    int64_t i = j0 + 4 * (int64_t)gi;
    i = i < j1 ? i : j1 - 1;  // clamped rows are copies of the slab's last row
    ssc[gi] = scales[(i * STRIDE) >> 6];
  }
  // this wave's 64 queries as B fragments: lanes (g, col) hold chunk 4 s + g of query 16 qb + col
  u32x4 qf[SI_QBW][KS];
  float tqv[SI_QBW];
  const int qbase = qt * SI_QPB + 16 * SI_QBW * w;
#pragma unroll
  for (int qb = 0; qb < SI_QBW; ++qb) {
    const int qi = qbase + 16 * qb + col;
    const bool v = qi < nq;
    const int8_t* qp = q8 + (int64_t)(v ? qi : 0) * EP + 16 * g;
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[qb][s] = *(const u32x4*)(qp + 64 * s);
    tqv[qb] = v ? tq8[qi] : 0.0f;
  }
  // A-fragment LDS addresses: row 16 rb + col, logical chunk 4 s + g at position (4 s + g) ^ f,
  // f = swz(16 rb + col) = (col >> 1) & 7 for every rb
  const int f = i8_swz<EP>(col);
  uint32_t lrd[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) lrd[s] = lds_addr(ring) + col * EP + 16 * ((4 * s + g) ^ f);
  // the tile keys of chunk c from its accumulators: per query the max over each 32-row tile,
  // scaled by the rows' tile scale (rows 4 g .. 4 g + 3 of row block rb share one: sample row
  // i -> catalog row 16 i) and the query's t; lane (g, col) then writes query 16 g + col's two
  // keys (tiles 2 c, 2 c + 1) as one 16-B store
  const int ntiles = (int)((j1 - j0 + 31) / 32);
  auto emit = [&](const i32x4 (&ac)[SI_RB][SI_QBW], int c) __attribute__((always_inline)) {
    float srb[SI_RB];
#pragma unroll
    for (int rb = 0; rb < SI_RB; ++rb) srb[rb] = ssc[(SI_CH / 4) * c + 4 * rb + g];
    float mq[SI_QBW][SI_NT];
#pragma unroll
    for (int qb = 0; qb < SI_QBW; ++qb)
#pragma unroll
      for (int h = 0; h < SI_NT; ++h) {
        float m = -__builtin_huge_valf();
#pragma unroll
        for (int r2 = 0; r2 < 2; ++r2) {
          const i32x4 v = ac[2 * h + r2][qb];
          const int mi = max(max(v[0], v[1]), max(v[2], v[3]));
          m = fmaxf(m, (float)mi * srb[2 * h + r2]);
        }
        const auto x16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m),
                                                          false, false);
        m = fmaxf(__uint_as_float(x16[0]), __uint_as_float(x16[1]));
        const auto x32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m),
                                                          false, false);
        m = fmaxf(__uint_as_float(x32[0]), __uint_as_float(x32[1])) * tqv[qb];
        mq[qb][h] = m == m ? m : -__builtin_huge_valf();
      }
    float mm[SI_NT];
#pragma unroll
    for (int h = 0; h < SI_NT; ++h) mm[h] = mq[0][h];
#pragma unroll
    for (int qb = 1; qb < SI_QBW; ++qb)
      if (g == qb)
#pragma unroll
        for (int h = 0; h < SI_NT; ++h) mm[h] = mq[qb][h];
    const int qi = qbase + 16 * g + col;
    if (g < SI_QBW && qi < nq) {
#pragma unroll
      for (int h = 0; h < SI_NT; h += 2) {
        const int t = SI_NT * c + h;  // tile within the slab (pairs never cross FL_CAP)
        if (t >= ntiles) break;
        const int64_t r0 = j0 + 32 * (int64_t)t;
        const uint64_t k0 = make_key(mm[h], (uint32_t)(r0 * STRIDE));
        const uint64_t k1 = make_key(mm[h + 1], (uint32_t)((r0 + 32) * STRIDE));
        *(u32x4*)(lists + ((int64_t)qi * n_slabs + slab) * FL_CAP + t) =
            u32x4{(uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)k1, (uint32_t)(k1 >> 32)};
      }
    }
  };
  // chunk c's MFMAs, with chunk c - 1's epilogue (emit) placed after the first k-step: its
  // VALU work issues between the MFMAs instead of after them (all waves of the block move in
  // lockstep between barriers, so no other wave would fill the MFMA pipes meanwhile)
  i32x4 accp[SI_RB][SI_QBW];
  for (int c = 0; c < n_ch; ++c) {
    const int younger = n_ch - 1 - c < SI_PD - 1 ? n_ch - 1 - c : SI_PD - 1;
    if (younger >= 2) wait_vm<2 * PPW>();
    else if (younger == 1) wait_vm<PPW>();
    else wait_vm<0>();
    lds_barrier();  // chunk c landed (every wave's pieces); every wave is done with chunk c - 1
    if (c + SI_PD < n_ch) issue(c + SI_PD);
    const uint32_t so = (uint32_t)((c % SI_SLOTS) * TILE_B);
    i32x4 acc[SI_RB][SI_QBW];
#pragma unroll
    for (int rb = 0; rb < SI_RB; ++rb)
#pragma unroll
      for (int qb = 0; qb < SI_QBW; ++qb) acc[rb][qb] = i32x4{0, 0, 0, 0};
    // k-step S's 4 A fragments are read while step S - 1's 16 MFMAs run (one step ahead; with
    // 8 waves the SIMD's other wave covers the LDS latency and one buffer fits 256 registers)
    constexpr int AB = (SI_NW == 4 && !TT_SI_OCC2) ? 2 : 1;
    u32x4 a[2][SI_RB];
#pragma unroll
    for (int rb = 0; rb < SI_RB; ++rb) a[0][rb] = lds_read128<0>(lrd[0] + so + rb * 16 * EP);
    static_for<KS>([&](auto s_) __attribute__((always_inline)) {
      constexpr int S = decltype(s_)::value;
      if constexpr (AB == 1) {
        if constexpr (S > 0) {
#pragma unroll
          for (int rb = 0; rb < SI_RB; ++rb) a[S & 1][rb] = lds_read128<0>(lrd[S] + so + rb * 16 * EP);
        }
        lds_wait<0>();
      } else if constexpr (S + 1 < KS) {
#pragma unroll
        for (int rb = 0; rb < SI_RB; ++rb)
          a[(S + 1) & 1][rb] = lds_read128<0>(lrd[S + 1] + so + rb * 16 * EP);
        lds_wait<SI_RB>();
      } else {
        lds_wait<0>();
      }
#pragma unroll
      for (int rb = 0; rb < SI_RB; ++rb) {
        reg_tie(a[S & 1][rb]);
#pragma unroll
        for (int qb = 0; qb < SI_QBW; ++qb)
          acc[rb][qb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
              __builtin_bit_cast(i32x4, a[S & 1][rb]), __builtin_bit_cast(i32x4, qf[qb][S]),
              acc[rb][qb], 0, 0, 0);
      }
      if constexpr (S == 0 && TT_SI_PIPE)
        if (c > 0) emit(accp, c - 1);
    });
    if (!TT_SI_PIPE) emit(acc, c);
#pragma unroll
    for (int rb = 0; rb < SI_RB; ++rb)
#pragma unroll
      for (int qb = 0; qb < SI_QBW; ++qb) accp[rb][qb] = acc[rb][qb];
  }
  if (TT_SI_PIPE && n_ch > 0) emit(accp, n_ch - 1);
  wait_vm<0>();
}

// sharded finish: pcount[q][i] = #rows over ALL shards with a >= t_i (all-reduced SUM).
// pcount[q][0] < k: the sample threshold did not certify -> exact fallback on every shard
// (identical decision on all ranks).  Else A_k >= t* = the highest probe with >= k rows, so
// every row of the exact top-k has a >= A_k - eps2 >= t* - eps2 = cut[q] (the band bound of
// the single-shard path with A_k relaxed to t*).
__global__ void k_probe_cut(const int* __restrict__ pcount, const float* __restrict__ stats,
                            const float* __restrict__ eps2, int nq, int k, int* flags, int* qsel,
                            int* qsel_n, float* __restrict__ cut) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  const int* pc = pcount + (int64_t)q * SH_P;
  if (pc[0] < k) {
    if (!flags[q]) flag_query(q, flags, qsel, qsel_n);
    return;
  }
  int i = 0;
  while (i + 1 < SH_P && pc[i + 1] >= k) ++i;
  cut[q] = probe_t(stats[2 * q], stats[2 * q + 1], i) - eps2[q];
}

// --------------------------------------------------------------------------- rerank
// Two-phase re-rank (band_p1 >= 0: k_select_reg stored the band's P1 = {a >= A_k}, k rows plus
// ties, first).  Phase 1 scores P1 exactly; s1 = their smallest exact score is a lower bound of
// the final k-th score s_k (P1 holds >= k rows).  A row of the rest of the band can only enter
// the top k if s >= s_k >= s1, and s <= a + eps, so phase 2 scores only the rows with
// a + eps >= s1 (a + eps < s1 means s < s1 <= s_k: strictly below, ties included).  In practice
// s1 ~ A_k, so phase 2 keeps the rows within ~eps of A_k instead of 2 eps: ~180 -> ~135 exact
// rows per query at 1M x 384 (tools/band_analysis.py), a quarter less HBM gather.
template <int EP>
__global__ __launch_bounds__(256) void k_rerank(const float* __restrict__ db, int64_t ld,
                                                const float* __restrict__ q, int64_t ldq,
                                                const uint64_t* __restrict__ band,
                                                const int* __restrict__ band_n,
                                                const int* __restrict__ band_p1,
                                                const float* __restrict__ eps2,
                                                const float* __restrict__ aref, int* flags,
                                                int* qsel, int* qsel_n, int64_t n_rows, int k,
                                                int64_t row_base, float* __restrict__ out_s,
                                                int64_t* __restrict__ out_i) {
  __shared__ uint64_t buf[BAND_CAP];
  // A decoded candidate row >= n_rows (a corrupted list or band entry) is never read: the row
  // is clamped for the loads and the query goes to the exact fallback instead (bad_row).
  bool bad_row = false;
  __shared__ __attribute__((aligned(16))) float qs[EP];
  __shared__ int nkeep;
  __shared__ unsigned long long kmin;
  const int qid = blockIdx.x;
  if (flags[qid]) return;  // served by the exact fallback
  const int nb = band_n[qid];
  const int p1 = band_p1 != nullptr ? band_p1[qid] : -1;
  const uint64_t* qband = band + (int64_t)qid * BAND_CAP;
  for (int i = threadIdx.x; i < EP; i += blockDim.x) qs[i] = q[(int64_t)qid * ldq + i];
  if (threadIdx.x == 0) {
    nkeep = 0;
    kmin = ~0ull;
  }
  __syncthreads();
  // exact keys of src[0 .. cnt) into dst[0 .. cnt) (dst may alias src element for element)
#if TT_RR_STAGED
  // Each wave takes 64 rows at a time and fetches them 64 dimensions (256 B per row) per
  // chunk: 16 lanes per row, 4 rows per wave-instruction, 16 instructions in flight (the next
  // chunk is loaded while this one is summed).  The chunk goes through a wave-private LDS
  // stage (16-B pieces XOR-swizzled by row: conflict-free writes and reads), and lane j then
  // runs row j's canonical FMA chain over those 64 dimensions -- the same order as below.
  // (Thread-per-row loads put 64 rows into every wave-instruction.)
  __shared__ __attribute__((aligned(16))) char stage[4][64 * 256];
  auto score = [&](const uint64_t* src, uint64_t* dst, int cnt) __attribute__((always_inline)) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    char* st = stage[w];
    const int sub = lane >> 4, piece = lane & 15;
    for (int e0 = 64 * w; e0 < cnt; e0 += 256) {
      const int ej = e0 + lane;
      uint32_t rj = key_row(src[ej < cnt ? ej : e0]);
      if ((int64_t)rj >= n_rows) {
        bad_row = true;
        rj = 0;
      }
      const float* rp[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t r = (uint32_t)__shfl((int)rj, 4 * i + sub, 64);
        rp[i] = db + (int64_t)r * ld + 4 * piece;
      }
      constexpr int NC = EP / 64, PF = TT_RR_PF;  // chunks; chunks loaded ahead
      float acc = 0.0f;
      // stage chunk c from v, refill v with chunk c + PF, run the chain over chunk c
      auto chunk = [&](int c, f32x4 (&v)[16]) __attribute__((always_inline)) {
        asm volatile("" ::: "memory");
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int row = 4 * i + sub;
          *(f32x4*)(st + row * 256 + 16 * (piece ^ (row & 15))) = v[i];
        }
        asm volatile("" ::: "memory");
        if (c + PF < NC) {
#pragma unroll
          for (int i = 0; i < 16; ++i) v[i] = *(const f32x4*)(rp[i] + 64 * (c + PF));
        }
        const char* my = st + lane * 256;
        const int sw = lane & 15;
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          const f32x4 x0 = *(const f32x4*)(my + 16 * ((4 * tt + 0) ^ sw));
          const f32x4 x1 = *(const f32x4*)(my + 16 * ((4 * tt + 1) ^ sw));
          const f32x4 x2 = *(const f32x4*)(my + 16 * ((4 * tt + 2) ^ sw));
          const f32x4 x3 = *(const f32x4*)(my + 16 * ((4 * tt + 3) ^ sw));
          const float* qt = qs + 64 * c + 16 * tt;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            acc = fmaf(x0[i], qt[0 + i], acc);
            acc = fmaf(x1[i], qt[4 + i], acc);
            acc = fmaf(x2[i], qt[8 + i], acc);
            acc = fmaf(x3[i], qt[12 + i], acc);
          }
        }
      };
      f32x4 v0[16], v1[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v0[i] = *(const f32x4*)rp[i];
      if (PF == 2 && NC > 1) {
#pragma unroll
        for (int i = 0; i < 16; ++i) v1[i] = *(const f32x4*)(rp[i] + 64);
      }
      if constexpr (PF == 1) {
#pragma unroll 1
        for (int c = 0; c < NC; ++c) chunk(c, v0);
      } else {
#pragma unroll 1
        for (int c = 0; c < NC; c += 2) {
          chunk(c, v0);
          if (c + 1 < NC) chunk(c + 1, v1);
        }
      }
      asm volatile("" ::: "memory");
      if (ej < cnt) dst[ej] = acc != acc ? 0ull : make_key(acc, rj);
    }
  };
#else
  auto score = [&](const uint64_t* src, uint64_t* dst, int cnt) __attribute__((always_inline)) {
    for (int e = threadIdx.x; e < cnt; e += blockDim.x) {
      uint32_t r = key_row(src[e]);
      if ((int64_t)r >= n_rows) {
        bad_row = true;
        r = 0;
      }
      const f32x4* xr = (const f32x4*)(db + (int64_t)r * ld);
      float acc = 0.0f;
#pragma unroll 4
      for (int t = 0; t < EP / 16; ++t) {
        const f32x4 x0 = xr[4 * t + 0], x1 = xr[4 * t + 1], x2 = xr[4 * t + 2], x3 = xr[4 * t + 3];
        const float* qt = qs + 16 * t;
        // canonical order: for i: for g: d = 16t + 4g + i
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc = fmaf(x0[i], qt[0 + i], acc);
          acc = fmaf(x1[i], qt[4 + i], acc);
          acc = fmaf(x2[i], qt[8 + i], acc);
          acc = fmaf(x3[i], qt[12 + i], acc);
        }
      }
      dst[e] = acc != acc ? 0ull : make_key(acc, r);
    }
  };
#endif
  int nsc = nb;  // rows scored into buf[0 .. nsc)
  if (p1 >= 0 && p1 <= nb && !TT_RR_ONEPHASE) {
    score(qband, buf, p1);  // phase 1: P1
    __syncthreads();
    // s1 = the smallest exact P1 key (a NaN score keys 0: then s1 = -inf, all rows stay)
    unsigned long long m = ~0ull;
    for (int i = threadIdx.x; i < p1; i += blockDim.x) m = min(m, (unsigned long long)buf[i]);
    for (int o = 32; o > 0; o >>= 1) m = min(m, (unsigned long long)__shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) atomicMin(&kmin, m);
    __syncthreads();
    const float s1 = kmin == 0ull || kmin == ~0ull ? -__builtin_huge_valf() : key_score(kmin);
    const float eps = 0.5f * eps2[qid];  // eps2 = 2 eps (x1.001)
    // phase 2: the rest of the band, rows with a + eps >= s1, compacted after P1
    for (int e = p1 + threadIdx.x; e < nb; e += blockDim.x) {
      const uint64_t key = qband[e];
      if (key_float((uint32_t)(key >> 32)) + eps >= s1) buf[p1 + atomicAdd(&nkeep, 1)] = key;
    }
    __syncthreads();
    nsc = p1 + nkeep;
    score(buf + p1, buf + p1, nsc - p1);
  } else {
    score(qband, buf, nb);
  }
  if (__syncthreads_or(bad_row)) {
    if (threadIdx.x == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  const int np = pow2_at_least(nsc);
  for (int i = nsc + threadIdx.x; i < np; i += blockDim.x) buf[i] = 0ull;
  block_sort_desc(buf, np);
  // certification of the full level's threshold (full_theta): the k-th exact score of the
  // scored rows is a lower bound of the query's s_k; below full_cert(aref) the level may have
  // dropped a band row -> exact fallback (a NaN exact score in the top k: also the fallback)
  if (aref != nullptr) {
    const bool ok = nsc >= k && buf[k - 1] != 0ull &&
                    key_score(buf[k - 1]) >= full_cert(aref[qid], eps2[qid]);
    if (!ok) {
      if (threadIdx.x == 0) flag_query(qid, flags, qsel, qsel_n);
      return;
    }
  }
  for (int i = threadIdx.x; i < k; i += blockDim.x) {
    float s = -__builtin_huge_valf();
    int64_t ix = -1;
    if (i < nsc && buf[i] != 0ull) {
      s = key_score(buf[i]);
      ix = row_base + (int64_t)key_row(buf[i]);
    }
    out_s[(int64_t)qid * k + i] = s;
    out_i[(int64_t)qid * k + i] = ix;
  }
}

// Sharded finish: a shard's part of a query's band is small (~1/W of it: ~25 rows at W = 8),
// and the block-per-query k_rerank (74 KB LDS: 2 blocks, i.e. 2 queries, per CU; a block-wide
// bitonic sort) spent 1.7 ms on 80k such queries.  Here one WAVE owns a query: the cut filter
// compacts the kept band rows by ballot into a wave-private list of RW_CAP keys, the rows are
// scored by the staged 64-row gather of k_rerank (same canonical FMA order, bit-identical),
// and each kept row's output slot is its rank (#keys ahead) -- no sort, no block barrier.  A
// shard whose part of the band outgrows the list (W = 2: ~8% of iid queries kept > 256 rows
// and used to take the shard's exact f32 fallback, 1642 of 20k queries per step) scores what
// it holds and keeps only its top k (rank < k: a row of the query's top k has fewer than k
// keys ahead of it in any subset), then goes on appending.
constexpr int RW_CAP = 256;
static_assert(RW_CAP - 64 >= FL_KMAX, "a reduced list leaves room for a 64-key chunk");
template <int EP>
__global__ __launch_bounds__(256) void k_rerank_wave(
    const float* __restrict__ db, int64_t ld, const float* __restrict__ q, int64_t ldq,
    const uint64_t* __restrict__ band, const int* __restrict__ band_n, int* flags, int* qsel,
    int* qsel_n, int nq, int64_t n_rows, int k, int64_t row_base, const float* __restrict__ cut,
    float* __restrict__ out_s, int64_t* __restrict__ out_i) {
  __shared__ __attribute__((aligned(16))) char stage[4][64 * 256];
  __shared__ uint64_t kept[4][RW_CAP];
  __shared__ __attribute__((aligned(16))) float qsh[4][EP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int qid = blockIdx.x * 4 + w;
  if (qid >= nq || flags[qid]) return;  // (flagged: served by the exact fallback)
  float* qs = qsh[w];
  uint64_t* buf = kept[w];
  char* st = stage[w];
  for (int i = lane; i < EP; i += 64) qs[i] = q[(int64_t)qid * ldq + i];
  const int nb_all = band_n[qid];
  const uint64_t* qband = band + (int64_t)qid * BAND_CAP;
  const float c = cut[qid];
  const int sub = lane >> 4, piece = lane & 15;
  int nb = 0, ns = 0;  // kept keys buf[0, nb); buf[0, ns) already hold exact-score keys
  bool bad_row = false;  // a decoded row >= n_rows is never read: exact fallback instead
  // exact keys for buf[from, nb) (band keys -> (canonical f32 score, row) keys, in place)
  auto score_from = [&](int from) __attribute__((always_inline)) {
    wave_sync();
    for (int e0 = from; e0 < nb; e0 += 64) {
      const int ej = e0 + lane;
      uint32_t rj = key_row(buf[ej < nb ? ej : e0]);
      if ((int64_t)rj >= n_rows) {
        bad_row = true;
        rj = 0;
      }
      const float* rp[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t r = (uint32_t)__shfl((int)rj, 4 * i + sub, 64);
        rp[i] = db + (int64_t)r * ld + 4 * piece;
      }
      constexpr int NC = EP / 64;
      float acc = 0.0f;
      f32x4 v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = *(const f32x4*)rp[i];
#pragma unroll 1
      for (int cc = 0; cc < NC; ++cc) {
        asm volatile("" ::: "memory");
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int row = 4 * i + sub;
          *(f32x4*)(st + row * 256 + 16 * (piece ^ (row & 15))) = v[i];
        }
        asm volatile("" ::: "memory");
        if (cc + 1 < NC) {
#pragma unroll
          for (int i = 0; i < 16; ++i) v[i] = *(const f32x4*)(rp[i] + 64 * (cc + 1));
        }
        const char* my = st + lane * 256;
        const int sw = lane & 15;
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          const f32x4 x0 = *(const f32x4*)(my + 16 * ((4 * tt + 0) ^ sw));
          const f32x4 x1 = *(const f32x4*)(my + 16 * ((4 * tt + 1) ^ sw));
          const f32x4 x2 = *(const f32x4*)(my + 16 * ((4 * tt + 2) ^ sw));
          const f32x4 x3 = *(const f32x4*)(my + 16 * ((4 * tt + 3) ^ sw));
          const float* qt = qs + 64 * cc + 16 * tt;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            acc = fmaf(x0[i], qt[0 + i], acc);
            acc = fmaf(x1[i], qt[4 + i], acc);
            acc = fmaf(x2[i], qt[8 + i], acc);
            acc = fmaf(x3[i], qt[12 + i], acc);
          }
        }
        wave_sync();  // every lane's chain read this chunk before the next one is staged
      }
      // the key can replace the band key in place: lane ej owns slot ej (read above)
      if (ej < nb) buf[ej] = acc != acc ? 0ull : make_key(acc, rj);
    }
    ns = nb;
    wave_sync();
  };
  // rank of key me at position e among buf[0, nb) (keys of distinct rows are distinct; equal
  // keys -- NaN scores, key 0 -- are ordered by position)
  auto rank_of = [&](uint64_t me, int e) __attribute__((always_inline)) {
    int rank = 0;
    for (int j = 0; j < nb; ++j) {
      const uint64_t o = buf[j];
      rank += (o > me || (o == me && j < e)) ? 1 : 0;
    }
    return rank;
  };
  for (int e0 = 0; e0 < nb_all; e0 += 64) {
    if (nb > RW_CAP - 64) {  // rare: keep the top k of the list (all scored) and go on
      score_from(ns);
      uint64_t mine[RW_CAP / 64];
      int rk[RW_CAP / 64];
#pragma unroll
      for (int cc = 0; cc < RW_CAP / 64; ++cc) {
        const int e = 64 * cc + lane;
        mine[cc] = e < nb ? buf[e] : 0ull;
        rk[cc] = e < nb ? rank_of(mine[cc], e) : RW_CAP;
      }
      wave_sync();
#pragma unroll
      for (int cc = 0; cc < RW_CAP / 64; ++cc)
        if (rk[cc] < k) buf[rk[cc]] = mine[cc];
      nb = ns = nb < k ? nb : k;
      wave_sync();
    }
    const int e = e0 + lane;
    const uint64_t key = e < nb_all ? qband[e] : 0ull;
    const bool keep = e < nb_all && key_float((uint32_t)(key >> 32)) >= c;
    const uint64_t bm = __ballot(keep);
    const int pos = nb + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
    if (keep) buf[pos] = key;
    nb += (int)__popcll(bm);
  }
  score_from(ns);
  if (__ballot(bad_row) != 0ull) {
    if (lane == 0) flag_query(qid, flags, qsel, qsel_n);
    return;
  }
  // output slot = rank; slots nb .. k-1 stay (-inf, -1)
  for (int e0 = 0; e0 < nb; e0 += 64) {
    const int e = e0 + lane;
    if (e < nb) {
      const uint64_t me = buf[e];
      const int rank = rank_of(me, e);
      if (rank < k) {
        out_s[(int64_t)qid * k + rank] = me ? key_score(me) : -__builtin_huge_valf();
        out_i[(int64_t)qid * k + rank] = me ? row_base + (int64_t)key_row(me) : -1;
      }
    }
  }
  for (int i = nb + lane; i < k; i += 64) {
    out_s[(int64_t)qid * k + i] = -__builtin_huge_valf();
    out_i[(int64_t)qid * k + i] = -1;
  }
}

__global__ void k_fill_i32(int* x, int n, int v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = v;
}
__global__ void k_fill_f32(float* x, int n, float v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = v;
}

// Per-query error bound eps2[q] = 2 eps_q (see the header).  One wave per query.
template <int EP>
__global__ __launch_bounds__(256) void k_query_eps(const float* __restrict__ q, int nq,
                                                   int64_t ldq, float X, float R,
                                                   float* __restrict__ eps2,
                                                   float* __restrict__ theta,
                                                   float* __restrict__ aref,
                                                   int* __restrict__ flags,
                                                   int* __restrict__ qsel_n,
                                                   uint16_t* __restrict__ q16,
                                                   int8_t* __restrict__ q8 = nullptr,
                                                   float* __restrict__ tq8 = nullptr) {
  const int qi = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (qi >= nq) return;
  if (q8) {  // the int8 sample level's coded query t m (k_sample_i8): t = max|q| / 127
    const float* qr = q + (int64_t)qi * ldq;
    float mx = 0.0f;
    for (int i = lane; i < EP; i += 64) mx = fmaxf(mx, fabsf(qr[i]));
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    const float t = mx / 127.0f;
    for (int i = lane; i < EP; i += 64) {
      int c = 0;
      if (t > 0.0f) {
        c = (int)rintf(qr[i] / t);
        c = c > 127 ? 127 : c < -127 ? -127 : c;
      }
      q8[(int64_t)qi * EP + i] = (int8_t)c;
    }
    if (lane == 0) tq8[qi] = t;
  }
  if (q16) {  // the bf16 image the ring levels load (the conversion k_filter_ring's f32 path does)
    const float* qr = q + (int64_t)qi * ldq;
    for (int c = lane; c < EP / 8; c += 64) {
      const f32x4 v0 = *(const f32x4*)(qr + 8 * c), v1 = *(const f32x4*)(qr + 8 * c + 4);
      *(u32x4*)(q16 + (int64_t)qi * EP + 8 * c) =
          u32x4{pack_bf16x2(v0[0], v0[1]), pack_bf16x2(v0[2], v0[3]), pack_bf16x2(v1[0], v1[1]),
                pack_bf16x2(v1[2], v1[3])};
    }
  }
  if (lane == 0) {  // filter state of query qi
    theta[qi] = -__builtin_huge_valf();
    aref[qi] = -__builtin_huge_valf();
    flags[qi] = 0;
    qsel_n[1 + qi] = 0;  // done[qi] (FilterWs layout)
    if (qi == 0) *qsel_n = 0;
  }
  const float e = query_eps2_wave<EP>(q + (int64_t)qi * ldq, X, R, lane);
  if (lane == 0) eps2[qi] = e;
}

__global__ void k_sub_arr(float* x, const float* y, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = x[i] - y[i];
}

// --------------------------------------------------------------------------- host
struct Level {
  int64_t stride, n_sample;
  int rows_per_slab, n_slabs, n_qt;
  int n_slabs_p = 0, rows_p = 0;  // balanced plan of a partial last query tile (plan_balance)
  bool dense;
  bool tmax;  // appends tile maxima (k_filter_ring<EP, 0>): every level sampled at stride > 1
};

struct FilterPlan {
  int n_levels, max_slabs, J;
  bool small;  // block-per-query selection path (k_select_small / k_final_small)
  bool topm;   // single-pass path (k_filter_topm + k_final_topm), nq <= TM_NQ
  Level lv[8];
};

// Levels over nested strided samples (stride 16^i, coarsest first).  The coarsest has
// <= SEL_CAP/2 rows and is scored densely (every row a candidate); the others stream through
// the ring kernel.  J = rows of a sample level's top list that feed the next threshold: the
// full catalog has ~16*J rows above a_J(stride-16 sample), comfortably >= k.
static bool select_reg_disabled() {  // TT_SELECT_REG=0: LDS-staged k_select_wave (timing builds)
  static const bool off = env_switch("TT_SELECT_REG", 1) == 0;
  return off;
}
// Small batches too take the k_query_eps launch (bf16 query image + per-query state) instead of
// folding the state into the first ring level: that fold's f32 query loads went out one k-step
// at a time (the bf16 conversion's NaN branch splits every step, and a hoisted f32 conversion
// does not fit the ring kernels' registers) -- ~15 us before the first tile of EVERY ring
// launch of the search, sample and full level alike (tools/blktime_small.py).
#ifndef TT_Q16_SMALL
#define TT_Q16_SMALL 1
#endif
TT_CHECK_EXP(TT_Q16_SMALL != 1, "TT_Q16_SMALL");
static bool q16_enabled() {  // TT_FILTER_Q16=0: ring levels load f32 queries (timing builds)
  static const bool on = env_switch("TT_FILTER_Q16", 1) != 0;
  return on;
}
static bool topm_disabled() {  // TT_FILTER_TOPM=0: the multi-level small path (timing builds)
  static const bool off = env_switch("TT_FILTER_TOPM", 1) == 0;
  return off;
}
static bool tmax_first_disabled() {  // TT_FILTER_TMAX_FIRST=0: full sample ladder (timing builds)
  static const bool off = env_switch("TT_FILTER_TMAX_FIRST", 1) == 0;
  return off;
}
constexpr int64_t SW_CAP_TILES = SW_CAP - 64;  // first-level tiles per query, with margin
#ifndef TT_SAMPLE_J_ADD
// J = ceil(k / 8) + TT_SAMPLE_J_ADD (plan_filter).  A query falls back when the stride-16
// sample holds >= J of the catalog's top 99 (then a_J(sample) > A_k): at k = 100 that is
// P(Bin(99, 1/16) >= J) = 1.1e-5 per query at J = 19, 7.1e-7 at 21, 1.5e-9 at 25, i.e.
// 0.11 / 0.007 / 0.00001 fallbacks per 10k-query step.  A/B x3 on one box (tools/
// bench_ab.sh): full level 5.48 / 5.53 / 5.57 ms, step 6.65 / 6.70 / 6.75 ms, 0 fallbacks;
// J = 21 (a fallback costs ~0.47 ms, tt_scan.hip adaptive fallback; 1.4 ms in round 2).
#define TT_SAMPLE_J_ADD 8
#endif
TT_CHECK_EXP(TT_SAMPLE_J_ADD != 8, "TT_SAMPLE_J_ADD");
static int64_t ring_tr(int ep) {                 // rows per k_filter_ring tile
  return ep == 64 ? RingCfg<64>::TR : ep == 128 ? RingCfg<128>::TR : ep == 256 ? RingCfg<256>::TR
         : ep == 384 ? RingCfg<384>::TR : ep == 512 ? RingCfg<512>::TR : RingCfg<768>::TR;
}
static int device_cus() {
  static const int cus = [] {
    int d = 0, v = 0;
    if (hipGetDevice(&d) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && v > 0)
      return v;
    return 256;  // MI355X
  }();
  return cus;
}

// Slab count of a ring level: the kernel runs one 512-thread block per CU (148 KB LDS), so
// the n_qt * slabs blocks execute in ceil(blocks / CUs) equal rounds.  Minimise
// rounds * (rows per slab + per-slab overhead ~ 3 tiles), slabs >= 1 tile-row chunk of 256
// rows, slabs <= 64 (list memory and k_select work grow with the slab count) -- except for
// small query batches (n_qt * 64 < 4 CUs' worth of blocks, e.g. the one-buyer /retrieve
// call): there up to 4 blocks per CU, so the catalog pass uses the whole chip instead of 64
// CUs (the selection then takes the multi-pass k_select_wave).
static int64_t ring_slabs(int n_qt, int64_t n_sample, int64_t sl_min = 1) {
  const int ncu = device_cus() * RG_BLOCKS_PER_CU;  // concurrent blocks
  // slabs of >= 128 rows (4 tiles); was 256, which capped the one-buyer stride-16 level
  // (62.5k rows) at 244 slabs, whose 64-row rounding then left 196 blocks on 256 CUs
  int64_t sl_max = n_sample / 128;
  const int64_t cap = (int64_t)n_qt * 64 >= 4 * ncu ? 64 : (4 * ncu + n_qt - 1) / n_qt;
  if (sl_max > cap) sl_max = cap;
  if (sl_max < sl_min) sl_max = sl_min;
  if (sl_max < 1) sl_max = 1;
  int64_t best = sl_min < 1 ? 1 : sl_min;
  double best_cost = 1e300;
  for (int64_t sl = best; sl <= sl_max; ++sl) {
    const int64_t rounds = ((int64_t)n_qt * sl + ncu - 1) / ncu;
    const int64_t rows = ((n_sample + sl - 1) / sl + 63) / 64 * 64;
    const double cost = (double)rounds * (double)(rows + 96);
    if (cost < best_cost * 0.999) {
      best_cost = cost;
      best = sl;
    }
  }
  return best;
}

// Balanced plan of the batched full level when its last query tile is partial (10k queries =
// 26 tiles of 384 + 16): a block of that tile streams its slab with ~1 of 8 waves computing and
// costs ~0.53 of a full block per row (round-5 block timeline, tools/blktime.py: 620 vs 1160
// us), so with uniform slabs the launch's CUs ran 4 or 5 full blocks plus or minus a cheap one
// -- 4.5% of the launch's CU time idle, most of it a ragged tail.  Here the full tiles take
// s_f slabs and the partial tile s_p ~ c_p s_f coarser ones, with (n_qt - 1) s_f + s_p = whole
// rounds of the chip, so every CU runs the same number of blocks of about the same cost.
// Taken when its rounds x (rows + 96) model beats the uniform plan's.
#ifndef TT_FILTER_BALANCE_DEFAULT
#define TT_FILTER_BALANCE_DEFAULT 1  // 0: uniform slabs unless TT_FILTER_BALANCE=1 (A/B builds)
#endif
TT_CHECK_EXP(TT_FILTER_BALANCE_DEFAULT != 1, "TT_FILTER_BALANCE_DEFAULT");
static bool balance_disabled() {  // TT_FILTER_BALANCE=0: uniform slabs
  static const bool off = env_switch("TT_FILTER_BALANCE", TT_FILTER_BALANCE_DEFAULT) == 0;
  return off;
}
static void plan_balance(Level& L, int nq, int qpb) {
  if (balance_disabled() || L.n_qt < 2) return;
  const int ncu = device_cus() * RG_BLOCKS_PER_CU;
  const double f = (double)(nq - (L.n_qt - 1) * qpb) / qpb;  // partial tile's share of queries
  const double cp = 0.5 + 0.5 * f;                              // its cost per row, vs a full tile
  if (f >= 1.0) return;
  const int64_t rounds_u = ((int64_t)L.n_qt * L.n_slabs + ncu - 1) / ncu;
  const double cost_u = (double)rounds_u * (L.rows_per_slab + 96);
  double best = cost_u;
  int bf = 0, bp = 0, rf_best = 0, rp_best = 0;
  for (int64_t R = 1; R <= 64; ++R) {
    const int64_t blocks = R * ncu;
    int64_t sf = (int64_t)((double)blocks / (L.n_qt - 1 + cp));
    for (; sf >= 1; --sf) {
      int64_t rf = ((L.n_sample + sf - 1) / sf + 63) / 64 * 64;
      const int64_t sf2 = (L.n_sample + rf - 1) / rf;
      const int64_t sp = blocks - (int64_t)(L.n_qt - 1) * sf2;
      if (sp < 16 || sp > sf2) continue;
      const int64_t rp = ((L.n_sample + sp - 1) / sp + 63) / 64 * 64;
      const int64_t sp2 = (L.n_sample + rp - 1) / rp;
      if (sp2 < 16 || rp >= (1 << 25) || rf >= (1 << 25)) continue;
      const double cost = (double)R * ((rf > cp * rp ? rf : cp * rp) + 96);
      if (cost < best * 0.999) {
        best = cost;
        bf = (int)sf2;
        bp = (int)sp2;
        rf_best = (int)rf;
        rp_best = (int)rp;
      }
      break;
    }
    if (R * ncu > 4 * (int64_t)L.n_qt * L.n_slabs) break;
  }
  if (bf > 0) {
    L.n_slabs = bf;
    L.rows_per_slab = rf_best;
    L.n_slabs_p = bp;
    L.rows_p = rp_best;
  }
}

static FilterPlan plan_filter_uncached(int64_t n, int nq, int k, int ep) {
  FilterPlan p;
  // ~16*J full-catalog rows lie above a_J(stride-16 sample); J = k/8 + 8 keeps that count
  // >= k except with probability P(Bin(k - 1, 1/16) >= J) (7e-7 at k = 100; TT_SAMPLE_J_ADD)
  p.J = (k + 7) / 8 + TT_SAMPLE_J_ADD;
  if (p.J > k) p.J = k;
  int64_t strides[8];
  int nl = 0;
  int64_t s = 1;
  while ((n + s - 1) / s > SEL_CAP / 2 && nl < 7) {
    strides[nl++] = s;
    s *= 16;
  }
  strides[nl++] = s;
  // Tile-max shortcut: a sample level appends one key per (query, 32-row tile), so a sample
  // whose tiles fit one query's selection buffer can be the FIRST level, at theta = -inf
  // (every tile max a candidate) -- the coarser levels and their selections (4 launches,
  // ~0.1 ms at 1M rows) are dropped.  Take the finest such sample; never the last level
  // (that one appends rows, not tile maxima).  TT_FILTER_TMAX_FIRST=0 restores the ladder.
  int first = -1;
  const int64_t TMAX_TR = ring_tr(ep);
  if (!tmax_first_disabled())
    for (int i = 1; i < nl && first < 0; ++i) {
      const int64_t ns = (n + strides[i] - 1) / strides[i];
      if (ns > SEL_CAP / 2 && (ns + TMAX_TR - 1) / TMAX_TR <= SW_CAP_TILES) first = i;
    }
  if (first > 0) nl = first + 1;
  p.n_levels = nl;
  p.max_slabs = 1;
  const int dense_qpb = FL_WAVES * 16 * (ep <= 384 ? 2 : 1);
  // queries per block of the ring instantiation a level will run (launch_level's rule)
  auto ring_qpb_v = [&](bool tmax) { return ring_qpb_rt(ep, ring_lvl(tmax, nq, ep)); };
  for (int i = 0; i < nl; ++i) {
    Level& L = p.lv[i];
    L.stride = strides[nl - 1 - i];
    L.n_sample = (n + L.stride - 1) / L.stride;
    L.dense = i == 0 && first < 0;
    L.tmax = L.stride != 1;
    const int qpb = L.dense ? dense_qpb : ring_qpb_v(L.stride != 1);
    L.n_qt = (nq + qpb - 1) / qpb;
    int64_t sl;
    if (L.dense) {
      sl = (L.n_sample + FL_CAP / 2 - 1) / (FL_CAP / 2);  // every row is a candidate
    } else if (i == 0) {
      // theta = -inf: every tile of a slab lands in its (query, slab) list of FL_CAP
      sl = ring_slabs(L.n_qt, L.n_sample, (L.n_sample + FL_CAP * TMAX_TR - 1) / (FL_CAP * TMAX_TR));
    } else {
      sl = ring_slabs(L.n_qt, L.n_sample);
    }
    if (sl < 1) sl = 1;
    // k_filter_ring's pool entries hold a row offset within the slab in 32 - QSH bits (QSH <= 7)
    if (!L.dense && sl < ((L.n_sample + (1 << 25) - 1) >> 25)) sl = (L.n_sample + (1 << 25) - 1) >> 25;
    int64_t r = (L.n_sample + sl - 1) / sl;
    r = (r + 63) / 64 * 64;
    L.rows_per_slab = (int)r;
    L.n_slabs = (int)((L.n_sample + r - 1) / r);
    if (i == nl - 1 && !L.dense && ring_lvl(false, nq, ep) == 1) plan_balance(L, nq, qpb);
    if (L.n_slabs > p.max_slabs) p.max_slabs = L.n_slabs;
  }
  p.small = nq <= SM_NQ && !select_reg_disabled();
  for (int i = 0; i < nl; ++i) p.small = p.small && p.lv[i].n_slabs <= SM_THREADS;
  // single pass for the smallest batches: lists [nq][G][TM_M] and counts [nq][G] fit the
  // level workspace once max_slabs >= G (FL_CAP >= TM_M)
  // (the bf16 single pass runs for nq <= TM_NQ_RUN; the int8 ones up to TM_NQ_I8 (ring) and
  // TM_NQ_I8T (tiled image))
  p.topm = nq <= TM_NQ_I8T && !topm_disabled() && device_cus() * TM_M <= TM_CAP &&
           device_cus() <= SM_THREADS;
  if (p.topm && p.max_slabs < device_cus()) p.max_slabs = device_cus();
  return p;
}

// plan_filter_uncached's slab searches cost ~9 us of host time per one-buyer call (two
// ring_slabs scans of up to 1024 candidates) -- ahead of the first launch, so on the
// synchronised /retrieve path they are latency.  Plans depend only on (n, nq, k, ep) and
// process-constant switches, so the last few are kept per thread.
static FilterPlan plan_filter(int64_t n, int nq, int k, int ep) {
  struct Entry {
    int64_t n;
    int nq, k, ep;
    FilterPlan p;
  };
  constexpr int NC = 8;
  thread_local Entry cache[NC];
  thread_local int used = 0, next = 0;
  for (int i = 0; i < used; ++i)
    if (cache[i].n == n && cache[i].nq == nq && cache[i].k == k && cache[i].ep == ep)
      return cache[i].p;
  Entry& e = cache[next];
  e.n = n, e.nq = nq, e.k = k, e.ep = ep;
  e.p = plan_filter_uncached(n, nq, k, ep);
  next = (next + 1) % NC;
  if (used < NC) ++used;
  return e.p;
}

struct FilterWs {
  uint64_t* lists;
  int* counts;
  float* theta;
  float* aref;
  float* eps2;
  float* cut;
  uint64_t* band;
  int* band_n;
  int* band_p1;  // rows of the band with a >= A_k, stored first (k_select_reg); -1: unordered
  int* flags;  // flags[nq], qsel[nq], qsel_n[1], done[nq] are contiguous: the per-query
  int* qsel;   // init zeroes flags[qi] and qsel_n[1 + qi] (= done[qi], the fused fallback
  int* qsel_n; // merge's per-tile arrival counter)
  int* done;
  void* scan_ws;
  int64_t scan_ws_bytes;
  uint16_t* q16;     // [nq][ep] bf16 query image (k_query_eps), for the ring levels
  bool q16_valid;    // written by this search's k_query_eps
  int8_t* q8;        // [nq][ep] int8-coded queries + tq8[nq] (k_query_eps), for k_sample_i8
  float* tq8;
  int64_t total;
};

static int64_t align256(int64_t b) { return (b + 255) / 256 * 256; }

static FilterWs carve(void* base, const FilterPlan& p, int64_t n, int d, int nq, int k) {
  FilterWs w;
  // base == nullptr: size / offset query -> pointers are offsets from a fake 4 KiB base
  char* c = base ? (char*)base : (char*)4096;
  int64_t off = 0;
  auto take = [&](int64_t bytes) {
    char* r = c + off;
    off += align256(bytes);
    return r;
  };
  w.lists = (uint64_t*)take((int64_t)nq * p.max_slabs * FL_CAP * 8);
  w.counts = (int*)take((int64_t)nq * p.max_slabs * 4);
  w.theta = (float*)take((int64_t)nq * 4);
  w.aref = (float*)take((int64_t)nq * 4);
  w.eps2 = (float*)take((int64_t)nq * 4);
  w.cut = (float*)take((int64_t)nq * 4);
  w.band = (uint64_t*)take((int64_t)nq * BAND_CAP * 8);
  w.band_n = (int*)take((int64_t)nq * 4);
  w.band_p1 = (int*)take((int64_t)nq * 4);
  int* fl = (int*)take(((int64_t)3 * nq + 1) * 4);
  w.flags = fl;
  w.qsel = fl + nq;
  w.qsel_n = fl + 2 * nq;
  w.done = w.qsel_n + 1;
  int64_t sb = 0;
  tt_scan_workspace_bytes(n, d, nq, k, &sb);
  w.scan_ws_bytes = sb;
  w.scan_ws = take(sb);
  w.q16 = (uint16_t*)take((int64_t)nq * tt_padded_dim(d) * 2);
  w.q16_valid = false;
  w.q8 = (int8_t*)take((int64_t)nq * tt_padded_dim(d));
  w.tq8 = (float*)take((int64_t)nq * 4);
  w.total = off;
  return w;
}

template <int EP>
static void launch_level(const Level& L, const uint16_t* xb, int64_t n, int64_t ld,
                         const float* q, int nq, int64_t ldq, const FilterWs& w,
                         hipStream_t st, const QueryInit& qi) {
  const int nblk = L.n_qt * L.n_slabs;
  if (L.dense) {
    constexpr int QB = EP <= 384 ? 2 : 1;
    hipLaunchKernelGGL((k_filter_dense<EP, QB>), dim3(nblk), dim3(64 * FL_WAVES), 0, st, xb, n,
                       ld, q, nq, ldq, w.theta, L.stride, L.n_sample, L.rows_per_slab,
                       L.n_slabs, L.n_qt, w.lists, w.counts);
  } else {
    const int lvl = ring_lvl(L.tmax, nq, EP);
    auto kern = lvl == 3 ? k_filter_ring<EP, 3> : lvl == 0 ? k_filter_ring<EP, 0>
                : lvl == 1 ? k_filter_ring<EP, 1> : k_filter_ring<EP, 2>;
    if constexpr (EP >= 512)
      if (lvl == 4) kern = k_filter_ring<EP, 4>;
    const int nb = L.n_slabs_p > 0 ? (L.n_qt - 1) * L.n_slabs + L.n_slabs_p : nblk;
    hipLaunchKernelGGL(kern, dim3(nb), dim3(64 * RG_WAVES), 0, st, xb, ld, q, nq, ldq, w.theta,
                       L.stride, L.n_sample, L.rows_per_slab, L.n_slabs, L.n_qt, w.lists,
                       w.counts, qi, w.q16_valid ? (const uint16_t*)w.q16 : nullptr,
                       L.n_slabs_p, L.rows_p);
  }
}

}  // namespace tt

using namespace tt;

// implemented in tt_scan.hip: exact f32 scan restricted to a device-side query list, the slab
// merge fused into the same launch
namespace tt {
int scan_f32_select_fused(const float* db, int64_t n, int32_t d, int64_t ld_db, int64_t row_base,
                          const float* q, int32_t nq, int64_t ld_q, int32_t k,
                          const int32_t* qsel, const int32_t* qsel_n, int* done,
                          float* out_score, int64_t* out_idx, void* workspace,
                          int64_t workspace_bytes, void* stream);
}

extern "C" int tt_filter_workspace_bytes(int64_t n, int32_t d, int32_t nq, int32_t k,
                                         int64_t* bytes) {
  TT_REQUIRE(bytes != nullptr, "bytes == NULL");
  TT_REQUIRE(n >= 1 && nq >= 1 && k >= 1, "n, nq, k must be >= 1");
  const int ep = tt_padded_dim(d);
  TT_REQUIRE(ep > 0, "d > 768");
  const FilterPlan p = plan_filter(n, nq, k, ep);
  *bytes = carve(nullptr, p, n, d, nq, k).total;
  return TT_OK;
}

extern "C" int tt_filter_fallback_offset(int64_t n, int32_t d, int32_t nq, int32_t k,
                                         int64_t* offset) {
  TT_REQUIRE(offset != nullptr && n >= 1 && nq >= 1 && k >= 1, "bad arguments");
  const int ep = tt_padded_dim(d);
  TT_REQUIRE(ep > 0, "d > 768");
  const FilterPlan p = plan_filter(n, nq, k, ep);
  const FilterWs w = carve(nullptr, p, n, d, nq, k);
  *offset = (int64_t)((char*)w.qsel_n - (char*)4096);
  return TT_OK;
}

// Diagnostic layout of a filter workspace (tests): byte offsets of the band keys
// [nq][BAND_CAP] u64, band counts [nq] i32, flags [nq] i32, the fallback count i32, and
// offsets[4] = BAND_CAP.  sharded != 0: the tt_sharded_filter_full/_finish workspace.
extern "C" int tt_filter_workspace_layout(int64_t n, int32_t d, int32_t nq, int32_t k,
                                          int32_t sharded, int64_t* offsets) {
  TT_REQUIRE(offsets != nullptr && n >= 1 && nq >= 1 && k >= 1, "bad arguments");
  const int ep = tt_padded_dim(d);
  TT_REQUIRE(ep > 0, "d > 768");
  FilterPlan p = plan_filter(n, nq, k, ep);
  if (sharded) {
    const Level last = p.lv[p.n_levels - 1];
    p.n_levels = 1;
    p.lv[0] = last;
    p.max_slabs = last.n_slabs;
  }
  const FilterWs w = carve(nullptr, p, n, d, nq, k);
  char* b = (char*)4096;
  offsets[0] = (int64_t)((char*)w.band - b);
  offsets[1] = (int64_t)((char*)w.band_n - b);
  offsets[2] = (int64_t)((char*)w.flags - b);
  offsets[3] = (int64_t)((char*)w.qsel_n - b);
  offsets[4] = BAND_CAP;
  return TT_OK;
}

namespace {
// the full level of a shard as a one-level plan: stride 1, dense when the shard is small
FilterPlan plan_full(int64_t n, int nq, int k, int ep) {
  FilterPlan p = plan_filter(n, nq, k, ep);
  const Level last = p.lv[p.n_levels - 1];
  p.n_levels = 1;
  p.lv[0] = last;
  p.max_slabs = last.n_slabs;
  p.topm = false;
  return p;
}

// Shared prologue of the single-shard call and the sharded stages: validation, plan, carve.
// full_only: the sharded full / finish stages' one-level plan (plan_full).
int filter_setup(const float* db, const uint16_t* db_bf16, int64_t n, int32_t d, int64_t ld_db,
                 const float* q, int32_t nq, int64_t ld_q, int32_t k, void* workspace,
                 int64_t workspace_bytes, int* ep_out, FilterPlan* p, FilterWs* w,
                 bool full_only = false) {
  TT_REQUIRE(n >= 1 && n <= 0x7fffffffLL, "need 1 <= n < 2^31");
  TT_REQUIRE(nq >= 1, "nq < 1");
  TT_REQUIRE(k >= 1 && k <= n, "need 1 <= k <= n");
  if (k > FL_KMAX) return fail(TT_ERR_UNSUPPORTED, "bf16 filter: k > 128");
  const int ep = tt_padded_dim(d);
  if (ep < 0) return fail(TT_ERR_UNSUPPORTED, "bf16 filter: d > 768");
  TT_REQUIRE(ld_db >= ep && ld_q >= ep && ld_db % 8 == 0 && ld_q % 4 == 0,
             "ld must be >= tt_padded_dim(d), ld_db % 8 == 0 (zero padded)");
  TT_REQUIRE((db == nullptr || ((uintptr_t)db % 16) == 0) && ((uintptr_t)db_bf16 % 16) == 0 &&
                 ((uintptr_t)q % 16) == 0, "pointers must be 16-B aligned");
  *p = full_only ? plan_full(n, nq, k, ep) : plan_filter(n, nq, k, ep);
  *w = carve(workspace, *p, n, d, nq, k);
  if (workspace == nullptr || workspace_bytes < w->total)
    return fail(TT_ERR_WORKSPACE, "bf16 filter: workspace too small");
  *ep_out = ep;
  return TT_OK;
}

// Per-query state (eps2, theta, aref, flags, qsel_n).  fold != nullptr and a ring first level
// (the tmax-first plan): that launch initialises it (*fold filled in, no launch here).
int filter_init(FilterWs& w, const float* q, int nq, int64_t ld_q, int ep, float x_norm_max,
                float x_resid_max, hipStream_t st, const FilterPlan* p = nullptr,
                QueryInit* fold = nullptr, bool want_q16 = false, bool want_q8 = false) {
  TT_REQUIRE(x_norm_max >= 0.0f && x_resid_max >= 0.0f,
             "x_norm_max / x_resid_max must be >= 0 (tt_bf16_image_bounds)");
  if (fold) *fold = QueryInit{0.0f, 0.0f, nullptr, nullptr, nullptr, nullptr};
  if (fold && p && !p->lv[0].dense && p->n_levels > 1) {
    *fold = QueryInit{x_norm_max, x_resid_max, w.eps2, w.aref, w.flags, w.qsel_n};
    return TT_OK;
  }
  // one launch: k_query_eps also resets flags / theta / aref / qsel_n (was a memset + 2 fills)
  const unsigned eps_grid = (unsigned)((nq + 3) / 4);
  switch (ep) {
#define TT_QE(E)                                                                              \
  case E:                                                                                     \
    hipLaunchKernelGGL(k_query_eps<E>, dim3(eps_grid), dim3(256), 0, st, q, nq, ld_q,         \
                       x_norm_max, x_resid_max, w.eps2, w.theta, w.aref, w.flags, w.qsel_n,  \
                       want_q16 ? w.q16 : nullptr, want_q8 ? w.q8 : nullptr,                 \
                       want_q8 ? w.tq8 : nullptr);                                           \
    break;
    TT_QE(64) TT_QE(128) TT_QE(256) TT_QE(384) TT_QE(512) TT_QE(768)
#undef TT_QE
  }
  w.q16_valid = want_q16;
  return check_launch("filter_init");
}

// whether this thread's last batched search ran its sample level on the int8 image (tests)
thread_local bool g_last_sample_i8 = false;
// the int8 image for the batched sample level (k_sample_i8), when the caller has one
struct I8Sample {
  const int8_t* x;
  int64_t ld;
  const float* scales;
};
#ifndef TT_SAMPLE_I8
#define TT_SAMPLE_I8 1  // 0: the batched sample level stays on the bf16 ring (A/B builds)
#endif
TT_CHECK_EXP(TT_SAMPLE_I8 != 1, "TT_SAMPLE_I8");
// the batched search's first level runs on the int8 image: a large batch at E = 384 whose plan
// starts with the stride-16 tile-max sample and has the full level after it
static bool sample_i8_applies(const FilterPlan& p, int nq, int ep, bool q16) {
  return TT_SAMPLE_I8 && ep == 384 && q16 && nq > RG_SMALL_NQ && !p.small &&
         p.n_levels == 2 && p.lv[0].tmax && !p.lv[0].dense && p.lv[0].stride == 16 &&
         p.lv[0].n_slabs_p == 0 && p.lv[0].rows_per_slab % 64 == 0 &&
         (int64_t)p.lv[0].rows_per_slab <= SI_MAXROWS;
}

// level li (+ its selection in `mode`); events around the full-catalog level
int filter_level(const FilterPlan& p, const FilterWs& w, int li, int mode, const uint16_t* db16,
                 int64_t n, int64_t ld_db, const float* q, int nq, int64_t ld_q, int k, int ep,
                 hipStream_t st, void* ev_start, void* ev_stop, const float* stats = nullptr,
                 int* pcount = nullptr, float* smax_out = nullptr, int fin = 0,
                 bool no_select = false,
                 const QueryInit& qi = QueryInit{0.0f, 0.0f, nullptr, nullptr, nullptr, nullptr},
                 const I8Sample* i8s = nullptr) {
  const Level& L = p.lv[li];
  const bool last = li == p.n_levels - 1;
  // k_filter_ring addresses a tile (TR sample rows) through one buffer resource: < 2 GiB
  if (!L.dense && L.stride * ld_db * 2 * ring_tr(ep) > 0x7fffffffLL)
    return fail(TT_ERR_UNSUPPORTED, "bf16 filter: catalog sample stride too large");
  if (last && ev_start && hipEventRecord((hipEvent_t)ev_start, st) != hipSuccess)
    return fail(TT_ERR_LAUNCH, "hipEventRecord(start)");
  if (i8s && li == 0 && !last) {  // sample_i8_applies checked the shape
    const int nqt = (nq + SI_QPB - 1) / SI_QPB;
    hipLaunchKernelGGL(k_sample_i8<384>, dim3((unsigned)(nqt * L.n_slabs)), dim3(64 * SI_NW), 0, st,
                       i8s->x, i8s->ld, i8s->scales, n, L.n_sample, L.rows_per_slab, L.n_slabs,
                       w.q8, w.tq8, nq, w.lists, w.counts);
  } else
  switch (ep) {
    case 64: launch_level<64>(L, db16, n, ld_db, q, nq, ld_q, w, st, qi); break;
    case 128: launch_level<128>(L, db16, n, ld_db, q, nq, ld_q, w, st, qi); break;
    case 256: launch_level<256>(L, db16, n, ld_db, q, nq, ld_q, w, st, qi); break;
    case 384: launch_level<384>(L, db16, n, ld_db, q, nq, ld_q, w, st, qi); break;
    case 512: launch_level<512>(L, db16, n, ld_db, q, nq, ld_q, w, st, qi); break;
    case 768: launch_level<768>(L, db16, n, ld_db, q, nq, ld_q, w, st, qi); break;
    default: return fail(TT_ERR_UNSUPPORTED, "bad padded dim");
  }
  int rc = check_launch("k_filter");
  if (rc) return rc;
  if (last && ev_stop && hipEventRecord((hipEvent_t)ev_stop, st) != hipSuccess)
    return fail(TT_ERR_LAUNCH, "hipEventRecord(stop)");
  if (no_select) return TT_OK;
  auto sel = select_reg_disabled()  ? k_select_wave
             : L.n_slabs <= 64      ? k_select_reg<false>
             : L.n_slabs <= 64 * SR_GMAX ? k_select_reg<true>
                                    : k_select_wave;
  hipLaunchKernelGGL(sel, dim3((nq + 3) / 4), dim3(256), 0, st, w.lists, w.counts,
                     L.n_slabs, k, p.J, w.eps2, mode, w.theta, w.aref, w.band, w.band_n,
                     w.band_p1, w.flags, w.qsel, w.qsel_n, nq, stats, pcount, smax_out, fin);
  return check_launch("k_select");
}

// the full level's threshold: aref = theta (a_J of the last sample, global max when sharded),
// theta = aref - 2 eps
int full_threshold(const FilterWs& w, int nq, hipStream_t st) {
  const unsigned g = (unsigned)((nq + 255) / 256);
  if (hipMemcpyAsync(w.aref, w.theta, (size_t)nq * 4, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return fail(TT_ERR_LAUNCH, "hipMemcpyAsync(aref)");
  hipLaunchKernelGGL(k_sub_arr, dim3(g), dim3(256), 0, st, w.theta, w.eps2, nq);
  return check_launch("k_sub_arr");
}

int filter_finish(const FilterWs& w, const float* db, int64_t n, int32_t d, int64_t ld_db,
                  int64_t row_base, const float* q, int nq, int64_t ld_q, int k, int ep,
                  float* out_score, int64_t* out_idx, hipStream_t st,
                  const float* cut = nullptr) {
  TT_REQUIRE(db != nullptr && out_score && out_idx, "null pointer");
  switch (ep) {
#define TT_RR(E)                                                                              \
  case E:                                                                                     \
    if (cut)                                                                                  \
      hipLaunchKernelGGL(k_rerank_wave<E>, dim3((nq + 3) / 4), dim3(256), 0, st, db, ld_db, q, \
                         ld_q, w.band, w.band_n, w.flags, w.qsel, w.qsel_n, nq, n, k,         \
                         row_base, cut, out_score, out_idx);                                  \
    else                                                                                      \
      hipLaunchKernelGGL(k_rerank<E>, dim3(nq), dim3(256), 0, st, db, ld_db, q, ld_q, w.band, \
                         w.band_n, w.band_p1, w.eps2, w.aref, w.flags, w.qsel, w.qsel_n, n, k,\
                         row_base, out_score, out_idx);                                       \
    break;
    TT_RR(64) TT_RR(128) TT_RR(256) TT_RR(384) TT_RR(512) TT_RR(768)
#undef TT_RR
  }
  int rc = check_launch("k_rerank");
  if (rc) return rc;
  // exact fallback for flagged queries (blocks exit at once when none is flagged)
  return scan_f32_select_fused(db, n, d, ld_db, row_base, q, nq, ld_q, k, w.qsel, w.qsel_n,
                               w.done, out_score, out_idx, w.scan_ws, w.scan_ws_bytes, st);
}
}  // namespace

// ---- fault injection for the decoded-row bounds checks (tests only, tt_debug_plant_bad_row)
namespace {
thread_local int g_plant_where = 0, g_plant_query = 0;

// one wave: the largest key of keys[0..n) gets row ~0 (low word 0); xk != nullptr: the key of
// the same slot in xk (the single pass's exact keys) instead.  keys[j] valid for j < n only.
__global__ void k_debug_plant(uint64_t* keys, uint64_t* xk, const int* counts, int n_lists,
                              int list_cap) {
  const int lane = threadIdx.x;
  uint64_t best = 0ull;
  int64_t at = -1;
  for (int b = 0; b < n_lists; ++b) {
    const int c = counts[b];
    for (int j = lane; j < c && j < list_cap; j += 64) {
      const int64_t o = (int64_t)b * list_cap + j;
      if (keys[o] > best) {
        best = keys[o];
        at = o;
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t ob = __shfl_xor(best, o, 64);
    const int64_t oa = __shfl_xor(at, o, 64);
    if (ob > best) {
      best = ob;
      at = oa;
    }
  }
  if (lane == 0 && at >= 0) {
    uint64_t* t = xk ? xk : keys;
    if (t[at] != 0ull) t[at] &= 0xffffffff00000000ull;
  }
}
}  // namespace

#if TT_EXP_BLKTIME
extern "C" int tt_debug_blkph(void* host, int32_t n) {  // timing builds only
  if (n > BLKTIME_MAX) n = BLKTIME_MAX;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_blkph), (size_t)n * 16) == hipSuccess ? n : -1;
}
extern "C" int tt_debug_blktimes(void* host, int32_t n) {  // timing builds only
  if (n > BLKTIME_MAX) n = BLKTIME_MAX;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_blktime), (size_t)n * 32) == hipSuccess ? n : -1;
}
#endif

#if TT_I8_EXP_CLK
extern "C" int tt_debug_i8clk(void* host) {  // timing builds only: [256][TM_WAVES][8] u64
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_i8clk), sizeof(g_i8clk)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int tt_debug_plant_bad_row(int32_t where, int32_t query) {
  TT_REQUIRE(where >= 0 && where <= 2 && query >= 0, "bad arguments");
  g_plant_where = where;
  g_plant_query = query;
  return TT_OK;
}

namespace {
int scan_topk_bf16f32(const float* db, const uint16_t* db_bf16, int64_t n, int32_t d,
                      int64_t ld_db, int64_t row_base, const float* q, int32_t nq, int64_t ld_q,
                      int32_t k, float x_norm_max, float x_resid_max, float* out_score,
                      int64_t* out_idx, void* workspace, int64_t workspace_bytes, void* stream,
                      void* ev_start, void* ev_stop, const I8Sample* i8 = nullptr) {
  g_last_sample_i8 = false;
  TT_REQUIRE(nq >= 0, "nq < 0");
  if (nq == 0) return TT_OK;
  int ep;
  FilterPlan p;
  FilterWs w;
  int rc = filter_setup(db, db_bf16, n, d, ld_db, q, nq, ld_q, k, workspace, workspace_bytes, &ep,
                        &p, &w);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (p.topm && nq <= TM_NQ_RUN) {  // single pass: stream + per-slab top-m, final, fallback
    TT_REQUIRE(db != nullptr && out_score && out_idx, "null pointer");
    TT_REQUIRE(x_norm_max >= 0.0f && x_resid_max >= 0.0f,
               "x_norm_max / x_resid_max must be >= 0 (tt_bf16_image_bounds)");
    const int G = device_cus();
    const int rows_per_blk = (int)((n + G - 1) / G);
    // lists [nq][G][TM_M] approximate keys, then the exact keys, same shape (plan_filter sized
    // the list region for max_slabs >= G lists of FL_CAP >= 2 TM_M per query)
    static_assert(2 * TM_M <= FL_CAP, "topm lists + exact keys must fit the list region");
    TT_REQUIRE(p.max_slabs >= G, "topm plan: list region smaller than one list per CU");
    uint64_t* xkeys = w.lists + (int64_t)nq * G * TM_M;
    if (ld_db * 2 * ring_tr(ep) > 0x7fffffffLL)
      return fail(TT_ERR_UNSUPPORTED, "bf16 filter: row too long");
    if (ev_start && hipEventRecord((hipEvent_t)ev_start, st) != hipSuccess)
      return fail(TT_ERR_LAUNCH, "hipEventRecord(start)");
    switch (ep) {
#define TT_TM(E)                                                                              \
  case E:                                                                                     \
    hipLaunchKernelGGL(k_filter_topm<E>, dim3(G), dim3(64 * TM_WAVES), 0, st, db_bf16, ld_db, \
                       n, q, nq, ld_q, rows_per_blk, db, x_norm_max, x_resid_max, w.eps2,     \
                       w.lists, xkeys, w.counts, w.flags, w.qsel_n);                          \
    break;
      TT_TM(64) TT_TM(128) TT_TM(256) TT_TM(384) TT_TM(512) TT_TM(768)
#undef TT_TM
    }
    if ((rc = check_launch("k_filter_topm"))) return rc;
    if (ev_stop && hipEventRecord((hipEvent_t)ev_stop, st) != hipSuccess)
      return fail(TT_ERR_LAUNCH, "hipEventRecord(stop)");
    if (g_plant_where == 2 && g_plant_query < nq) {  // test hook: corrupt an exact key
      hipLaunchKernelGGL(k_debug_plant, dim3(1), dim3(64), 0, st,
                         w.lists + (int64_t)g_plant_query * G * TM_M,
                         xkeys + (int64_t)g_plant_query * G * TM_M,
                         w.counts + (int64_t)g_plant_query * G, G, TM_M);
      g_plant_where = 0;
      if ((rc = check_launch("k_debug_plant"))) return rc;
    }
    switch (ep) {
#define TT_TF(E)                                                                              \
  case E:                                                                                     \
    hipLaunchKernelGGL(k_final_topm<E>, dim3(nq), dim3(SM_THREADS), 0, st, w.lists, xkeys,    \
                       w.counts, G, k, w.eps2, w.flags, w.qsel, w.qsel_n, n, row_base,        \
                       out_score, out_idx);                                                   \
    break;
      TT_TF(64) TT_TF(128) TT_TF(256) TT_TF(384) TT_TF(512) TT_TF(768)
#undef TT_TF
    }
    if ((rc = check_launch("k_final_topm"))) return rc;
    return scan_f32_select_fused(db, n, d, ld_db, row_base, q, nq, ld_q, k, w.qsel, w.qsel_n,
                                 w.done, out_score, out_idx, w.scan_ws, w.scan_ws_bytes, st);
  }
  QueryInit qinit;
  // k_query_eps (one launch) writes the per-query state AND the bf16 query image the ring
  // levels load (TT_Q16_SMALL=0 timing builds: small batches fold the state into the first level)
  const bool q16 = (nq > RG_SMALL_NQ || TT_Q16_SMALL) && q16_enabled();
  const I8Sample* i8s = i8 && sample_i8_applies(p, nq, ep, q16) ? i8 : nullptr;
  g_last_sample_i8 = i8s != nullptr;
  if ((rc = filter_init(w, q, nq, ld_q, ep, x_norm_max, x_resid_max, st, &p, q16 ? nullptr : &qinit,
                        q16, i8s != nullptr)))
    return rc;
  if (q16) qinit = QueryInit{0.0f, 0.0f, nullptr, nullptr, nullptr, nullptr};
  // small batches: block-per-query selection (k_select_small) and a fused selection +
  // f32-MFMA re-rank of the full level (k_final_small)
  const bool small = p.small;
  for (int li = 0; li < p.n_levels; ++li) {
    const bool last = li == p.n_levels - 1;
    // the last sample level's selection writes the full level's threshold a_J - 2 eps itself
    // (was a copy + k_sub_arr launch: full_threshold, kept for the sharded protocol)
    const int fin = li == p.n_levels - 2;
    if ((rc = filter_level(p, w, li, last ? 1 : 0, db_bf16, n, ld_db, q, nq, ld_q, k, ep, st,
                           ev_start, ev_stop, nullptr, nullptr, nullptr, fin, small,
                           li == 0 ? qinit : QueryInit{0.0f, 0.0f, nullptr, nullptr, nullptr, nullptr},
                           i8s)))
      return rc;
    if (small && !last) {
      hipLaunchKernelGGL(k_select_small, dim3(nq), dim3(SM_THREADS), 0, st, w.lists, w.counts,
                         p.lv[li].n_slabs, p.J, w.eps2, w.theta, w.aref, w.flags, w.qsel,
                         w.qsel_n, fin);
      if ((rc = check_launch("k_select_small"))) return rc;
    }
  }
  if (small) {
    TT_REQUIRE(db != nullptr && out_score && out_idx, "null pointer");
    const int ns = p.lv[p.n_levels - 1].n_slabs;
    switch (ep) {
#define TT_FS(E)                                                                              \
  case E:                                                                                     \
    hipLaunchKernelGGL(k_final_small<E>, dim3(nq), dim3(SM_THREADS), 0, st, w.lists,          \
                       w.counts, ns, k, w.eps2, w.aref, w.flags, w.qsel, w.qsel_n, db, ld_db, \
                       n, q, ld_q, row_base, out_score, out_idx);                             \
    break;
      TT_FS(64) TT_FS(128) TT_FS(256) TT_FS(384) TT_FS(512) TT_FS(768)
#undef TT_FS
    }
    if ((rc = check_launch("k_final_small"))) return rc;
    return scan_f32_select_fused(db, n, d, ld_db, row_base, q, nq, ld_q, k, w.qsel, w.qsel_n,
                                 w.done, out_score, out_idx, w.scan_ws, w.scan_ws_bytes, st);
  }
  if (g_plant_where == 1 && g_plant_query < nq) {  // test hook: corrupt a band key
    hipLaunchKernelGGL(k_debug_plant, dim3(1), dim3(64), 0, st,
                       w.band + (int64_t)g_plant_query * BAND_CAP, (uint64_t*)nullptr,
                       w.band_n + g_plant_query, 1, BAND_CAP);
    g_plant_where = 0;
    if ((rc = check_launch("k_debug_plant"))) return rc;
  }
  return filter_finish(w, db, n, d, ld_db, row_base, q, nq, ld_q, k, ep, out_score, out_idx, st);
}
}  // namespace

extern "C" int tt_scan_topk_bf16f32(const float* db, const uint16_t* db_bf16, int64_t n,
                                    int32_t d, int64_t ld_db, int64_t row_base, const float* q,
                                    int32_t nq, int64_t ld_q, int32_t k, float x_norm_max,
                                    float x_resid_max, float* out_score, int64_t* out_idx,
                                    void* workspace, int64_t workspace_bytes, void* stream,
                                    void* ev_start, void* ev_stop) {
  const int rc = scan_topk_bf16f32(db, db_bf16, n, d, ld_db, row_base, q, nq, ld_q, k, x_norm_max,
                                   x_resid_max, out_score, out_idx, workspace, workspace_bytes,
                                   stream, ev_start, ev_stop);
  // the test hook is armed for ONE call: disarmed whichever path (or early return) the call took,
  // so it can never corrupt a later search on this thread
  g_plant_where = 0;
  return rc;
}

extern "C" int tt_scan_topk_bf16f32_i8s(const float* db, const uint16_t* db_bf16,
                                        const int8_t* db_i8, const float* tile_scales, int64_t n,
                                        int32_t d, int64_t ld_db, int64_t ld_i8, int64_t row_base,
                                        const float* q, int32_t nq, int64_t ld_q, int32_t k,
                                        float x_norm_max, float x_resid_max, float* out_score,
                                        int64_t* out_idx, void* workspace, int64_t workspace_bytes,
                                        void* stream, void* ev_start, void* ev_stop) {
  TT_REQUIRE(db_i8 == nullptr || (tile_scales != nullptr && ld_i8 >= tt_padded_dim(d) &&
                                  ld_i8 % 16 == 0 && ((uintptr_t)db_i8 % 16) == 0),
             "int8 image: tile scales, ld_i8 >= tt_padded_dim(d), multiple of 16, 16-B aligned");
  const I8Sample i8{db_i8, ld_i8, tile_scales};
  const int rc = scan_topk_bf16f32(db, db_bf16, n, d, ld_db, row_base, q, nq, ld_q, k, x_norm_max,
                                   x_resid_max, out_score, out_idx, workspace, workspace_bytes,
                                   stream, ev_start, ev_stop, db_i8 ? &i8 : nullptr);
  g_plant_where = 0;
  return rc;
}

extern "C" int tt_debug_last_sample_i8(void) { return g_last_sample_i8 ? 1 : 0; }

// Test hook: while set, the int8 single pass reports TT_ERR_UNSUPPORTED for every shape (and
// tt_i8_single_pass_ok says 0), as it does past its row limit or on a GPU with > 256 CUs.
static bool g_i8_force_unsupported = false;
extern "C" int tt_debug_i8_force_unsupported(int32_t on) {
  g_i8_force_unsupported = on != 0;
  return TT_OK;
}
// The shape limits of tt_scan_topk_i8f32 without a launch: the single-pass plan (nq <= 8,
// device_cus() * TM_M <= TM_CAP, TT_FILTER_TOPM), the per-block scale-tile limit (rows per CU
// <= 65536) and the 31-bit tile offsets.  1: the call would run, 0: it would return
// TT_ERR_UNSUPPORTED (the caller then takes tt_scan_topk_bf16f32).
static bool i8_single_pass_fits(int64_t n, int ep, int nq, int k, int64_t ld_i8,
                                bool tiled = false) {
  if (g_i8_force_unsupported || (ep != 384 && ep != 768) || (tiled && ep != 384) || nq < 1 ||
      nq > (tiled ? TM_NQ_I8T : TM_NQ_I8) || k < 1 || k > FL_KMAX || k > n || n < 1 ||
      n > 0x7fffffffLL)
    return false;
  if (!plan_filter(n, nq, k, ep).topm) return false;
  const int G = device_cus();
  const int64_t rpb = ((n + G - 1) / G + 63) / 64 * 64;
  return rpb / 64 <= I8_MAXTILES && ld_i8 * (24576 / ep) <= 0x7fffffffLL;
}

extern "C" int tt_i8_single_pass_ok(int64_t n, int32_t d, int32_t nq, int32_t k, int64_t ld_i8) {
  const int ep = tt_padded_dim(d);
  return ep > 0 && i8_single_pass_fits(n, ep, nq, k, ld_i8 > 0 ? ld_i8 : ep) ? 1 : 0;
}

extern "C" int tt_i8t_single_pass_ok(int64_t n, int32_t d, int32_t nq, int32_t k) {
  const int ep = tt_padded_dim(d);
  return ep > 0 && i8_single_pass_fits(n, ep, nq, k, ep, true) ? 1 : 0;
}

namespace {
// tt_scan_topk_i8f32 (row-major image, LDS-ring stream k_filter_topm_i8) and
// tt_scan_topk_i8t_f32 (tiled image, register-fed stream k_filter_topm_i8r): the same plan,
// workspace, final and fallback
int i8_single_pass(const float* db, const int8_t* img, bool tiled, const float* tile_scales,
                   int64_t n, int32_t d, int64_t ld_db, int64_t ld_i8, int64_t row_base,
                   const float* q, int32_t nq, int64_t ld_q, int32_t k, float x_norm_max,
                   float x_resid_max, float s_max, float* out_score, int64_t* out_idx,
                   void* workspace, int64_t workspace_bytes, void* stream, void* ev_start,
                   void* ev_stop) {
  TT_REQUIRE(nq >= 0, "nq < 0");
  if (nq == 0) return TT_OK;
  TT_REQUIRE(db != nullptr && img != nullptr && tile_scales != nullptr && out_score &&
                 out_idx, "null pointer");
  const int ep = tt_padded_dim(d);
  if (ep != 384 && ep != 768) return fail(TT_ERR_UNSUPPORTED, "int8 single pass: E 384 / 768");
  if (tiled && ep != 384) return fail(TT_ERR_UNSUPPORTED, "tiled int8 single pass: E 384");
  if (nq > (tiled ? TM_NQ_I8T : TM_NQ_I8))
    return fail(TT_ERR_UNSUPPORTED, tiled ? "tiled int8 single pass: nq <= 32"
                                          : "int8 single pass: nq <= 8");
  if (tiled) ld_i8 = ep;
  TT_REQUIRE(ld_i8 >= ep && ld_i8 % 16 == 0 && ((uintptr_t)img % 16) == 0,
             "int8 image: ld_i8 >= tt_padded_dim(d), multiple of 16, 16-B aligned");
  TT_REQUIRE(x_norm_max >= 0.0f && x_resid_max >= 0.0f && s_max >= 0.0f,
             "bounds must be >= 0 (tt_i8_image)");
  if (g_i8_force_unsupported) return fail(TT_ERR_UNSUPPORTED, "int8 single pass: forced (test)");
  int epx;
  FilterPlan p;
  FilterWs w;
  int rc = filter_setup(db, (const uint16_t*)img, n, d, ld_db, q, nq, ld_q, k, workspace,
                        workspace_bytes, &epx, &p, &w);
  if (rc) return rc;
  if (!p.topm) return fail(TT_ERR_UNSUPPORTED, "int8 single pass: not a single-pass plan");
  const int G = device_cus();
  TT_REQUIRE(p.max_slabs >= G, "topm plan: list region smaller than one list per CU");
  const int64_t rpb = ((n + G - 1) / G + 63) / 64 * 64;
  if (rpb / 64 > I8_MAXTILES) return fail(TT_ERR_UNSUPPORTED, "int8 single pass: n too large");
  if (ld_i8 * (24576 / ep) > 0x7fffffffLL) return fail(TT_ERR_UNSUPPORTED, "int8: row too long");
  hipStream_t st = (hipStream_t)stream;
  uint64_t* xkeys = w.lists + (int64_t)nq * G * TM_M;
  if (ev_start && hipEventRecord((hipEvent_t)ev_start, st) != hipSuccess)
    return fail(TT_ERR_LAUNCH, "hipEventRecord(start)");
  // candidate buffers laid out for 4 queries (4x the rows each) or for 8
  auto kern = ep == 384 ? (nq <= 4 ? k_filter_topm_i8<384, 4> : k_filter_topm_i8<384, TM_NQ_I8>)
                        : (nq <= 4 ? k_filter_topm_i8<768, 4> : k_filter_topm_i8<768, TM_NQ_I8>);
  if (tiled)  // (rpb <= 65536 rows: a slab's tiled bytes fit the buffer resource's record count)
    kern = nq <= 4    ? k_filter_topm_i8r<384, 4, 1>
           : nq <= 8  ? k_filter_topm_i8r<384, 8, 1>
           : nq <= 16 ? k_filter_topm_i8r<384, 16, 1>
                      : k_filter_topm_i8r<384, 32, 2>;
  hipLaunchKernelGGL(kern, dim3(G), dim3(64 * TM_WAVES), 0, st, img, ld_i8, tile_scales, n, q,
                     nq, ld_q, (int)rpb, db, ld_db, x_norm_max, x_resid_max, s_max, w.eps2,
                     w.lists, xkeys, w.counts, w.flags, w.qsel_n);
  if ((rc = check_launch(tiled ? "k_filter_topm_i8r" : "k_filter_topm_i8"))) return rc;
  if (ev_stop && hipEventRecord((hipEvent_t)ev_stop, st) != hipSuccess)
    return fail(TT_ERR_LAUNCH, "hipEventRecord(stop)");
  if (ep == 384)
    hipLaunchKernelGGL(k_final_topm_i8<384>, dim3(nq), dim3(SM_THREADS), 0, st, w.lists, xkeys,
                       w.counts, G, k, w.eps2, w.flags, w.qsel, w.qsel_n, n, row_base, out_score,
                       out_idx);
  else
    hipLaunchKernelGGL(k_final_topm_i8<768>, dim3(nq), dim3(SM_THREADS), 0, st, w.lists, xkeys,
                       w.counts, G, k, w.eps2, w.flags, w.qsel, w.qsel_n, n, row_base, out_score,
                       out_idx);
  if ((rc = check_launch("k_final_topm_i8"))) return rc;
  return scan_f32_select_fused(db, n, d, ld_db, row_base, q, nq, ld_q, k, w.qsel, w.qsel_n,
                               w.done, out_score, out_idx, w.scan_ws, w.scan_ws_bytes, st);
}
}  // namespace

extern "C" int tt_scan_topk_i8f32(const float* db, const int8_t* db_i8, const float* tile_scales,
                                  int64_t n, int32_t d, int64_t ld_db, int64_t ld_i8,
                                  int64_t row_base, const float* q, int32_t nq, int64_t ld_q,
                                  int32_t k, float x_norm_max, float x_resid_max, float s_max,
                                  float* out_score, int64_t* out_idx, void* workspace,
                                  int64_t workspace_bytes, void* stream, void* ev_start,
                                  void* ev_stop) {
  return i8_single_pass(db, db_i8, false, tile_scales, n, d, ld_db, ld_i8, row_base, q, nq, ld_q,
                        k, x_norm_max, x_resid_max, s_max, out_score, out_idx, workspace,
                        workspace_bytes, stream, ev_start, ev_stop);
}

extern "C" int tt_scan_topk_i8t_f32(const float* db, const int8_t* db_i8t,
                                    const float* tile_scales, int64_t n, int32_t d, int64_t ld_db,
                                    int64_t row_base, const float* q, int32_t nq, int64_t ld_q,
                                    int32_t k, float x_norm_max, float x_resid_max, float s_max,
                                    float* out_score, int64_t* out_idx, void* workspace,
                                    int64_t workspace_bytes, void* stream, void* ev_start,
                                    void* ev_stop) {
  return i8_single_pass(db, db_i8t, true, tile_scales, n, d, ld_db, 0, row_base, q, nq, ld_q, k,
                        x_norm_max, x_resid_max, s_max, out_score, out_idx, workspace,
                        workspace_bytes, stream, ev_start, ev_stop);
}

// ------------------------------------------------------------------ sharded (multi-GPU)
namespace {
__global__ void k_pack_stats(const float* __restrict__ theta, const float* __restrict__ smax,
                             int nq, float* __restrict__ stats) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nq) {
    stats[2 * i] = theta[i];
    stats[2 * i + 1] = smax[i];
  }
}

// full-level threshold from the exchanged sample statistic: aref = theta_g, theta = theta_g - eps2
__global__ void k_stats_theta(const float* __restrict__ stats, const float* __restrict__ eps2,
                              int nq, float* __restrict__ aref, float* __restrict__ theta) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nq) {
    aref[i] = stats[2 * i];
    theta[i] = stats[2 * i] - eps2[i];
  }
}

int sharded_setup(const float* db, const uint16_t* db_bf16, int64_t n, int32_t d, int64_t ld_db,
                  const float* q, int32_t nq, int64_t ld_q, int32_t k, void* workspace,
                  int64_t workspace_bytes, int* ep, FilterPlan* p, FilterWs* w) {
  return filter_setup(db, db_bf16, n, d, ld_db, q, nq, ld_q, k, workspace, workspace_bytes, ep, p,
                      w, true);
}
}  // namespace

extern "C" int tt_sharded_workspace_bytes(int64_t n, int32_t d, int32_t nq, int32_t k,
                                          int64_t* bytes) {
  TT_REQUIRE(bytes != nullptr, "bytes == NULL");
  TT_REQUIRE(n >= 1 && nq >= 1 && k >= 1, "n, nq, k must be >= 1");
  const int ep = tt_padded_dim(d);
  TT_REQUIRE(ep > 0, "d > 768");
  *bytes = carve(nullptr, plan_full(n, nq, k, ep), n, d, nq, k).total;
  return TT_OK;
}

extern "C" int tt_sharded_fallback_offset(int64_t n, int32_t d, int32_t nq, int32_t k,
                                          int64_t* offset) {
  TT_REQUIRE(offset != nullptr && n >= 1 && nq >= 1 && k >= 1, "bad arguments");
  const int ep = tt_padded_dim(d);
  TT_REQUIRE(ep > 0, "d > 768");
  const FilterWs w = carve(nullptr, plan_full(n, nq, k, ep), n, d, nq, k);
  *offset = (int64_t)((char*)w.qsel_n - (char*)4096);
  return TT_OK;
}

extern "C" int tt_sharded_filter_begin(const uint16_t* sample_bf16, int64_t n_sample, int32_t d,
                                       int64_t ld, const float* q, int32_t nq, int64_t ld_q,
                                       int32_t k, float* stats, void* workspace,
                                       int64_t workspace_bytes, void* stream) {
  TT_REQUIRE(stats != nullptr, "stats == NULL");
  TT_REQUIRE(nq >= 0, "nq < 0");
  if (nq == 0) return TT_OK;
  int ep;
  FilterPlan p;
  FilterWs w;
  // the sample may hold fewer than k rows: plan with k' = min(k, n_sample), J from k
  const int32_t kk = (int64_t)k > n_sample ? (int32_t)n_sample : k;
  TT_REQUIRE(k >= 1 && k <= FL_KMAX, "need 1 <= k <= 128");
  int rc = filter_setup(nullptr, sample_bf16, n_sample, d, ld, q, nq, ld_q, kk, workspace,
                        workspace_bytes, &ep, &p, &w);
  if (rc) return rc;
  p = plan_filter(n_sample, nq, k, ep);  // same J as the single-catalog call for this k
  {
    // The replicated sample IS the single-catalog call's first (tile-max) level when its
    // tiles fit one selection: one level at theta = -inf whose J-th largest tile maximum (a
    // lower bound of a_J, exactly the single-GPU threshold) replaces the sample's own two-level
    // ladder and its exact a_J -- one filter launch and one selection fewer per step.  Only
    // when the level's slabs fit the workspace carved for the generic plan.
    const int64_t TR = ring_tr(ep);
    const int qpb = ring_qpb_rt(ep, ring_lvl(true, nq, ep));
    if (n_sample > SEL_CAP / 2 && (n_sample + TR - 1) / TR <= SW_CAP_TILES && p.n_levels > 1) {
      Level L;
      L.stride = 1;
      L.n_sample = n_sample;
      L.dense = false;
      L.tmax = true;
      L.n_qt = (nq + qpb - 1) / qpb;
      int64_t sl = ring_slabs(L.n_qt, n_sample, (n_sample + FL_CAP * TR - 1) / (FL_CAP * TR));
      int64_t r = (n_sample + sl - 1) / sl;
      r = (r + 63) / 64 * 64;
      L.rows_per_slab = (int)r;
      L.n_slabs = (int)((n_sample + r - 1) / r);
      if (L.n_slabs <= p.max_slabs) {
        p.n_levels = 1;
        p.lv[0] = L;
      }
    }
  }
  hipStream_t st = (hipStream_t)stream;
  if ((rc = filter_init(w, q, nq, ld_q, ep, 0.0f, 0.0f, st, nullptr, nullptr,
                        nq > RG_SMALL_NQ && q16_enabled())))
    return rc;
  for (int li = 0; li < p.n_levels; ++li) {
    const bool last = li == p.n_levels - 1;
    if ((rc = filter_level(p, w, li, 0, sample_bf16, n_sample, ld, q, nq, ld_q, k, ep, st, nullptr,
                           nullptr, nullptr, nullptr, last ? w.cut : nullptr)))
      return rc;
  }
  hipLaunchKernelGGL(k_pack_stats, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, w.theta,
                     w.cut, nq, stats);
  return check_launch("k_pack_stats");
}

extern "C" int tt_sharded_filter_full(const uint16_t* db_bf16, int64_t n, int32_t d,
                                      int64_t ld_db, const float* q, int32_t nq, int64_t ld_q,
                                      int32_t k, float x_norm_max, float x_resid_max,
                                      const float* stats, int32_t* probe_counts, void* workspace,
                                      int64_t workspace_bytes, void* stream, void* ev_start,
                                      void* ev_stop) {
  TT_REQUIRE(stats != nullptr && probe_counts != nullptr, "null pointer");
  TT_REQUIRE(nq >= 0, "nq < 0");
  if (nq == 0) return TT_OK;
  int ep;
  FilterPlan p;
  FilterWs w;
  int rc = sharded_setup(nullptr, db_bf16, n, d, ld_db, q, nq, ld_q, k, workspace, workspace_bytes,
                         &ep, &p, &w);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if ((rc = filter_init(w, q, nq, ld_q, ep, x_norm_max, x_resid_max, st, nullptr, nullptr,
                        nq > RG_SMALL_NQ && q16_enabled())))
    return rc;
  hipLaunchKernelGGL(k_stats_theta, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, stats,
                     w.eps2, nq, w.aref, w.theta);
  if ((rc = check_launch("k_stats_theta"))) return rc;
  return filter_level(p, w, 0, 2, db_bf16, n, ld_db, q, nq, ld_q, k, ep, st, ev_start, ev_stop,
                      stats, probe_counts, nullptr);
}

extern "C" int tt_sharded_filter_finish(const float* db, const uint16_t* db_bf16, int64_t n,
                                        int32_t d, int64_t ld_db, int64_t row_base,
                                        const float* q, int32_t nq, int64_t ld_q, int32_t k,
                                        const float* stats, const int32_t* probe_counts,
                                        float* out_score, int64_t* out_idx, void* workspace,
                                        int64_t workspace_bytes, void* stream) {
  TT_REQUIRE(stats != nullptr && probe_counts != nullptr, "null pointer");
  TT_REQUIRE(nq >= 0, "nq < 0");
  if (nq == 0) return TT_OK;
  int ep;
  FilterPlan p;
  FilterWs w;
  int rc = sharded_setup(db, db_bf16, n, d, ld_db, q, nq, ld_q, k, workspace, workspace_bytes,
                         &ep, &p, &w);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_probe_cut, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st,
                     probe_counts, stats, w.eps2, nq, k, w.flags, w.qsel, w.qsel_n, w.cut);
  if ((rc = check_launch("k_probe_cut"))) return rc;
  return filter_finish(w, db, n, d, ld_db, row_base, q, nq, ld_q, k, ep, out_score, out_idx, st,
                       w.cut);
}
