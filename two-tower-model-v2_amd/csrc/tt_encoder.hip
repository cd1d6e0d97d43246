// tt_encoder.hip -- item-tower text encoder (MiniLM-class BERT) + projection head (gfx950).
//
// Replaces (reference file:line):
//   ItemTower.encode_text -> SentenceTransformer.encode   src/models/item_tower.py:100-124
//     (BertModel forward + mean pooling over the attention mask, normalize_embeddings=False)
//   ItemTower.encode_categorical + forward                item_tower.py:126-211
//     (concat [text | brand | category] -> Linear -> ReLU -> (Dropout: eval) -> Linear ->
//      F.normalize)
//
// Sequences are PACKED (varlen): the T = sum(L_i) real tokens of a batch are rows of one
// [T, H] activation matrix and cu_seqlens[n_seq+1] delimits them.  The reference pads each
// length-sorted batch of 32 to its longest text; padded keys are masked out of attention and
// padded rows out of the mean pool, so packing computes the same function with no work on
// padding.
//
// Kernels (one layer = 4 GEMMs + attention + 2 LayerNorms):
//   k_gemm<T>    C[M,N] = A[M,K] . W[N,K]^T (+bias, GELU/ReLU, +residual), f32 out (+bf16 copy).
//                128x128 block tile, 4 waves of 64x64, MFMA v_mfma_f32_16x16x4_f32 (T = float:
//                the parity path) or v_mfma_f32_16x16x32_bf16 (T = bf16: the fast path, f32
//                accumulate).  Tiles stream HBM/L2 -> LDS with global_load_lds_dwordx4 (no VGPR
//                round trip), double-buffered; XOR-swizzled 16-B chunks make the ds_read_b128
//                fragment reads conflict-free.  Both element types use 128-B LDS rows
//                (BK = 32 f32 / 64 bf16), so the data path is shared.
//   k_layernorm  wave per row (H <= 1024), two-pass mean/variance, optional bf16 copy.
//   k_embed_ln   word + token-type + position embeddings -> LayerNorm (BertEmbeddings).
//   k_attn       block per (sequence, head): K/V of the head in LDS, one thread per query
//                row, two passes (row max, then exp-weighted sum), f32.
//   k_mean_pool  block per sequence (sentence-transformers Pooling, mean mode).
#include "tt_common.hpp"

#include <type_traits>

namespace tt {

typedef __bf16 bf16x8e __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

enum { ACT_NONE = 0, ACT_GELU = 1, ACT_RELU = 2 };

constexpr int GM_BM = 128, GM_BN = 128;
constexpr int GM_TILE_B = GM_BM * 128;  // one operand tile: 128 rows x 128 B
constexpr int GM_STAGE_B = 2 * GM_TILE_B;

template <typename T>
struct GemmElt;
template <>
struct GemmElt<float> {
  static constexpr int BK = 32;  // elements per 128-B LDS row
};
template <>
struct GemmElt<uint16_t> {
  static constexpr int BK = 64;
};

__device__ __forceinline__ void enc_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
template <int N>
__device__ __forceinline__ void enc_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}

// The bf16 path's GELU: erf by Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7 absolute, far
// below the bf16 rounding of the outputs it feeds): ~12 VALU ops instead of erff's ~35, which
// made the FFN1 GEMM's epilogue VALU-bound.  The f32 (parity) path keeps erff.
__device__ __forceinline__ float gelu_fast(float x) {
  // the exact operation sequence of gelu2_fast's lanes (below), so that the element-wise edge
  // path and the packed full-tile path give identical bits (chunking never changes a row)
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(z, 0.3275911f, 1.0f));
  float p = fmaf(t, 1.061405429f, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float ex = __builtin_amdgcn_exp2f((z * -1.4426950408889634f) * z);
  const float e = copysignf(fmaf(-(p * t), ex, 1.0f), x);  // erf(x / sqrt 2)
  const float hx = x * 0.5f;
  return fmaf(hx, e, hx);
}

typedef __bf16 bf16x2e __attribute__((ext_vector_type(2)));
typedef float f32x2e __attribute__((ext_vector_type(2)));
// gelu_fast on two values with packed math (v_pk_fma_f32 / v_pk_mul_f32 take both lanes of a
// pair per instruction): 20 instructions per pair instead of ~30 -- the FFN1 epilogue's GELU
// was all of its non-MFMA VALU (PMC: 5.4 VALU per MFMA, i.e. VALU-issue-bound).  The same
// A-S 7.1.26 formula; only the operation grouping differs from gelu_fast.
__device__ __forceinline__ f32x2e gelu2_fast(f32x2e x) {
  const f32x2e one = {1.0f, 1.0f};
  const f32x2e z = __builtin_elementwise_abs(x) * 0.70710678118654752f;
  const f32x2e d = __builtin_elementwise_fma(z, f32x2e{0.3275911f, 0.3275911f}, one);
  const f32x2e t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2e p = __builtin_elementwise_fma(t, f32x2e{1.061405429f, 1.061405429f},
                                       f32x2e{-1.453152027f, -1.453152027f});
  p = __builtin_elementwise_fma(p, t, f32x2e{1.421413741f, 1.421413741f});
  p = __builtin_elementwise_fma(p, t, f32x2e{-0.284496736f, -0.284496736f});
  p = __builtin_elementwise_fma(p, t, f32x2e{0.254829592f, 0.254829592f});
  const f32x2e zz = (z * -1.4426950408889634f) * z;  // -z^2 log2(e)
  const f32x2e ex = {__builtin_amdgcn_exp2f(zz.x), __builtin_amdgcn_exp2f(zz.y)};
  const f32x2e e = __builtin_elementwise_copysign(__builtin_elementwise_fma(-(p * t), ex, one), x);
  const f32x2e hx = x * 0.5f;
  return __builtin_elementwise_fma(hx, e, hx);  // 0.5 x (1 + erf(x / sqrt 2))
}
__device__ __forceinline__ void gelu4_fast(f32x4& y) {
  const f32x2e lo = gelu2_fast(f32x2e{y[0], y[1]}), hi = gelu2_fast(f32x2e{y[2], y[3]});
  y = f32x4{lo.x, lo.y, hi.x, hi.y};
}
// two floats -> packed bf16 (round to nearest even) in one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pack_bf16_hw(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2e{a, b}, bf16x2e));
}

// XCD-aware tile order: consecutive logical tiles (same A rows, all N tiles) on one XCD.
__device__ __forceinline__ int enc_xcd_remap(int bid, int nblk) {
  const int q = nblk / 8, r = nblk % 8, x = bid % 8, local = bid / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + local;
}

// timing-only experiment switches (results WRONG when set): tools/exp_filter.sh FILE=tt_encoder
#ifndef TT_GEXP_NOSTORE
#define TT_GEXP_NOSTORE 0  // 1: skip k_gemm_big's epilogue; 2: compute it, skip its bf16 stores
#endif
// Epilogue of one wave's 64x64 accumulator tile, stored straight from registers.  The MFMAs
// compute the TRANSPOSED block D = W . A^T, so lane (g = l >> 4, rl = l & 15) of block (i, j)
// holds C[m = mw0 + 16 i + rl][n = nw0 + 16 j + 4 g + v], v = 0..3: four consecutive columns of
// one row -> one 16-B (f32) / 8-B (bf16) store, bias and residual read as 16-B vectors; the
// 4 j-blocks of a row fill its 128-B (bf16) / 256-B (f32) span back to back.
// C or C16 may be NULL (write only the copy the consumer needs).  Returns the number of
// vector-memory stores the lane issued when it is a compile-time count (16 per output copy on
// the full-tile path, 8 for a bf16-only output), or 0 for the element-wise edge path: a persistent caller waits for
// vmcnt(that count) before reusing its DMA ring, without draining the stores.
// ACTC >= 0: the activation as a compile-time constant (no per-element branch); BFO: the
// caller guarantees the bf16-only output form (C == NULL, res == NULL, C16 16-B aligned,
// ldc16 % 8 == 0) -- the persistent kernel's specialisations.
// Split-bf16 interleaved rows ("x3i"), the x3 encoder's activation / weight format: a row of N
// f32 values is 2N bf16, per 32 columns first their hi = bf16(v) then their lo = bf16(v - hi).
// A 128-B LDS row of a GEMM stage is then one 32-k block's hi (chunks 0-3) and lo (4-7): the
// bf16 kernels' two k-halves become the hi and lo operands of the same 32 k.
__device__ __forceinline__ int x3i_col(int n) { return 64 * (n >> 5) + (n & 31); }

// OM: output form.  0 = generic (C and / or C16, residual), 1 = BFO, 2 = SPLIT: the x3
// encoder's split-bf16 interleaved rows (C == NULL,
// res == NULL): C16 row m holds, per 32 columns, hi = bf16(y) then lo = bf16(y - hi)
// (x3i_col; ldc16 >= 2N, N % 32 == 0, 16-B aligned rows), i.e. the A operand of the next x3
// GEMM.  split_n > 0 selects the same form at run time in the generic epilogue (k_gemm's
// small-M path).
template <bool FAST, int ACTC = -1, int OM = 0>
__device__ __forceinline__ int gemm_wave_epilogue(f32x4 (&acc)[4][4], int mw0, int nw0,
                                                   int lane, int M, int N,
                                                   const float* __restrict__ bias,
                                                   const float* __restrict__ res, int64_t ldr,
                                                   float* __restrict__ C, int64_t ldc,
                                                   uint16_t* __restrict__ C16, int64_t ldc16,
                                                   int act, const float* lbias = nullptr,
                                                   int split_n = 0) {
  constexpr bool BFO = OM == 1, SPL = OM == 2;
  const int g = lane >> 4, rl = lane & 15;
  if constexpr (ACTC >= 0) act = ACTC;
  if constexpr (BFO || SPL) {
    C = nullptr;
    res = nullptr;
  }
  if constexpr (SPL) split_n = N;
  const bool vec = (N % 4) == 0 && (ldc % 4) == 0 && (!res || (ldr % 4) == 0) &&
                   (!C16 || (ldc16 % 4) == 0) && ((uintptr_t)bias % 16) == 0 &&
                   ((uintptr_t)res % 16) == 0 && ((uintptr_t)C % 16) == 0 &&
                   ((uintptr_t)C16 % 8) == 0 && mw0 + 64 <= M && nw0 + 64 <= N &&
                   (!SPL || ((N % 32) == 0 && (ldc16 % 8) == 0 && ((uintptr_t)C16 % 16) == 0)) &&
                   (SPL || split_n == 0);
  if (vec) {
    // full tile: every bias / residual load is issued before the first use, so their
    // latencies overlap (a load-use chain per 16x16 block serialises ~16 L2 round trips)
    f32x4 bv[4], rv[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bv[j] = lbias  ? *(const f32x4*)(lbias + nw0 + 16 * j + 4 * g)  // LDS copy: no vmcnt wait
              : bias ? *(const f32x4*)(bias + nw0 + 16 * j + 4 * g)
                     : f32x4{0.f, 0.f, 0.f, 0.f};
    if (res) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          rv[i][j] = *(const f32x4*)(res + (int64_t)(mw0 + 16 * i + rl) * ldr + nw0 + 16 * j + 4 * g);
    }
    if constexpr (SPL) {
      // split planes: the BFO path's permlane16_swap pairing, once for hi and once for lo
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t m = mw0 + 16 * i + rl;
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          uint32_t ph[2][2], pl[2][2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int j = 2 * jp + h;
            f32x4 y = acc[i][j] + bv[j];
            if (FAST && act == ACT_GELU) {
              gelu4_fast(y);
            } else {
#pragma unroll
              for (int u = 0; u < 4; ++u) {
                if (act == ACT_GELU) y[u] = gelu_erf(y[u]);
                else if (act == ACT_RELU) y[u] = y[u] > 0.0f ? y[u] : 0.0f;
              }
            }
            ph[h][0] = pack_bf16_hw(y[0], y[1]);
            ph[h][1] = pack_bf16_hw(y[2], y[3]);
            pl[h][0] = pack_bf16_hw(y[0] - __uint_as_float(ph[h][0] << 16),
                                    y[1] - __uint_as_float(ph[h][0] & 0xffff0000u));
            pl[h][1] = pack_bf16_hw(y[2] - __uint_as_float(ph[h][1] << 16),
                                    y[3] - __uint_as_float(ph[h][1] & 0xffff0000u));
          }
          const auto s0 = __builtin_amdgcn_permlane16_swap(ph[0][0], ph[1][0], false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(ph[0][1], ph[1][1], false, false);
          const auto t0 = __builtin_amdgcn_permlane16_swap(pl[0][0], pl[1][0], false, false);
          const auto t1 = __builtin_amdgcn_permlane16_swap(pl[0][1], pl[1][1], false, false);
          const int n = nw0 + 32 * jp + 16 * (g & 1) + 8 * (g >> 1);  // 8 columns, one 32-block
          uint16_t* o = C16 + m * ldc16 + x3i_col(n);
          *(u32x4*)o = u32x4{s0[0], s1[0], s0[1], s1[1]};
          *(u32x4*)(o + 32) = u32x4{t0[0], t1[0], t0[1], t1[1]};
        }
      }
      return 16;
    }
    if (BFO || (!C && (ldc16 % 8) == 0 && ((uintptr_t)C16 % 16) == 0)) {
      // bf16-only output: v_permlane16_swap pairs blocks j0 = 2 jp and j1 = 2 jp + 1 so that
      // each lane holds 8 consecutive columns -> one 16-B store (8 per lane instead of 16
      // 8-B ones; the epilogue was store-issue-bound).  After the swap lane row g holds
      // columns 32 jp + 16 (g & 1) + 8 (g >> 1) .. + 7.
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t m = mw0 + 16 * i + rl;
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          uint32_t pk[2][2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int j = 2 * jp + h;
            f32x4 y = acc[i][j] + bv[j];
            if (FAST && act == ACT_GELU) {
              gelu4_fast(y);
            } else {
#pragma unroll
              for (int u = 0; u < 4; ++u) {
                if (act == ACT_GELU) y[u] = gelu_erf(y[u]);
                else if (act == ACT_RELU) y[u] = y[u] > 0.0f ? y[u] : 0.0f;
              }
            }
            if (res) y = y + rv[i][j];
            pk[h][0] = pack_bf16_hw(y[0], y[1]);
            pk[h][1] = pack_bf16_hw(y[2], y[3]);
          }
          const auto s0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
          const int n = nw0 + 32 * jp + 16 * (g & 1) + 8 * (g >> 1);
          if (TT_GEXP_NOSTORE != 2 || s0[0] == 0x12345678u)
            *(u32x4*)(C16 + m * ldc16 + n) = u32x4{s0[0], s1[0], s0[1], s1[1]};
        }
      }
      return 8;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t m = mw0 + 16 * i + rl;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = nw0 + 16 * j + 4 * g;
        f32x4 y = acc[i][j] + bv[j];
        if (FAST && act == ACT_GELU) {
          gelu4_fast(y);
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            if (act == ACT_GELU) y[u] = gelu_erf(y[u]);
            else if (act == ACT_RELU) y[u] = y[u] > 0.0f ? y[u] : 0.0f;
          }
        }
        if (res) y = y + rv[i][j];
        if (C) *(f32x4*)(C + m * ldc + n) = y;
        if (C16) *(uint2*)(C16 + m * ldc16 + n) = uint2{pack_bf16_hw(y[0], y[1]),
                                                        pack_bf16_hw(y[2], y[3])};
      }
    }
    return (C ? 16 : 0) + (C16 ? 16 : 0);
  }
  // edge tiles / unaligned operands: element-wise with bounds checks
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mw0 + 16 * i + rl;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = nw0 + 16 * j + 4 * g;
      for (int u = 0; u < 4 && n + u < N; ++u) {
        float y = acc[i][j][u] + (bias ? bias[n + u] : 0.0f);
        if (act == ACT_GELU) y = FAST ? gelu_fast(y) : gelu_erf(y);
        else if (act == ACT_RELU) y = y > 0.0f ? y : 0.0f;
        if (res) y = y + res[(int64_t)m * ldr + n + u];
        if (C) C[(int64_t)m * ldc + n + u] = y;
        if (C16) {
          const uint16_t hv = f32_to_bf16_rne(y);
          if (split_n > 0) {
            uint16_t* o = C16 + (int64_t)m * ldc16 + x3i_col(n + u);
            o[0] = hv;
            o[32] = f32_to_bf16_rne(y - __uint_as_float((uint32_t)hv << 16));
          } else {
            C16[(int64_t)m * ldc16 + n + u] = hv;
          }
        }
      }
    }
  }
  return 0;
}

// Split-bf16 ("x3") operands: an f32 value a = hi + lo + r with hi = bf16(a), lo = bf16(a - hi)
// (a - hi is exact in f32), |r| <= 2^-17 |a|.  Eight f32 (two 16-B LDS fragments) -> the hi
// and lo bf16x8 MFMA operands: 4 v_cvt_pk_bf16_f32 + 8 unpacks + 8 subtracts + 4 packs.
__device__ __forceinline__ void split_bf16x8(const u32x4& f0, const u32x4& f1, bf16x8e& hi,
                                             bf16x8e& lo) {
  const f32x4 a = __builtin_bit_cast(f32x4, f0), b = __builtin_bit_cast(f32x4, f1);
  const u32x4 h = {pack_bf16_hw(a[0], a[1]), pack_bf16_hw(a[2], a[3]), pack_bf16_hw(b[0], b[1]),
                   pack_bf16_hw(b[2], b[3])};
  auto lo16 = [](uint32_t p) { return __uint_as_float(p << 16); };
  auto hi16 = [](uint32_t p) { return __uint_as_float(p & 0xffff0000u); };
  const u32x4 l = {pack_bf16_hw(a[0] - lo16(h[0]), a[1] - hi16(h[0])),
                   pack_bf16_hw(a[2] - lo16(h[1]), a[3] - hi16(h[1])),
                   pack_bf16_hw(b[0] - lo16(h[2]), b[1] - hi16(h[2])),
                   pack_bf16_hw(b[2] - lo16(h[3]), b[3] - hi16(h[3]))};
  hi = __builtin_bit_cast(bf16x8e, h);
  lo = __builtin_bit_cast(bf16x8e, l);
}

// X3 (T = float only): the f32 data path (tiles, swizzle, epilogue) with the products on bf16
// MFMA: per 32-k stage each lane's 8 f32 of a row (its two read steps' chunks) are split into
// hi / lo bf16x8 and acc += W_hi A_hi + W_lo A_hi + W_hi A_lo (the lo.lo term, <= 2^-18
// relative, dropped): 3 v_mfma_f32_16x16x32_bf16 instead of 8 v_mfma_f32_16x16x4_f32 per
// 16x16 block and stage -- 16x the f32 MFMA rate, 3x the work.  The k -> lane assignment (the
// chunks of both read steps) is the same for A and W, so each MFMA still pairs equal k.
// Pre-split weights for X3M = 2: W [N, K] f32 -> Wx [N, 2K] bf16; per 32-k block of a row,
// 32 hi then 32 lo, each in the GEMM lanes' slot order (slot 8 g + u <- k = 4 g + u for u < 4,
// 16 + 4 g + (u - 4) for u >= 4: the f32 tile's chunks g and 4 + g).  Thread per 8 slots.
__global__ __launch_bounds__(256) void k_x3_split_w(const float* __restrict__ W, int64_t ldw,
                                                    int N, int K, uint16_t* __restrict__ out,
                                                    int64_t ldo) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (row, 32-k block, group g)
  const int nb = K / 32;
  if (e >= (int64_t)N * nb * 4) return;
  const int g = (int)(e & 3), kb = (int)((e >> 2) % nb), n = (int)((e >> 2) / nb);
  const float* wr = W + (int64_t)n * ldw + 32 * kb;
  const u32x4 f0 = *(const u32x4*)(wr + 4 * g), f1 = *(const u32x4*)(wr + 16 + 4 * g);
  bf16x8e hi, lo;
  split_bf16x8(f0, f1, hi, lo);
  uint16_t* o = out + (int64_t)n * ldo + 64 * kb + 8 * g;
  *(u32x4*)o = __builtin_bit_cast(u32x4, hi);
  *(u32x4*)(o + 32) = __builtin_bit_cast(u32x4, lo);
}

// x3i weights: W [N, K] f32 -> [N, 2K] bf16 interleaved (x3i_col).  Thread per element.
__global__ __launch_bounds__(256) void k_x3i_w(const float* __restrict__ W, int64_t ldw, int N,
                                               int K, uint16_t* __restrict__ out, int64_t ldo) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)N * K) return;
  const int n = (int)(e / K), k = (int)(e % K);
  const float v = W[(int64_t)n * ldw + k];
  const uint16_t hv = f32_to_bf16_rne(v);
  uint16_t* o = out + (int64_t)n * ldo + x3i_col(k);
  o[0] = hv;
  o[32] = f32_to_bf16_rne(v - __uint_as_float((uint32_t)hv << 16));
}

// X3M = 2: W arrives pre-split (k_x3_split_w): each 32-k stage of a W row is 128 B = 32 hi
// then 32 lo bf16 in the lanes' slot order, so the W tile's read step 0 / 1 chunks ARE the
// lane's hi / lo operands -- only A is split in the loop (half the VALU of X3M = 1, which was
// VALU-bound: 192 VALU beside 48 MFMAs per wave and stage).  W is passed as float* (the same
// 128-B rows per 32 k), ldw in those 4-B units.
// X3I (T = bf16): the stage's A and W rows are x3i interleaved (K here = 2 x the product's K):
// per 32 k, acc += W_hi A_hi + W_lo A_hi + W_hi A_lo -- the split-bf16 (x3) product with the
// bf16 kernels' data path and no split VALU (the producers wrote the operands split).
template <typename T, int X3M = 0, bool X3I = false>
__global__ __launch_bounds__(256, 2) void k_gemm(const T* __restrict__ A, int64_t lda,
                                                 const T* __restrict__ W, int64_t ldw,
                                                 const float* __restrict__ bias,
                                                 const float* __restrict__ res, int64_t ldr,
                                                 float* __restrict__ C, int64_t ldc,
                                                 uint16_t* __restrict__ C16, int64_t ldc16,
                                                 int M, int N, int K, int act, int split_n) {
  constexpr int BK = GemmElt<T>::BK;
  constexpr int EPC = 16 / sizeof(T);  // elements per 16-B chunk
  __shared__ __attribute__((aligned(16))) char smem[2 * GM_STAGE_B];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int n_tn = (N + GM_BN - 1) / GM_BN;
  const int lb = enc_xcd_remap(blockIdx.x, gridDim.x);
  const int tm = lb / n_tn, tn = lb % n_tn;
  const int m0 = tm * GM_BM, n0 = tn * GM_BN;

  // DMA mapping: piece p (0..15) of a tile = LDS bytes [1024p, +1024) = rows 8p..8p+7;
  // lane i -> row 8p + (i >> 3), physical chunk i & 7, logical chunk (i & 7) ^ ((row >> 1) & 7).
  // Wave w issues pieces w, w+4, w+8, w+12 of each operand.
  int64_t a_off[4], w_off[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = w + 4 * j;
    const int row = 8 * p + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    int am = m0 + row;
    am = am < M ? am : M - 1;
    int wn_ = n0 + row;
    wn_ = wn_ < N ? wn_ : N - 1;  // rows past N: clamped loads, masked stores
    a_off[j] = (int64_t)am * lda + c * EPC;
    w_off[j] = (int64_t)wn_ * ldw + c * EPC;
  }
  auto issue = [&](int kt) {
    char* st = smem + (kt & 1) * GM_STAGE_B;
    const int64_t k0 = (int64_t)kt * BK, ka = k0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = w + 4 * j;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(A + a_off[j] + ka),
          (__attribute__((address_space(3))) void*)(st + 1024 * p), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(W + w_off[j] + k0),
          (__attribute__((address_space(3))) void*)(st + GM_TILE_B + 1024 * p), 16, 0, 0);
    }
  };

  // fragment read offsets (bytes within a tile): row r = 64*wm + 16 i + (l & 15) (A) or
  // 64*wn + 16 j + (l & 15) (W); logical chunk c = 4 s + (l >> 4), s = read step 0..1.
  const int g = lane >> 4, rl = lane & 15;
  int fa[4][2], fb[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ra = 64 * wm + 16 * i + rl, rb = 64 * wn + 16 * i + rl;
      const int c = 4 * s + g;
      fa[i][s] = ra * 128 + 16 * (c ^ ((ra >> 1) & 7));
      fb[i][s] = GM_TILE_B + rb * 128 + 16 * (c ^ ((rb >> 1) & 7));
    }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  issue(0);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) {
      issue(kt + 1);
      enc_wait_vm<8>();
    } else {
      enc_wait_vm<0>();
    }
    enc_lds_barrier();
    // all 16 fragment reads of the stage issued up front; counted waits per read step
    const uint32_t sb = lds_addr(smem) + (uint32_t)((kt & 1) * GM_STAGE_B);
    u32x4 av[2][4], bv[2][4];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        av[s][i] = lds_read128<0>(sb + fa[i][s]);
        bv[s][i] = lds_read128<0>(sb + fb[i][s]);
      }
    if constexpr (X3M != 0) {
      static_assert(sizeof(T) == 4, "x3: f32 operands");
      lds_wait<0>();
      bf16x8e ahi[4], alo[4], bhi[4], blo[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        reg_tie(av[0][i]);
        reg_tie(av[1][i]);
        reg_tie(bv[0][i]);
        reg_tie(bv[1][i]);
        split_bf16x8(av[0][i], av[1][i], ahi[i], alo[i]);
        if constexpr (X3M == 2) {
          bhi[i] = __builtin_bit_cast(bf16x8e, bv[0][i]);
          blo[i] = __builtin_bit_cast(bf16x8e, bv[1][i]);
        } else {
          split_bf16x8(bv[0][i], bv[1][i], bhi[i], blo[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bhi[j], ahi[i], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(blo[j], ahi[i], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bhi[j], alo[i], acc[i][j], 0, 0, 0);
        }
    } else if constexpr (X3I) {
      static_assert(sizeof(T) == 2, "x3i: bf16 operands");
      lds_wait<0>();
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        reg_tie(av[0][i]);
        reg_tie(av[1][i]);
        reg_tie(bv[0][i]);
        reg_tie(bv[1][i]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bf16x8e ah = __builtin_bit_cast(bf16x8e, av[0][i]), al = __builtin_bit_cast(bf16x8e, av[1][i]);
          const bf16x8e bh = __builtin_bit_cast(bf16x8e, bv[0][j]), bl = __builtin_bit_cast(bf16x8e, bv[1][j]);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, ah, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl, ah, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, al, acc[i][j], 0, 0, 0);
        }
    } else {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (s == 0) lds_wait<8>();
      else lds_wait<0>();
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        reg_tie(av[s][i]);
        reg_tie(bv[s][i]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if constexpr (sizeof(T) == 4) {
            const f32x4 a = __builtin_bit_cast(f32x4, av[s][i]), b = __builtin_bit_cast(f32x4, bv[s][j]);
#pragma unroll
            for (int u = 0; u < 4; ++u)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[u], a[u], acc[i][j], 0, 0, 0);
          } else {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(  // D = W . A^T (see epilogue)
                __builtin_bit_cast(bf16x8e, bv[s][j]), __builtin_bit_cast(bf16x8e, av[s][i]),
                acc[i][j], 0, 0, 0);
          }
        }
    }
    }
    enc_lds_barrier();
  }

  gemm_wave_epilogue<sizeof(T) == 2>(acc, m0 + 64 * wm, n0 + 64 * wn, lane, M, N, bias, res, ldr,
                                     C, ldc, C16, ldc16, act, nullptr, split_n);
}

// Large-M bf16 GEMM: persistent blocks (one per CU, 8 waves of 64x64 = 256x128 tiles), a
// 3-slot LDS ring (48 KB stages) fed two stages ahead, ONE barrier per k-stage.  The ring runs
// ACROSS tiles: the last two k-steps of a tile already load the first two stages of the
// block's next tile, so the epilogue's stores and the next tile's pipeline fill overlap
// instead of each launch-sized tile paying its DMA latency and store drain in full (measured:
// the 128x128 kernel spends ~3/4 of its time outside the MFMA loop at K = 384).
// DMA layout / swizzle / fragment reads / epilogue as k_gemm.
constexpr int GB_BN = 128, GB_MAXN = 2048;

// T = float: the split-bf16 (x3) product of k_gemm<float, true> on this ring -- a stage is 32
// f32 (the same 128-B LDS rows, so DMA, swizzle and fragment reads are unchanged), and the
// stage's two read steps form one 8-f32 slot set per lane (split_bf16x8, 3 MFMAs per block).
template <int GB_BM, int GB_SLOTS, int ACT, int BFO, typename T = uint16_t, bool X3I = false>
__global__ __launch_bounds__(GB_BM * 2, 512 / (GB_BM * 2)) void k_gemm_big(const T* __restrict__ A, int64_t lda,
                                                     const T* __restrict__ W, int64_t ldw,
                                                     const float* __restrict__ bias,
                                                     const float* __restrict__ res, int64_t ldr,
                                                     float* __restrict__ C, int64_t ldc,
                                                     uint16_t* __restrict__ C16, int64_t ldc16,
                                                     int M, int N, int K, int act) {
  constexpr bool X3 = sizeof(T) == 4;
  constexpr int BK = 128 / sizeof(T), EPC = 16 / sizeof(T);
  constexpr int GB_A_B = GB_BM * 128, GB_W_B = GB_BN * 128, GB_STAGE_B = GB_A_B + GB_W_B;
  constexpr int NW = GB_BM / 32;        // waves: (BM / 64) x 2 of 64 x 64
  constexpr int WP = 16 / NW;           // W pieces per wave and stage (A: 4)
  constexpr int OPS = 4 + WP;           // DMA instructions per lane and stage
  __shared__ __attribute__((aligned(16))) char smem[GB_SLOTS * GB_STAGE_B];
  // the bias in LDS: a global bias load in the epilogue would wait (in-order vmcnt) for the
  // next tile's DMA stages issued just before it
  __shared__ __attribute__((aligned(16))) float sbias[GB_MAXN];
  const int tid = threadIdx.x, lane = tid & 63;
  const bool lds_bias = bias && N <= GB_MAXN && ((uintptr_t)bias % 16) == 0;
  if (lds_bias)
    for (int e = tid; e < N; e += GB_BM * 2) sbias[e] = bias[e];  // visible after stage 0's barrier
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int n_tn = (N + GB_BN - 1) / GB_BN;
  const int ntiles = ((M + GB_BM - 1) / GB_BM) * n_tn;
  const int nk = K / BK;
  // tile r of this block: logical tile (XCD-contiguous ranges; gridDim.x % 8 == 0 keeps a
  // block on one XCD's range)
  auto tile_of = [&](int r) { return enc_xcd_remap(blockIdx.x + r * gridDim.x, ntiles); };
  const int n_mine = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;

  // DMA: A = BM / 8 pieces of 8 rows x 128 B, W = 16 pieces; wave w issues A pieces w + NW j
  // (j < 4) and W pieces w + NW j (j < WP).  Chunk swizzle as k_gemm.  Offsets of the current
  // (cur) and next (nxt) tile.
  struct Offs {
    int64_t a[4], w[WP];
  };
  auto offsets = [&](int lt) __attribute__((always_inline)) {
    Offs o;
    const int m0 = (lt / n_tn) * GB_BM, n0 = (lt % n_tn) * GB_BN;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = 8 * (w + NW * j) + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      int am = m0 + row;
      am = am < M ? am : M - 1;
      o.a[j] = (int64_t)am * lda + c * EPC;
    }
#pragma unroll
    for (int j = 0; j < WP; ++j) {
      const int row = 8 * (w + NW * j) + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      int wr = n0 + row;
      wr = wr < N ? wr : N - 1;
      o.w[j] = (int64_t)wr * ldw + c * EPC;
    }
    return o;
  };
  auto issue = [&](const Offs& o, int kt, int gs) __attribute__((always_inline)) {
    char* st = smem + (gs % GB_SLOTS) * GB_STAGE_B;
    const int64_t k0 = (int64_t)kt * BK, ka = k0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(A + o.a[j] + ka),
          (__attribute__((address_space(3))) void*)(st + 1024 * (w + NW * j)), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < WP; ++j)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(W + o.w[j] + k0),
          (__attribute__((address_space(3))) void*)(st + GB_A_B + 1024 * (w + NW * j)), 16, 0, 0);
  };

  const int g = lane >> 4, rl = lane & 15;
  int fa[4][2], fb[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ra = 64 * wm + 16 * i + rl, rb = 64 * wn + 16 * i + rl;
      const int c = 4 * s + g;
      fa[i][s] = ra * 128 + 16 * (c ^ ((ra >> 1) & 7));
      fb[i][s] = GB_A_B + rb * 128 + 16 * (c ^ ((rb >> 1) & 7));
    }

  if (n_mine <= 0) return;
  // loads run two k-stages ahead in ONE sequence over (tile r, stage k) of this block
  int r_i = 0, k_i = 0, g_i = 0;  // next stage to issue and its global index
  Offs o_i = offsets(tile_of(0));
  auto issue_next = [&]() __attribute__((always_inline)) {
    if (r_i >= n_mine) return;
    issue(o_i, k_i, g_i);
    ++g_i;
    if (++k_i == nk) {
      k_i = 0;
      if (++r_i < n_mine) o_i = offsets(tile_of(r_i));
    }
  };
#pragma unroll
  for (int p = 0; p < GB_SLOTS - 1; ++p) issue_next();
  int gs = 0;  // global stage index of (tile r, k-step 0) = r * nk
  int nst = 0;  // stores issued by the previous tile's epilogue (0: unknown -> drain)
  for (int r = 0; r < n_mine; ++r) {
    const int lt = tile_of(r);
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt) {
      // loads allowed in flight: the one stage issued after this one, if any.  The first stage
      // of a tile also follows the previous tile's epilogue stores: drain everything.
      // younger than this stage's loads: the later stages already issued and, at a tile's
      // first stage, the previous epilogue's stores (16 or 32 per lane, never waited for here;
      // an edge tile's element-wise epilogue: drain)
      if (kt == 0 && r > 0) {
        if (nst == 32) enc_wait_vm<32>();
        else if (nst == 16) enc_wait_vm<16>();
        else if (nst == 8) enc_wait_vm<8>();
        else enc_wait_vm<0>();
      } else if (g_i <= gs + kt + GB_SLOTS - 2) {
        enc_wait_vm<0>();
      } else {
        enc_wait_vm<OPS * (GB_SLOTS - 2)>();
      }
      enc_lds_barrier();  // stage visible to all; every wave is done with the slot refilled next
      issue_next();
      const uint32_t sb = lds_addr(smem) + (uint32_t)(((gs + kt) % GB_SLOTS) * GB_STAGE_B);
      u32x4 av[2][4], bv[2][4];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          av[s][i] = lds_read128<0>(sb + fa[i][s]);
          bv[s][i] = lds_read128<0>(sb + fb[i][s]);
        }
      if constexpr (X3) {
        lds_wait<0>();
        bf16x8e ahi[4], alo[4], bhi[4], blo[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          reg_tie(av[0][i]);
          reg_tie(av[1][i]);
          reg_tie(bv[0][i]);
          reg_tie(bv[1][i]);
          split_bf16x8(av[0][i], av[1][i], ahi[i], alo[i]);
          split_bf16x8(bv[0][i], bv[1][i], bhi[i], blo[i]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bhi[j], ahi[i], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(blo[j], ahi[i], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bhi[j], alo[i], acc[i][j], 0, 0, 0);
          }
      } else if constexpr (X3I) {
        lds_wait<0>();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          reg_tie(av[0][i]);
          reg_tie(av[1][i]);
          reg_tie(bv[0][i]);
          reg_tie(bv[1][i]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const bf16x8e ah = __builtin_bit_cast(bf16x8e, av[0][i]), al = __builtin_bit_cast(bf16x8e, av[1][i]);
            const bf16x8e bh = __builtin_bit_cast(bf16x8e, bv[0][j]), bl = __builtin_bit_cast(bf16x8e, bv[1][j]);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, ah, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl, ah, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, al, acc[i][j], 0, 0, 0);
          }
      } else {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (s == 0) lds_wait<8>();
        else lds_wait<0>();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          reg_tie(av[s][i]);
          reg_tie(bv[s][i]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(  // D = W . A^T
                __builtin_bit_cast(bf16x8e, bv[s][j]), __builtin_bit_cast(bf16x8e, av[s][i]),
                acc[i][j], 0, 0, 0);
      }
      }
    }
    if (TT_GEXP_NOSTORE != 1)
      nst = gemm_wave_epilogue<!X3, ACT, BFO>(acc, (lt / n_tn) * GB_BM + 64 * wm, (lt % n_tn) * GB_BN + 64 * wn,
                               lane, M, N, bias, res, ldr, C, ldc, C16, ldc16, act,
                               lds_bias ? sbias : nullptr);
    else if (acc[0][0][0] == 123.456f && acc[3][3][3] == 1.5f) C[0] = acc[1][1][1];
    gs += nk;
  }
}

// Wide-tile variant of k_gemm_big: 256 x 256 tiles (8 waves as 4 (M) x 2 (N) of 64 x 128),
// 2-slot ring of 64-KB stages one stage ahead.  Per stage a CU moves 64 KB HBM/L2 -> LDS for
// 8.4 MFLOP (131 flop/B, vs 87 for 256 x 128), which is what bounds the persistent 256 x 128
// kernel at K = 384 (the MFMA pipes sat idle ~70 % waiting for its 48-KB stages).  Wave
// epilogue = two gemm_wave_epilogue calls (64-column halves).
#ifndef TT_GWEXP_NOEPI
#define TT_GWEXP_NOEPI 0  // timing-only (results WRONG): k_gemm_wide without its epilogue
#endif
template <int ACT, int BFO, bool X3I = false>
__global__ __launch_bounds__(512, 1) void k_gemm_wide(const uint16_t* __restrict__ A, int64_t lda,
                                                      const uint16_t* __restrict__ W, int64_t ldw,
                                                      const float* __restrict__ bias,
                                                      const float* __restrict__ res, int64_t ldr,
                                                      float* __restrict__ C, int64_t ldc,
                                                      uint16_t* __restrict__ C16, int64_t ldc16,
                                                      int M, int N, int K, int act) {
  constexpr int BM = 256, BN = 256, BK = 64, EPC = 8, SLOTS = 2;
  constexpr int A_B = BM * 128, STAGE_B = A_B + BN * 128;
  __shared__ __attribute__((aligned(16))) char smem[SLOTS * STAGE_B];
  __shared__ __attribute__((aligned(16))) float sbias[GB_MAXN];
  const int tid = threadIdx.x, lane = tid & 63;
  const bool lds_bias = bias && N <= GB_MAXN && ((uintptr_t)bias % 16) == 0;
  if (lds_bias)
    for (int e = tid; e < N; e += 512) sbias[e] = bias[e];  // visible after stage 0's barrier
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int n_tn = (N + BN - 1) / BN;
  const int ntiles = ((M + BM - 1) / BM) * n_tn;
  const int nk = K / BK;
  auto tile_of = [&](int r) { return enc_xcd_remap(blockIdx.x + r * gridDim.x, ntiles); };
  const int n_mine = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;

  // DMA: A and W = 32 pieces each of 8 rows x 128 B; wave w issues pieces w + 8 j (j < 4) of
  // both.  Row 8 (w + 8 j) + (lane >> 3): the swizzle (row >> 1) & 7 does not depend on j.
  const int drow = 8 * w + (lane >> 3);
  const int dchunk = ((lane & 7) ^ ((drow >> 1) & 7)) * EPC;
  struct Offs {
    int64_t a[4], w[4];
  };
  auto offsets = [&](int lt) __attribute__((always_inline)) {
    Offs o;
    const int m0 = (lt / n_tn) * BM, n0 = (lt % n_tn) * BN;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int am = m0 + drow + 64 * j;
      am = am < M ? am : M - 1;
      o.a[j] = (int64_t)am * lda + dchunk;
      int wr = n0 + drow + 64 * j;
      wr = wr < N ? wr : N - 1;  // rows past N: clamped loads, no stores
      o.w[j] = (int64_t)wr * ldw + dchunk;
    }
    return o;
  };
  auto issue = [&](const Offs& o, int kt, int gs) __attribute__((always_inline)) {
    char* st = smem + (gs & 1) * STAGE_B;
    const int64_t k0 = (int64_t)kt * BK, ka = k0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(A + o.a[j] + ka),
          (__attribute__((address_space(3))) void*)(st + 1024 * (w + 8 * j)), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(W + o.w[j] + k0),
          (__attribute__((address_space(3))) void*)(st + A_B + 1024 * (w + 8 * j)), 16, 0, 0);
  };

  // fragment rows 64 wm + 16 i + rl (A) / 128 wn + 16 j + rl (W): swizzle (rl >> 1) & 7 for
  // every i, j -> blocks are ds_read immediates (2048 B apart)
  const int g = lane >> 4, rl = lane & 15;
  uint32_t fa[2], fb[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int c = (4 * s + g) ^ ((rl >> 1) & 7);
    fa[s] = (64 * wm + rl) * 128 + 16 * c;
    fb[s] = A_B + (128 * wn + rl) * 128 + 16 * c;
  }

  if (n_mine <= 0) return;
  int r_i = 0, k_i = 0, g_i = 0;
  Offs o_i = offsets(tile_of(0));
  auto issue_next = [&]() __attribute__((always_inline)) {
    if (r_i >= n_mine) return;
    issue(o_i, k_i, g_i);
    ++g_i;
    if (++k_i == nk) {
      k_i = 0;
      if (++r_i < n_mine) o_i = offsets(tile_of(r_i));
    }
  };
  issue_next();
  int gs = 0, nst = 0;
  for (int r = 0; r < n_mine; ++r) {
    const int lt = tile_of(r);
    f32x4 acc[2][4][4];  // [column half][i][j]
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt) {
      // younger than this stage's loads: at a tile's first stage, the previous epilogue's
      // stores (nst per lane; an edge tile's element-wise epilogue: drain)
      if (kt == 0 && r > 0 && nst == 16) enc_wait_vm<16>();
      else if (kt == 0 && r > 0 && nst == 32) enc_wait_vm<32>();
      else enc_wait_vm<0>();
      enc_lds_barrier();  // stage visible to all; the other slot is free again
      issue_next();
      const uint32_t sb = lds_addr(smem) + (uint32_t)(((gs + kt) & 1) * STAGE_B);
      if constexpr (X3I) {
        // x3i: the stage's hi (k-half 0) and lo (k-half 1) of the same 32 k; A's 8 fragments
        // stay for the stage, W's 8 per 64-column half
        u32x4 av[2][4];
        const uint32_t pa0 = sb + fa[0], pa1 = sb + fa[1];
        av[0][0] = lds_read128<0>(pa0);
        av[0][1] = lds_read128<2048>(pa0);
        av[0][2] = lds_read128<4096>(pa0);
        av[0][3] = lds_read128<6144>(pa0);
        av[1][0] = lds_read128<0>(pa1);
        av[1][1] = lds_read128<2048>(pa1);
        av[1][2] = lds_read128<4096>(pa1);
        av[1][3] = lds_read128<6144>(pa1);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t pb0 = sb + fb[0] + 8192 * h, pb1 = sb + fb[1] + 8192 * h;
          u32x4 bh[4], bl[4];
          bh[0] = lds_read128<0>(pb0);
          bh[1] = lds_read128<2048>(pb0);
          bh[2] = lds_read128<4096>(pb0);
          bh[3] = lds_read128<6144>(pb0);
          bl[0] = lds_read128<0>(pb1);
          bl[1] = lds_read128<2048>(pb1);
          bl[2] = lds_read128<4096>(pb1);
          bl[3] = lds_read128<6144>(pb1);
          lds_wait<0>();
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            reg_tie(av[0][i]);
            reg_tie(av[1][i]);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            reg_tie(bh[j]);
            reg_tie(bl[j]);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const bf16x8e ah = __builtin_bit_cast(bf16x8e, av[0][i]), al = __builtin_bit_cast(bf16x8e, av[1][i]);
              const bf16x8e wh = __builtin_bit_cast(bf16x8e, bh[j]), wl = __builtin_bit_cast(bf16x8e, bl[j]);
              acc[h][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, ah, acc[h][i][j], 0, 0, 0);
              acc[h][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, ah, acc[h][i][j], 0, 0, 0);
              acc[h][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, al, acc[h][i][j], 0, 0, 0);
            }
        }
        continue;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const uint32_t pa = sb + fa[s], pb = sb + fb[s];
        u32x4 av[4], bv[8];
        av[0] = lds_read128<0>(pa);
        av[1] = lds_read128<2048>(pa);
        av[2] = lds_read128<4096>(pa);
        av[3] = lds_read128<6144>(pa);
        bv[0] = lds_read128<0>(pb);
        bv[1] = lds_read128<2048>(pb);
        bv[2] = lds_read128<4096>(pb);
        bv[3] = lds_read128<6144>(pb);
        bv[4] = lds_read128<8192>(pb);
        bv[5] = lds_read128<10240>(pb);
        bv[6] = lds_read128<12288>(pb);
        bv[7] = lds_read128<14336>(pb);
        lds_wait<4>();
#pragma unroll
        for (int i = 0; i < 4; ++i) reg_tie(av[i]);
#pragma unroll
        for (int j = 0; j < 4; ++j) reg_tie(bv[j]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[0][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8e, bv[j]), __builtin_bit_cast(bf16x8e, av[i]),
                acc[0][i][j], 0, 0, 0);
        lds_wait<0>();
#pragma unroll
        for (int j = 4; j < 8; ++j) reg_tie(bv[j]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[1][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8e, bv[4 + j]), __builtin_bit_cast(bf16x8e, av[i]),
                acc[1][i][j], 0, 0, 0);
      }
    }
    if (TT_GWEXP_NOEPI) {  // timing-only: every accumulator live, nothing stored
      float t = 0.0f;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) t += (acc[h][i][j][0] + acc[h][i][j][1]) + (acc[h][i][j][2] + acc[h][i][j][3]);
      if (t == 1.2345f) C16[0] = 1;
      nst = 0;
      gs += nk;
      continue;
    }
    const int m0 = (lt / n_tn) * BM + 64 * wm, n0 = (lt % n_tn) * BN + 128 * wn;
    nst = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = gemm_wave_epilogue<true, ACT, BFO>(acc[h], m0, n0 + 64 * h, lane, M, N, bias,
                                                       res, ldr, C, ldc, C16, ldc16, act,
                                                       lds_bias ? sbias : nullptr);
      nst = (h == 0 || (c > 0 && nst > 0)) ? nst + c : 0;
    }
    gs += nk;
  }
}

// Fused GEMM + LayerNorm for the two H-wide GEMMs of a BERT layer (bf16 path):
//   BertSelfOutput / BertOutput: x = LayerNorm(A . W^T + bias + x)      (A = ctx, K = H; or
//   A = GELU(ffn), K = I).  One block owns whole 384-wide rows, so the LayerNorm statistics
// are reduced in LDS inside the epilogue and the pre-LayerNorm sum never reaches HBM: per
// token row this writes x (f32, the residual stream) and its bf16 copy once, instead of a GEMM
// writing y and a LayerNorm pass re-reading it (≈3.8 KB/row and one launch saved per call).
// Persistent blocks (one per CU, 8 waves as 2 (M) x 4 (N), wave tile 64 x 96 = 4 x 6 MFMA
// blocks), 128 x 384 tiles, k-stages of 64: the A tile (128 rows x 128 B, from HBM) streams
// through a 3-slot LDS ring issued two stages ahead, W (384 rows x 128 B, L2-resident) through
// a 2-slot ring one stage ahead; both run across tiles, so the next tile's first stages are in
// flight during the epilogue.
// The MFMA computes D = W . A^T as k_gemm_big (lane (g, rl) of block (i, j) holds row
// 16 i + rl, columns 16 j + 4 g .. + 3).  In place: x is read (residual) before it is
// overwritten, by the block that owns the rows.
constexpr int GL_H = 384, GL_NJ = 6, GL_ASLOTS = 3, GL_WSLOTS = 2;
constexpr int GL_W_B = GL_H * 128;
// timing-only experiment switches (results WRONG when set), tools/exp_filter.sh FILE=tt_encoder
// + tools/exp_gemm.sh.  Measured at M = 370761 (K = 384 / 1536): base 471 / 752 us, no W
// stream after the prologue 439 / 669, no epilogue 111 / 504 -> the LayerNorm epilogue (its
// residual reads and x / x16 writes, 1.42 GB at K = 384) is what the fused kernel waits on.
#ifndef TT_GL_NT
#define TT_GL_NT 0  // A (read once: a block owns whole rows) non-temporal: A/B no change
#endif
#ifndef TT_GLEXP_NOW
#define TT_GLEXP_NOW 0  // W streamed for the first stages only
#endif
#ifndef TT_GLEXP_NOEPI
#define TT_GLEXP_NOEPI 0  // no residual loads / LayerNorm / stores
#endif  // vector-memory stores per lane in a full tile
TT_CHECK_EXP(TT_GEXP_NOSTORE || TT_GWEXP_NOEPI || TT_GLEXP_NOW || TT_GLEXP_NOEPI || TT_GL_NT,
             "TT_G*EXP_* / TT_GL_NT (results wrong or untested)");

// BM = 128 (8 waves as 2 (M) x 4 (N) of 64 x 96), 96 (2 x 4 of 48 x 96) or 80 (1 (M) x 8 (N)
// of 80 x 48): a batch of ~18k token rows is 144 tiles of 128 on 256 CUs, 192 of 96, 230 of 80
// -- tt_gemm_ln_bf16 picks by rounds x tile cost.  The LayerNorm statistics are reduced in a
// layout-independent order (each row's 384 columns as 8 partial sums of 48 columns, each
// partial summed over its lanes, the 8 combined by a fixed tree), so a row's bits do not
// depend on the tile height the batch size selected.
// SPL: the x3 encoder -- A and W are x3i interleaved rows (K = 2 x the product's K; per 32 k
// the three split-bf16 products, as k_gemm<X3I>) and x's bf16 copy is written interleaved too.
template <int BM, bool SPL = false>
__global__ __launch_bounds__(512, 1) void k_gemm_ln(const uint16_t* __restrict__ A, int64_t lda,
                                                    const uint16_t* __restrict__ W, int64_t ldw,
                                                    const float* __restrict__ bias,
                                                    const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, float eps,
                                                    float* __restrict__ X, int64_t ldx,
                                                    uint16_t* __restrict__ X16, int64_t ldx16,
                                                    int M, int K, int st16) {
  static_assert(BM == 128 || BM == 96 || BM == 80, "k_gemm_ln: BM");
  constexpr int WM_N = BM == 80 ? 1 : 2;     // waves along M
  constexpr int WN_N = 8 / WM_N;             // waves along N
  constexpr int NJ = (GL_H / 16) / WN_N;     // 16-column blocks per wave (6 or 3)
  constexpr int HJ = 3;                      // blocks per 48-column partial
  constexpr int NP = NJ / HJ;                // partials per wave (2 or 1)
  constexpr int BK = 64, EPC = 8, WR = BM / WM_N, MI = WR / 16;  // rows per wave / 16-row blocks
  constexpr int A_B = BM * 128, WBASE = GL_ASLOTS * A_B;
  constexpr int APIECES = BM / 8;            // 1-KB A pieces per stage (10, 12 or 16)
  // stores per lane of a full tile's epilogue (vmcnt holds at most 63: a stronger wait is safe)
  constexpr int STORES = MI * NJ * (SPL ? 3 : 2) > 63 ? 63 : MI * NJ * (SPL ? 3 : 2);
  __shared__ __attribute__((aligned(16))) char smem[WBASE + GL_WSLOTS * GL_W_B];
  __shared__ float red[2][8][BM];  // [mean | var pass][48-column partial][tile row]
  __shared__ __attribute__((aligned(16))) float prm[3][GL_H];  // bias, gamma, beta
  const int tid = threadIdx.x, lane = tid & 63;
  for (int e = tid; e < GL_H; e += 512) {
    prm[0][e] = bias[e];
    prm[1][e] = gamma[e];
    prm[2][e] = beta[e];
  }  // visible after the first stage's barrier
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WN_N, wn = w % WN_N;
  const int ntiles = (M + BM - 1) / BM;
  const int nk = K / BK;
  auto tile_of = [&](int r) { return enc_xcd_remap(blockIdx.x + r * gridDim.x, ntiles); };
  const int n_mine = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  if (n_mine <= 0) return;

  // DMA: A = APIECES pieces of 8 rows x 128 B, W = 48 pieces; wave w issues A pieces w + 8j
  // (j < 2; pieces past APIECES fold back onto earlier ones, written twice with the same
  // bytes, so every wave issues 2 and the vmcnt accounting is uniform) and W pieces w + 8j
  // (j < 6); chunk swizzle as k_gemm.
  // W piece w + 8j = rows 64 j + 8 w + (lane >> 3): a per-lane 32-bit offset (the swizzle
  // (row >> 1) & 7 does not depend on j) plus the uniform base W + 64 j ldw
  const int w_row0 = 8 * w + (lane >> 3);
  const int w_lane = w_row0 * (int)ldw + ((lane & 7) ^ ((w_row0 >> 1) & 7)) * EPC;
  auto apiece = [&](int j) {
    const int pc = w + 8 * j;
    return pc < APIECES ? pc : pc - (16 - APIECES);
  };
  auto a_offsets = [&](int lt, int64_t (&ao)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = 8 * apiece(j) + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      int am = lt * BM + row;
      am = am < M ? am : M - 1;
      ao[j] = (int64_t)am * lda + c * EPC;
    }
  };
  auto issue_a = [&](const int64_t (&ao)[2], int kt, int t) __attribute__((always_inline)) {
    char* st = smem + (t % GL_ASLOTS) * A_B;
    const int64_t k0 = (int64_t)kt * BK, ka = k0;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(A + ao[j] + ka),
          (__attribute__((address_space(3))) void*)(st + 1024 * apiece(j)), 16, 0,
          TT_GL_NT ? 2 : 0);
  };
  auto issue_w = [&](int kt, int t) __attribute__((always_inline)) {
    char* st = smem + WBASE + (t % GL_WSLOTS) * GL_W_B;
    const int64_t k0 = (int64_t)kt * BK;
#pragma unroll
    for (int j = 0; j < GL_NJ; ++j)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(W + (k0 + (int64_t)(64 * j) * ldw) + w_lane),
          (__attribute__((address_space(3))) void*)(st + 1024 * (w + 8 * j)), 16, 0, 0);
  };

  // fragment rows WR wm + 16 i + rl (A) / 16 NJ wn + 16 j + rl (W): the swizzle (row >> 1) & 7
  // = (rl >> 1) & 7 is the same for every i, j, so block i / j is 2048 B further
  const int g = lane >> 4, rl = lane & 15;
  uint32_t fa[2], fb[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int c = (4 * s + g) ^ ((rl >> 1) & 7);
    fa[s] = (WR * wm + rl) * 128 + 16 * c;
    fb[s] = (16 * NJ * wn + rl) * 128 + 16 * c;
  }

  // the block's stages t = r * nk + kt in one sequence: A(t) issued at stage t - 2, W(t) at
  // stage t - 1, in the order W(t + 1), A(t + 2), so waiting for W(t) leaves exactly A(t + 1)'s
  // two pieces younger
  const int nstages = n_mine * nk;
  int ra_i = 0, ka_i = 0, ta_i = 0;  // next A stage to issue
  int64_t ao_i[2];
  a_offsets(tile_of(0), ao_i);
  auto issue_next_a = [&]() __attribute__((always_inline)) {
    if (ta_i >= nstages) return;
    issue_a(ao_i, ka_i, ta_i);
    ++ta_i;
    if (++ka_i == nk) {
      ka_i = 0;
      if (++ra_i < n_mine) a_offsets(tile_of(ra_i), ao_i);
    }
  };
  issue_next_a();
  issue_w(0, 0);
  issue_next_a();
  int gs = 0;
  bool prev_full = true;
  const float inv_h = 1.0f / (float)GL_H;
  for (int r = 0; r < n_mine; ++r) {
    const int m0 = tile_of(r) * BM;
    f32x4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt) {
      // younger than this stage's W pieces: A(t + 1) (2 per lane, if issued) and, at a tile's
      // first stage, the previous epilogue's residual loads and STORES stores (a ragged
      // tile: drain all)
      const int t = gs + kt;
      if (kt == 0 && r > 0) {
        if (prev_full) enc_wait_vm<STORES>();
        else enc_wait_vm<0>();
      } else if (ta_i > t + 1) {
        enc_wait_vm<2>();
      } else {
        enc_wait_vm<0>();
      }
      enc_lds_barrier();  // stage t visible to all; slots of stage t - 1 are free again
      if (t + 1 < nstages && (!TT_GLEXP_NOW || t + 1 < GL_WSLOTS))
        issue_w(kt + 1 < nk ? kt + 1 : 0, t + 1);
      issue_next_a();
      const uint32_t sa = lds_addr(smem) + (uint32_t)((t % GL_ASLOTS) * A_B);
      const uint32_t sw = lds_addr(smem) + (uint32_t)(WBASE + (t % GL_WSLOTS) * GL_W_B);
      // fragment reads of both k-halves issued up front; s = 1 lands under s = 0's MFMAs
      u32x4 av[2][MI], bv[2][NJ];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const uint32_t pa = sa + fa[s], pb = sw + fb[s];
#pragma unroll
        for (int i = 0; i < MI; ++i) av[s][i] = lds_read128<0>(pa + 2048 * i);
#pragma unroll
        for (int j = 0; j < NJ; ++j) bv[s][j] = lds_read128<0>(pb + 2048 * j);
      }
      if constexpr (SPL) {  // x3i: hi (k-half 0) and lo (k-half 1) of the same 32 k
        lds_wait<0>();
#pragma unroll
        for (int s = 0; s < 2; ++s) {
#pragma unroll
          for (int i = 0; i < MI; ++i) reg_tie(av[s][i]);
#pragma unroll
          for (int j = 0; j < NJ; ++j) reg_tie(bv[s][j]);
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            const bf16x8e ah = __builtin_bit_cast(bf16x8e, av[0][i]), al = __builtin_bit_cast(bf16x8e, av[1][i]);
            const bf16x8e wh = __builtin_bit_cast(bf16x8e, bv[0][j]), wl = __builtin_bit_cast(bf16x8e, bv[1][j]);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, ah, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, ah, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, al, acc[i][j], 0, 0, 0);
          }
      } else {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (s == 0) lds_wait<(MI + NJ) < 15 ? MI + NJ : 15>();
        else lds_wait<0>();
#pragma unroll
        for (int i = 0; i < MI; ++i) reg_tie(av[s][i]);
#pragma unroll
        for (int j = 0; j < NJ; ++j) reg_tie(bv[s][j]);
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int i = 0; i < MI; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8e, bv[s][j]), __builtin_bit_cast(bf16x8e, av[s][i]),
                acc[i][j], 0, 0, 0);
      }
      }
    }
    gs += nk;

    if (TT_GLEXP_NOEPI) {  // keep every accumulator live (no dead-code MFMAs), store nothing
      float t = 0.0f;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) t += (acc[i][j][0] + acc[i][j][1]) + (acc[i][j][2] + acc[i][j][3]);
      if (t == 1.2345f) X[0] = t;
      prev_full = false;
      continue;
    }
    // ---- epilogue: y = acc + bias + x ; x = LayerNorm(y) (biased variance, two passes).
    // Residual rows are loaded one 16-row block ahead (NJ x 16 B per lane in flight while the
    // previous block is summed); bias / gamma / beta come from LDS.  Statistics: per row, 8
    // partials of 48 columns (a wave's HJ blocks, lane-summed), combined by a fixed tree.
    const bool full = m0 + BM <= M;
    const int nw0 = 16 * NJ * wn + 4 * g;
    const float* xr0 = X + (int64_t)(m0 + WR * wm + rl) * ldx + nw0;
    auto xrow = [&](int i) __attribute__((always_inline)) {
      const int m = m0 + WR * wm + 16 * i + rl;
      return X + (int64_t)(m < M ? m : M - 1) * ldx + nw0;  // rows past M: clamped reads
    };
    auto tree8 = [](const float* r) __attribute__((always_inline)) {
      return ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    };
    float mean[MI], rstd[MI];
    {
      f32x4 rv[2][NJ];
      const float* p0 = full ? xr0 : xrow(0);
#pragma unroll
      for (int j = 0; j < NJ; ++j) rv[0][j] = *(const f32x4*)(p0 + 16 * j);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        if (i + 1 < MI) {
          const float* p1 = full ? xr0 + (int64_t)(16 * (i + 1)) * ldx : xrow(i + 1);
#pragma unroll
          for (int j = 0; j < NJ; ++j) rv[(i + 1) & 1][j] = *(const f32x4*)(p1 + 16 * j);
        }
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          float sp = 0.0f;
#pragma unroll
          for (int jj = 0; jj < HJ; ++jj) {
            const int j = HJ * p + jj;
            acc[i][j] += rv[i & 1][j] + *(const f32x4*)(&prm[0][nw0 + 16 * j]);
            sp += (acc[i][j][0] + acc[i][j][1]) + (acc[i][j][2] + acc[i][j][3]);
          }
          sp += __shfl_xor(sp, 16, 64);
          sp += __shfl_xor(sp, 32, 64);
          if (g == 0) red[0][NP * wn + p][WR * wm + 16 * i + rl] = sp;
        }
      }
    }
    enc_lds_barrier();
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = WR * wm + 16 * i + rl;
      float rr[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) rr[c] = red[0][c][row];
      mean[i] = tree8(rr) * inv_h;
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        float q = 0.0f;
#pragma unroll
        for (int jj = 0; jj < HJ; ++jj)
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float d = acc[i][HJ * p + jj][u] - mean[i];
            q = fmaf(d, d, q);
          }
        q += __shfl_xor(q, 16, 64);
        q += __shfl_xor(q, 32, 64);
        if (g == 0) red[1][NP * wn + p][row] = q;
      }
    }
    enc_lds_barrier();
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = WR * wm + 16 * i + rl;
      float rr[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) rr[c] = red[1][c][row];
      rstd[i] = 1.0f / sqrtf(tree8(rr) * inv_h + eps);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = nw0 + 16 * j;
      const f32x4 gm = *(const f32x4*)(&prm[1][n]), bt = *(const f32x4*)(&prm[2][n]);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[i][j][u] = (acc[i][j][u] - mean[i]) * rstd[i] * gm[u] + bt[u];
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int64_t m = m0 + WR * wm + 16 * i + rl;
      if (!full && m >= M) continue;
      // x16: blocks j = 2 jp, 2 jp + 1 re-paired by v_permlane16_swap so each lane holds 8
      // consecutive columns -> 16-B stores (hi and lo each for x3i), a full 128-B x3i line per
      // row and block pair.  Single blocks' 8-B stores (32-B pieces of a line from 4 separate
      // instructions) made the x16 copy cost as much as the rest of the epilogue: Wo+LN at
      // 370k rows 709 -> 449 us without them, the f32 x stores ~free.
      int jbeg = 0;
      if (st16) {
#pragma unroll
        for (int jp = 0; jp < NJ / 2; ++jp) {
          uint32_t ph[2][2], pw[2][2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const f32x4 y = acc[i][2 * jp + h];
            ph[h][0] = pack_bf16_hw(y[0], y[1]);
            ph[h][1] = pack_bf16_hw(y[2], y[3]);
            if constexpr (SPL) {
              pw[h][0] = pack_bf16_hw(y[0] - __uint_as_float(ph[h][0] << 16),
                                      y[1] - __uint_as_float(ph[h][0] & 0xffff0000u));
              pw[h][1] = pack_bf16_hw(y[2] - __uint_as_float(ph[h][1] << 16),
                                      y[3] - __uint_as_float(ph[h][1] & 0xffff0000u));
            }
          }
          const auto s0 = __builtin_amdgcn_permlane16_swap(ph[0][0], ph[1][0], false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(ph[0][1], ph[1][1], false, false);
          const int n = 16 * NJ * wn + 32 * jp + 16 * (g & 1) + 8 * (g >> 1);
          if constexpr (SPL) {
            const auto t0 = __builtin_amdgcn_permlane16_swap(pw[0][0], pw[1][0], false, false);
            const auto t1 = __builtin_amdgcn_permlane16_swap(pw[0][1], pw[1][1], false, false);
            uint16_t* o = X16 + m * ldx16 + x3i_col(n);
            *(u32x4*)o = u32x4{s0[0], s1[0], s0[1], s1[1]};
            *(u32x4*)(o + 32) = u32x4{t0[0], t1[0], t0[1], t1[1]};
          } else {
            *(u32x4*)(X16 + m * ldx16 + n) = u32x4{s0[0], s1[0], s0[1], s1[1]};
          }
        }
        jbeg = NJ / 2 * 2;
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) *(f32x4*)(X + m * ldx + nw0 + 16 * j) = acc[i][j];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (j < jbeg) continue;
        const int n = nw0 + 16 * j;
        const uint2 hv = uint2{pack_bf16_hw(acc[i][j][0], acc[i][j][1]),
                               pack_bf16_hw(acc[i][j][2], acc[i][j][3])};
        if constexpr (SPL) {
          uint16_t* o = X16 + m * ldx16 + x3i_col(n);
          *(uint2*)o = hv;
          *(uint2*)(o + 32) =
              uint2{pack_bf16_hw(acc[i][j][0] - __uint_as_float(hv.x << 16),
                                 acc[i][j][1] - __uint_as_float(hv.x & 0xffff0000u)),
                    pack_bf16_hw(acc[i][j][2] - __uint_as_float(hv.y << 16),
                                 acc[i][j][3] - __uint_as_float(hv.y & 0xffff0000u))};
        } else {
          *(uint2*)(X16 + m * ldx16 + n) = hv;
        }
      }
    }
    prev_full = full;
  }
}

// LayerNorm over rows of width H (<= 1024): wave per row.  torch.nn.LayerNorm semantics
// (biased variance, (x - mean) / sqrt(var + eps) * gamma + beta).
__global__ __launch_bounds__(256) void k_layernorm(const float* __restrict__ x, int64_t ldx,
                                                   const float* __restrict__ gamma,
                                                   const float* __restrict__ beta, float eps,
                                                   float* __restrict__ y, int64_t ldy,
                                                   uint16_t* __restrict__ y16, int64_t ldy16,
                                                   int64_t rows, int H) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + w; r < rows; r += (int64_t)gridDim.x * 4) {
    const float* xr = x + r * ldx;
    float v[16];
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int e = lane + 64 * i;
      v[i] = e < H ? xr[e] : 0.0f;
      s += v[i];
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mean = s / (float)H;
    float q = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int e = lane + 64 * i;
      const float d = e < H ? v[i] - mean : 0.0f;
      q = fmaf(d, d, q);
    }
    for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
    const float rstd = 1.0f / sqrtf(q / (float)H + eps);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int e = lane + 64 * i;
      if (e < H) {
        const float o = (v[i] - mean) * rstd * gamma[e] + beta[e];
        y[r * ldy + e] = o;
        if (y16) y16[r * ldy16 + e] = f32_to_bf16_rne(o);
      }
    }
  }
}

// BertEmbeddings: (word[id] + token_type[0]) + position[t - start] -> LayerNorm.
__global__ __launch_bounds__(256) void k_embed_ln(const int32_t* __restrict__ ids,
                                                  const int32_t* __restrict__ cu, int n_seq,
                                                  int64_t T, const float* __restrict__ word,
                                                  int vocab, const float* __restrict__ pos,
                                                  const float* __restrict__ type0,
                                                  const float* __restrict__ gamma,
                                                  const float* __restrict__ beta, float eps,
                                                  float* __restrict__ y, uint16_t* __restrict__ y16,
                                                  int H, int split16) {
  // split16: y16 rows are x3i interleaved (ld 2H) for the x3 encoder, else bf16 copies (ld H)
  // blocks (sequence, chunk of 4 tokens), wave per token (the position is t - cu[seq]; a
  // per-token binary search over cu was 13 dependent loads per token at 5k sequences).  Was a
  // block per sequence whose waves walked its tokens: at configs[1]'s 256 sequences that is
  // ~18 dependent gather round trips per wave (129 us per batch); the loop below still covers
  // every token when gridDim.y * 4 < a sequence's length.
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t t0 = cu[blockIdx.x], t1 = cu[blockIdx.x + 1];
  for (int64_t t = t0 + 4 * (int64_t)blockIdx.y + w; t < t1; t += 4 * (int64_t)gridDim.y) {
    const int p = (int)(t - t0);
    int id = ids[t];
    id = (id >= 0 && id < vocab) ? id : 0;
    const float* wr = word + (int64_t)id * H;
    const float* pr = pos + (int64_t)p * H;
    float v[16];
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int e = lane + 64 * i;
      v[i] = e < H ? (wr[e] + type0[e]) + pr[e] : 0.0f;
      s += v[i];
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mean = s / (float)H;
    float q = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int e = lane + 64 * i;
      const float d = e < H ? v[i] - mean : 0.0f;
      q = fmaf(d, d, q);
    }
    for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
    const float rstd = 1.0f / sqrtf(q / (float)H + eps);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int e = lane + 64 * i;
      if (e < H) {
        const float o = (v[i] - mean) * rstd * gamma[e] + beta[e];
        y[t * H + e] = o;
        if (y16) {
          const uint16_t hv = f32_to_bf16_rne(o);
          if (split16) {
            uint16_t* d = y16 + t * 2 * H + x3i_col(e);
            d[0] = hv;
            d[32] = f32_to_bf16_rne(o - __uint_as_float((uint32_t)hv << 16));
          } else {
            y16[t * H + e] = hv;
          }
        }
      }
    }
  }
}

// k_embed_ln for H % 4 == 0, H <= 256 NV: a wave embeds FOUR tokens of its sequence at once
// with 16-B loads and stores (all 4 x NV row gathers in flight after the 4 id loads), blocks of
// (sequence, 16 tokens).  The one-token-per-wave form waited 72% of its wave cycles on the
// dependent id -> row gather (727 us per 370k-token Mode A step).  Per element the same
// (word + type) + position sum; the LayerNorm statistics reduce 4 contiguous elements per lane
// and then across lanes.  x3i output: a lane's 4 columns lie in one 32-column block.
template <int NV>
__global__ __launch_bounds__(256) void k_embed_ln4(const int32_t* __restrict__ ids,
                                                   const int32_t* __restrict__ cu, int n_seq,
                                                   int64_t T, const float* __restrict__ word,
                                                   int vocab, const float* __restrict__ pos,
                                                   const float* __restrict__ type0,
                                                   const float* __restrict__ gamma,
                                                   const float* __restrict__ beta, float eps,
                                                   float* __restrict__ y, uint16_t* __restrict__ y16,
                                                   int H, int split16) {
  constexpr int TPW = 4;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t t0 = cu[blockIdx.x], t1 = cu[blockIdx.x + 1];
  const int H4 = H >> 2;
  const float inv_h = 1.0f / (float)H;
  for (int64_t tb = t0 + (int64_t)TPW * (4 * (int64_t)blockIdx.y + w); tb < t1;
       tb += (int64_t)TPW * 4 * gridDim.y) {
    int id[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int v = tb + j < t1 ? ids[tb + j] : 0;
      id[j] = (v >= 0 && v < vocab) ? v : 0;
    }
    f32x4 v[TPW][NV];
    float sm[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int p = tb + j < t1 ? (int)(tb + j - t0) : 0;
      const float* wr = word + (int64_t)id[j] * H;
      const float* pr = pos + (int64_t)p * H;
      sm[j] = 0.0f;
#pragma unroll
      for (int c = 0; c < NV; ++c) {
        const int e4 = lane + 64 * c;
        if (e4 < H4) {
          const f32x4 wv = *(const f32x4*)(wr + 4 * e4), tv = *(const f32x4*)(type0 + 4 * e4);
          const f32x4 pv = *(const f32x4*)(pr + 4 * e4);
          v[j][c] = (wv + tv) + pv;
          sm[j] += (v[j][c][0] + v[j][c][1]) + (v[j][c][2] + v[j][c][3]);
        } else {
          v[j][c] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
#pragma unroll
    for (int j = 0; j < TPW; ++j)
      for (int o = 32; o > 0; o >>= 1) sm[j] += __shfl_xor(sm[j], o, 64);
    float q[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const float mean = sm[j] * inv_h;
      q[j] = 0.0f;
#pragma unroll
      for (int c = 0; c < NV; ++c)
        if (lane + 64 * c < H4)
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float d = v[j][c][u] - mean;
            q[j] = fmaf(d, d, q[j]);
          }
    }
#pragma unroll
    for (int j = 0; j < TPW; ++j)
      for (int o = 32; o > 0; o >>= 1) q[j] += __shfl_xor(q[j], o, 64);
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int64_t t = tb + j;
      if (t >= t1) continue;
      const float mean = sm[j] * inv_h;
      const float rstd = 1.0f / sqrtf(q[j] * inv_h + eps);
#pragma unroll
      for (int c = 0; c < NV; ++c) {
        const int e4 = lane + 64 * c;
        if (e4 >= H4) continue;
        const f32x4 gm = *(const f32x4*)(gamma + 4 * e4), bt = *(const f32x4*)(beta + 4 * e4);
        f32x4 o;
#pragma unroll
        for (int u = 0; u < 4; ++u) o[u] = (v[j][c][u] - mean) * rstd * gm[u] + bt[u];
        *(f32x4*)(y + t * H + 4 * e4) = o;
        if (y16) {
          const uint2 hv = uint2{pack_bf16_hw(o[0], o[1]), pack_bf16_hw(o[2], o[3])};
          if (split16) {
            uint16_t* d = y16 + t * 2 * H + x3i_col(4 * e4);
            *(uint2*)d = hv;
            *(uint2*)(d + 32) = uint2{pack_bf16_hw(o[0] - __uint_as_float(hv.x << 16),
                                                   o[1] - __uint_as_float(hv.x & 0xffff0000u)),
                                      pack_bf16_hw(o[2] - __uint_as_float(hv.y << 16),
                                                   o[3] - __uint_as_float(hv.y & 0xffff0000u))};
          } else {
            *(uint2*)(y16 + t * H + 4 * e4) = hv;
          }
        }
      }
    }
  }
}

// host: the embedding LayerNorm launch (k_embed_ln4 when H % 4 == 0 and H <= 1024)
static int embed_ln_launch(const tt_bert_model* m, const int32_t* ids, const int32_t* cu,
                           int n_seq, int64_t T, int max_len, float* x, uint16_t* x16, int H,
                           int split16, hipStream_t st) {
  if (H % 4 == 0 && H <= 1024 && ((uintptr_t)m->word_emb % 16) == 0 &&
      ((uintptr_t)m->pos_emb % 16) == 0 && ((uintptr_t)m->type_emb % 16) == 0 &&
      ((uintptr_t)m->emb_ln_g % 16) == 0 && ((uintptr_t)m->emb_ln_b % 16) == 0 &&
      ((uintptr_t)x % 16) == 0 && ((uintptr_t)x16 % 8) == 0) {
    const unsigned chunks = (unsigned)(max_len > 16 ? (max_len + 15) / 16 : 1);
    auto kern = H <= 256 ? k_embed_ln4<1> : H <= 512 ? k_embed_ln4<2> : k_embed_ln4<4>;
    hipLaunchKernelGGL(kern, dim3((unsigned)n_seq, chunks), dim3(256), 0, st, ids, cu, n_seq, T,
                       m->word_emb, m->vocab, m->pos_emb, m->type_emb, m->emb_ln_g, m->emb_ln_b,
                       m->ln_eps, x, x16, H, split16);
    return check_launch("k_embed_ln4");
  }
  const unsigned chunks = (unsigned)(max_len > 4 ? (max_len + 3) / 4 : 1);
  hipLaunchKernelGGL(k_embed_ln, dim3((unsigned)n_seq, chunks), dim3(256), 0, st, ids, cu, n_seq,
                     T, m->word_emb, m->vocab, m->pos_emb, m->type_emb, m->emb_ln_g, m->emb_ln_b,
                     m->ln_eps, x, x16, H, split16);
  return check_launch("k_embed_ln");
}

// Multi-head self-attention over packed sequences.  qkv: [T, 3H] (Q | K | V, head h at
// columns h*DH within each third).  Block per (sequence, head); K and V of the head live in
// LDS; thread = query row.  softmax(q.k / sqrt(DH)) . v, keys restricted to the sequence.
template <int DH>
__global__ __launch_bounds__(128) void k_attn(const float* __restrict__ qkv, int64_t ldq,
                                              const int32_t* __restrict__ cu, int H, int heads,
                                              float scale, float* __restrict__ out,
                                              int64_t ldo, uint16_t* __restrict__ out16) {
  extern __shared__ float kv[];  // [L][DH] keys then [L][DH] values
  const int sq = blockIdx.x / heads, h = blockIdx.x % heads;
  const int t0 = cu[sq], L = cu[sq + 1] - t0;
  float* ks = kv;
  float* vs = kv + (int64_t)L * DH;
  for (int e = threadIdx.x; e < L * DH; e += blockDim.x) {
    const int j = e / DH, c = e % DH;
    const float* row = qkv + (int64_t)(t0 + j) * ldq;
    ks[e] = row[H + h * DH + c];
    vs[e] = row[2 * H + h * DH + c];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < L; i += blockDim.x) {
    const float* qr = qkv + (int64_t)(t0 + i) * ldq + h * DH;
    float q[DH];
#pragma unroll
    for (int c = 0; c < DH; ++c) q[c] = qr[c];
    float m = -__builtin_huge_valf();
    for (int j = 0; j < L; ++j) {
      const float* kr = ks + j * DH;
      float s = 0.0f;
#pragma unroll
      for (int c = 0; c < DH; ++c) s = fmaf(q[c], kr[c], s);
      m = fmaxf(m, s * scale);
    }
    float acc[DH];
#pragma unroll
    for (int c = 0; c < DH; ++c) acc[c] = 0.0f;
    float l = 0.0f;
    for (int j = 0; j < L; ++j) {
      const float* kr = ks + j * DH;
      float s = 0.0f;
#pragma unroll
      for (int c = 0; c < DH; ++c) s = fmaf(q[c], kr[c], s);
      const float p = expf(s * scale - m);
      l += p;
      const float* vr = vs + j * DH;
#pragma unroll
      for (int c = 0; c < DH; ++c) acc[c] = fmaf(p, vr[c], acc[c]);
    }
    const float inv = 1.0f / l;
    float* orow = out + (int64_t)(t0 + i) * ldo + h * DH;
#pragma unroll
    for (int c = 0; c < DH; ++c) {
      const float o = acc[c] * inv;
      orow[c] = o;
      if (out16) out16[(int64_t)(t0 + i) * ldo + h * DH + c] = f32_to_bf16_rne(o);
    }
  }
}

// MFMA attention for head dim 32: block (4 waves) per (sequence, head), wave per 16-query tile.
// Computes S^T = K Q^T (keys x queries) so that, in the MFMA C layout, lane (g = l >> 4,
// q = l & 15) holds the scores of query q for keys 4g..4g+3 of each 16-key block -- exactly
// the B-operand layout of the next product O^T = V^T P^T.  The probabilities never leave
// registers; softmax statistics are per column (query) = a lane, reduced over g with two
// cross-lane xors.  Keys stream in chunks of 32 with online (rescaled) softmax.
//   BF = true : v_mfma_f32_16x16x32_bf16 (K, Q, V, P in bf16, f32 accumulate/softmax).
//   BF = false: v_mfma_f32_16x16x4_f32 (everything f32: the parity path).
//   X3 (BF = false): the f32 data path, each product on split-bf16 MFMA (split_bf16x8: hi.hi +
//        lo.hi + hi.lo, 3 v_mfma_f32_16x16x32_bf16 per 8 f32 MFMAs); the 8 k-slots of a lane are
//        the f32 path's two 4-wide groups (dims 4g.., 16 + 4g.. / keys kc + 4g.., kc + 16 + 4g..).
// LDS: K [Lk][32] (rows padded to 144 B f32 / 80 B bf16) and V^T [32][vst] (vst = 128k + 4 f32
// / 128k + 8 bf16 elements): both fragment reads are bank-conflict-free.
template <bool BF, typename TI, bool X3 = false>
__global__ __launch_bounds__(256) void k_attn32_mfma(const TI* __restrict__ qkv, int64_t ldq,
                                                     const int32_t* __restrict__ cu, int H,
                                                     int heads, float scale,
                                                     float* __restrict__ out, int64_t ldo,
                                                     uint16_t* __restrict__ out16,
                                                     int split16) {
  // split16 (X3 only, out == NULL): out16 rows [hi | lo] (ldo = 2H, lo at column H + c), the
  // A operand of a Wo GEMM over [hi | lo] planes
  constexpr int DH = 32;
  constexpr int ES = BF ? 2 : 4;
  constexpr int KROW = DH * ES + 16;
  extern __shared__ __attribute__((aligned(16))) char sm[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, ql = lane & 15;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);  // a sequence's heads on one XCD (see below)
  const int sq = lb / heads, h = lb % heads;
  const int t0 = cu[sq], L = cu[sq + 1] - t0;
  const int Lk = (L + 31) & ~31;
  const int vst = ((Lk + 127) & ~127) + (BF || X3 ? 8 : 4);
  char* Ks = sm;
  char* Vt = sm + (size_t)Lk * KROW;
  // X3: operands split ONCE here (a K / V element feeds every query tile of the sequence), in
  // bf16 hi | lo form, with the lane's 8 MFMA k-slots contiguous: dim (key-in-chunk) c sits at
  // slot 8 ((c & 15) >> 2) + 4 (c >> 4) + (c & 3) -- slots 8g..8g+7 of lane group g are c =
  // 4g..4g+3, 16+4g..16+4g+3, the f32 path's two groups.  K row: hi[32] then lo[32] (bf16);
  // V^T: plane hi [32][vst] then plane lo [32][vst] (bf16).
  uint16_t* Vhi = (uint16_t*)Vt;
  uint16_t* Vlo = Vhi + (size_t)32 * vst;
  if constexpr (X3) {
    for (int e = tid; e < Lk * DH; e += 256) {
      const int j = e / DH, c = e % DH;
      float kv = 0.0f, vv = 0.0f;
      if (j < L) {
        const TI* row = qkv + (int64_t)(t0 + j) * ldq + h * DH + c;
        kv = row[H];
        vv = row[2 * H];
      }
      const int sc_ = 8 * ((c & 15) >> 2) + 4 * (c >> 4) + (c & 3);
      const int jo = j & 31, sj = (j & ~31) + 8 * ((jo & 15) >> 2) + 4 * (jo >> 4) + (jo & 3);
      const uint16_t kh = f32_to_bf16_rne(kv), vh = f32_to_bf16_rne(vv);
      const uint16_t kl = f32_to_bf16_rne(kv - __uint_as_float((uint32_t)kh << 16));
      const uint16_t vl = f32_to_bf16_rne(vv - __uint_as_float((uint32_t)vh << 16));
      uint16_t* kr = (uint16_t*)(Ks + j * KROW);
      kr[sc_] = kh;
      kr[32 + sc_] = kl;
      Vhi[(size_t)c * vst + sj] = vh;
      Vlo[(size_t)c * vst + sj] = vl;
    }
  } else
  if constexpr (sizeof(TI) == 2) {
    // bf16 input: 16-B chunks (8 dims) of each K / V row -- one global load each (the head's
    // 64-B slice of a token row is 4 chunks); K rows copied whole, V transposed into V^T
    for (int e = tid; e < Lk * 4; e += 256) {
      const int j = e >> 2, c8 = 8 * (e & 3);
      u32x4 kq = {0u, 0u, 0u, 0u}, vq = {0u, 0u, 0u, 0u};
      if (j < L) {
        const TI* row = qkv + (int64_t)(t0 + j) * ldq + h * DH + c8;
        kq = *(const u32x4*)(row + H);
        vq = *(const u32x4*)(row + 2 * H);
      }
      *(u32x4*)(Ks + j * KROW + c8 * 2) = kq;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        *(uint16_t*)(Vt + ((size_t)(c8 + i) * vst + j) * 2) = (uint16_t)(vq[i >> 1] >> (16 * (i & 1)));
    }
  } else
  for (int e = tid; e < Lk * DH; e += 256) {
    const int j = e / DH, c = e % DH;
    float kv = 0.0f, vv = 0.0f;
    if constexpr (sizeof(TI) == 2) {  // bf16 input (BF only): copy the bits
      uint16_t kb = 0, vb = 0;
      if (j < L) {
        const TI* row = qkv + (int64_t)(t0 + j) * ldq + h * DH + c;
        kb = row[H];
        vb = row[2 * H];
      }
      *(uint16_t*)(Ks + j * KROW + c * 2) = kb;
      *(uint16_t*)(Vt + ((size_t)c * vst + j) * 2) = vb;
      continue;
    } else if (j < L) {
      const TI* row = qkv + (int64_t)(t0 + j) * ldq + h * DH + c;
      kv = row[H];
      vv = row[2 * H];
    }
    if (BF) {
      *(uint16_t*)(Ks + j * KROW + c * 2) = f32_to_bf16_rne(kv);
      *(uint16_t*)(Vt + ((size_t)c * vst + j) * 2) = f32_to_bf16_rne(vv);
    } else {
      *(float*)(Ks + j * KROW + c * 4) = kv;
      *(float*)(Vt + ((size_t)c * vst + j) * 4) = vv;
    }
  }
  __syncthreads();
  for (int q0 = 16 * w; q0 < L; q0 += 64) {
    const int qr = q0 + ql < L ? q0 + ql : L - 1;
    const TI* qp = qkv + (int64_t)(t0 + qr) * ldq + h * DH;
    f32x4 qa = {0.f, 0.f, 0.f, 0.f}, qb = {0.f, 0.f, 0.f, 0.f};
    bf16x8e qf;
    if constexpr (sizeof(TI) == 2) {  // slots 8g + j <-> dims 8g + j, bits copied
      qf = __builtin_bit_cast(bf16x8e, *(const u32x4*)(qp + 8 * g));
    } else if (!BF) {
      qa = *(const f32x4*)(qp + 4 * g);
      qb = *(const f32x4*)(qp + 16 + 4 * g);
    } else {  // slots 8g + j <-> dims 8g + j
      const f32x4 x0 = *(const f32x4*)(qp + 8 * g), x1 = *(const f32x4*)(qp + 8 * g + 4);
      u32x4 u = {(uint32_t)f32_to_bf16_rne(x0[0]) | ((uint32_t)f32_to_bf16_rne(x0[1]) << 16),
                 (uint32_t)f32_to_bf16_rne(x0[2]) | ((uint32_t)f32_to_bf16_rne(x0[3]) << 16),
                 (uint32_t)f32_to_bf16_rne(x1[0]) | ((uint32_t)f32_to_bf16_rne(x1[1]) << 16),
                 (uint32_t)f32_to_bf16_rne(x1[2]) | ((uint32_t)f32_to_bf16_rne(x1[3]) << 16)};
      qf = __builtin_bit_cast(bf16x8e, u);
    }
    bf16x8e qhi, qlo;  // X3: the query's split operands
    if (X3) split_bf16x8(__builtin_bit_cast(u32x4, qa), __builtin_bit_cast(u32x4, qb), qhi, qlo);
    float m = -__builtin_huge_valf(), lsum = 0.0f;
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    for (int kc = 0; kc < Lk; kc += 32) {
      f32x4 sc[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const char* kr = Ks + (kc + 16 * b + ql) * KROW;
        f32x4 z = {0.f, 0.f, 0.f, 0.f};
        if (BF) {
          const u32x4 kf = *(const u32x4*)(kr + 16 * g);
          z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8e, kf), qf, z, 0, 0, 0);
        } else if (X3) {
          const bf16x8e khi = __builtin_bit_cast(bf16x8e, *(const u32x4*)(kr + 16 * g));
          const bf16x8e klo = __builtin_bit_cast(bf16x8e, *(const u32x4*)(kr + 64 + 16 * g));
          z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(khi, qhi, z, 0, 0, 0);
          z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(klo, qhi, z, 0, 0, 0);
          z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(khi, qlo, z, 0, 0, 0);
        } else {  // slot g <-> dim 4g + u (u < 4), 16 + 4g + (u - 4) (u >= 4)
          const f32x4 ka = *(const f32x4*)(kr + 16 * g), kb = *(const f32x4*)(kr + 64 + 16 * g);
#pragma unroll
          for (int u = 0; u < 4; ++u) z = __builtin_amdgcn_mfma_f32_16x16x4f32(ka[u], qa[u], z, 0, 0, 0);
#pragma unroll
          for (int u = 0; u < 4; ++u) z = __builtin_amdgcn_mfma_f32_16x16x4f32(kb[u], qb[u], z, 0, 0, 0);
        }
        // z[v] = score(key kc + 16b + 4g + v, query q0 + ql)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int key = kc + 16 * b + 4 * g + v;
          z[v] = key < L ? z[v] * scale : -__builtin_huge_valf();
        }
        sc[b] = z;
      }
      float cm = fmaxf(fmaxf(fmaxf(sc[0][0], sc[0][1]), fmaxf(sc[0][2], sc[0][3])),
                       fmaxf(fmaxf(sc[1][0], sc[1][1]), fmaxf(sc[1][2], sc[1][3])));
      cm = fmaxf(cm, __shfl_xor(cm, 16, 64));
      cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
      const float mn = fmaxf(m, cm);
      const float corr = expf(m - mn);
      m = mn;
      float ps = 0.0f;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          sc[b][v] = expf(sc[b][v] - mn);
          ps += sc[b][v];
        }
      ps += __shfl_xor(ps, 16, 64);
      ps += __shfl_xor(ps, 32, 64);
      lsum = lsum * corr + ps;
#pragma unroll
      for (int db = 0; db < 2; ++db) acc[db] = acc[db] * corr;
      if (BF) {  // P^T slots: j < 4 <-> key kc + 4g + j, j >= 4 <-> kc + 16 + 4g + (j - 4)
        u32x4 pu = {(uint32_t)f32_to_bf16_rne(sc[0][0]) | ((uint32_t)f32_to_bf16_rne(sc[0][1]) << 16),
                    (uint32_t)f32_to_bf16_rne(sc[0][2]) | ((uint32_t)f32_to_bf16_rne(sc[0][3]) << 16),
                    (uint32_t)f32_to_bf16_rne(sc[1][0]) | ((uint32_t)f32_to_bf16_rne(sc[1][1]) << 16),
                    (uint32_t)f32_to_bf16_rne(sc[1][2]) | ((uint32_t)f32_to_bf16_rne(sc[1][3]) << 16)};
        const bf16x8e pf = __builtin_bit_cast(bf16x8e, pu);
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          const char* vr = Vt + ((size_t)(16 * db + ql) * vst + kc + 4 * g) * 2;
          const uint64_t lo = *(const uint64_t*)vr, hi = *(const uint64_t*)(vr + 32);
          u32x4 vu = {(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
          acc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8e, vu), pf,
                                                            acc[db], 0, 0, 0);
        }
      } else if (X3) {  // slots: keys kc + 4g + v (v < 4), kc + 16 + 4g + (v - 4)
        bf16x8e phi, plo;
        split_bf16x8(__builtin_bit_cast(u32x4, sc[0]), __builtin_bit_cast(u32x4, sc[1]), phi, plo);
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          const size_t vo = (size_t)(16 * db + ql) * vst + kc + 8 * g;
          const bf16x8e vhi = __builtin_bit_cast(bf16x8e, *(const u32x4*)(Vhi + vo));
          const bf16x8e vlo = __builtin_bit_cast(bf16x8e, *(const u32x4*)(Vlo + vo));
          acc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vhi, phi, acc[db], 0, 0, 0);
          acc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vlo, phi, acc[db], 0, 0, 0);
          acc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vhi, plo, acc[db], 0, 0, 0);
        }
      } else {  // per 16-key block b and v: slot g <-> key kc + 16b + 4g + v
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const f32x4 vv = *(const f32x4*)(Vt + ((size_t)(16 * db + ql) * vst + kc + 16 * b + 4 * g) * 4);
#pragma unroll
            for (int v = 0; v < 4; ++v)
              acc[db] = __builtin_amdgcn_mfma_f32_16x16x4f32(vv[v], sc[b][v], acc[db], 0, 0, 0);
          }
      }
    }
    // acc[db][v] = O^T[dim 16 db + 4 g + v][query q0 + ql]
    if (q0 + ql < L) {
      const float inv = 1.0f / lsum;
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const f32x4 o = acc[db] * inv;
        if (out) *(f32x4*)(out + (int64_t)(t0 + q0 + ql) * ldo + h * DH + 16 * db + 4 * g) = o;
        if (out16) {  // 4 consecutive dims: one 8-B store
          uint16_t* o16 = out16 + (int64_t)(t0 + q0 + ql) * ldo + h * DH + 16 * db + 4 * g;
          const uint2 hv = uint2{(uint32_t)f32_to_bf16_rne(o[0]) | ((uint32_t)f32_to_bf16_rne(o[1]) << 16),
                                 (uint32_t)f32_to_bf16_rne(o[2]) | ((uint32_t)f32_to_bf16_rne(o[3]) << 16)};
          *(uint2*)o16 = hv;
          if (X3 && split16)
            *(uint2*)(o16 + H) = uint2{pack_bf16_hw(o[0] - __uint_as_float(hv.x << 16),
                                                    o[1] - __uint_as_float(hv.x & 0xffff0000u)),
                                       pack_bf16_hw(o[2] - __uint_as_float(hv.y << 16),
                                                    o[3] - __uint_as_float(hv.y & 0xffff0000u))};
        }
      }
    }
  }
}

// bf16 fast path of k_attn32_mfma (bf16 qkv in, bf16 context out; the f32 instantiations
// above stay the parity path).  Same MFMA dataflow; the VALU per MFMA (83 in the shared
// kernel: PMC) is cut by: scores scaled by scale*log2(e) inside the exponent (v_exp_f32 =
// exp2), a two-pass softmax (below), bf16 packing by v_cvt_pk_bf16_f32, key masking only in a
// sequence's last 32-key chunk, and V^T staged two keys per lane as packed dwords (8
// ds_write_b32 per 2 rows instead of 16 ds_write_b16, no two lanes writing halves of a dword).
// HG heads of one sequence per block, 4 waves per head: HG = 2 stages 2 consecutive heads
// (their Q/K/V slices are a full 128-B line of a qkv row instead of half of one) and amortises
// the block's fixed latency (cu loads, staging, barrier) over 2 heads.
template <int HG>
__global__ __launch_bounds__(256 * HG) void k_attn32_bf16(
    const uint16_t* __restrict__ qkv, int64_t ldq, const int32_t* __restrict__ cu, int H,
    int heads, float scale, uint16_t* __restrict__ out16, int64_t ldo) {
  constexpr int DH = 32, KROW = DH * 2 + 16;
  constexpr int WPH = 4, NT = 64 * HG * WPH;
  extern __shared__ __attribute__((aligned(16))) char sm[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int hh = w / WPH, wsub = w % WPH;
  const int g = lane >> 4, ql = lane & 15;
  // the heads of one sequence read parts of the same 128-B lines of qkv: keep them on one XCD
  // (one L2) -- with the hardware's round-robin placement each XCD fetched every line
  const int groups = heads / HG;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int sq = lb / groups, h0 = (lb % groups) * HG, h = h0 + hh;
  const int t0 = cu[sq], L = cu[sq + 1] - t0;
  const int Lk = (L + 31) & ~31;
  const int vst = ((Lk + 127) & ~127) + 8;  // V^T row stride (bf16 elements)
  const size_t per_head = (size_t)Lk * KROW + (size_t)32 * vst * 2;
  char* Ks = sm + hh * per_head;
  char* Vt = Ks + (size_t)Lk * KROW;
  // this wave's first query fragment is loaded before the K/V staging, so its latency overlaps
  // the staging loads instead of following the barrier (then one group ahead in the loop)
  auto load_q = [&](int q0_) {
    const int qr = q0_ + ql < L ? q0_ + ql : L - 1;
    return *(const u32x4*)(qkv + (int64_t)(t0 + qr) * ldq + h * DH + 8 * g);
  };
  u32x4 qnext = load_q(16 * wsub < L ? 16 * wsub : 0);
  // K rows: 16-B chunks copied whole; V^T: lane pair of keys (2p, 2p+1) x 8 dims -> 8 dwords;
  // item e = (key pair p, head hs of the group, 8-dim chunk c8), chunk fastest
  for (int e = tid; e < (Lk / 2) * 4 * HG; e += NT) {
    const int cc = e % (4 * HG), hs = cc >> 2;
    const int p = e / (4 * HG), c8 = 8 * (cc & 3), j = 2 * p;
    char* Ks = sm + hs * per_head;
    char* Vt = Ks + (size_t)Lk * KROW;
    u32x4 k0 = {0u, 0u, 0u, 0u}, k1 = k0, v0 = k0, v1 = k0;
    const uint16_t* row = qkv + (int64_t)(t0 + j) * ldq + (h0 + hs) * DH + c8;
    if (j < L) {
      k0 = *(const u32x4*)(row + H);
      v0 = *(const u32x4*)(row + 2 * H);
    }
    if (j + 1 < L) {
      k1 = *(const u32x4*)(row + ldq + H);
      v1 = *(const u32x4*)(row + ldq + 2 * H);
    }
    *(u32x4*)(Ks + j * KROW + c8 * 2) = k0;
    *(u32x4*)(Ks + (j + 1) * KROW + c8 * 2) = k1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t a = (v0[i >> 1] >> (16 * (i & 1))) & 0xffffu;
      const uint32_t b = (v1[i >> 1] >> (16 * (i & 1))) & 0xffffu;
      *(uint32_t*)(Vt + ((size_t)(c8 + i) * vst + j) * 2) = a | (b << 16);
    }
  }
  __syncthreads();
  const float sl2 = scale * 1.4426950408889634f;  // scores in log2 units
  // Two passes over the keys per 16-query group (the kernel is VALU-bound, the MFMAs cheap):
  // pass 1 finds each query's maximum raw score (lane-partial maxima, one cross-lane reduce),
  // pass 2 recomputes S and accumulates exp2(s * sl2 - m * sl2) and P.V with that fixed
  // offset -- no per-chunk cross-lane max, rescale of the accumulators or correction exp of
  // the online form (59 -> ~32 VALU per 32-key chunk), and the row sums stay lane-partial
  // until the end.  Measured: the same 284 us per layer at 365k tokens as the online form
  // (the VALU was not the limiter); kept for its exact row maximum.
  for (int q0 = 16 * wsub; q0 < L; q0 += 16 * WPH) {
    const bf16x8e qf = __builtin_bit_cast(bf16x8e, qnext);
    if (q0 + 16 * WPH < L) qnext = load_q(q0 + 16 * WPH);
    auto scores = [&](int kc, f32x4 (&sc)[2]) __attribute__((always_inline)) {
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const u32x4 kf = *(const u32x4*)(Ks + (kc + 16 * b + ql) * KROW + 16 * g);
        sc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8e, kf), qf,
                                                        f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      }
      // sc[b][v] = score(key kc + 16b + 4g + v, query q0 + ql); mask past L (last chunk only)
      if (kc + 32 > L) {
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int v = 0; v < 4; ++v)
            if (kc + 16 * b + 4 * g + v >= L) sc[b][v] = -__builtin_huge_valf();
      }
    };
    float m = -__builtin_huge_valf();
    for (int kc = 0; kc < Lk; kc += 32) {
      f32x4 sc[2];
      scores(kc, sc);
      m = fmaxf(m, fmaxf(fmaxf(fmaxf(sc[0][0], sc[0][1]), fmaxf(sc[0][2], sc[0][3])),
                         fmaxf(fmaxf(sc[1][0], sc[1][1]), fmaxf(sc[1][2], sc[1][3]))));
    }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    const float m2 = m * sl2;
    float lpart = 0.0f;
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    for (int kc = 0; kc < Lk; kc += 32) {
      f32x4 sc[2];
      scores(kc, sc);
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          sc[b][v] = __builtin_amdgcn_exp2f(fmaf(sc[b][v], sl2, -m2));
          lpart += sc[b][v];
        }
      // P^T slots: j < 4 <-> key kc + 4g + j, j >= 4 <-> kc + 16 + 4g + (j - 4)
      const u32x4 pu = {pack_bf16_hw(sc[0][0], sc[0][1]), pack_bf16_hw(sc[0][2], sc[0][3]),
                        pack_bf16_hw(sc[1][0], sc[1][1]), pack_bf16_hw(sc[1][2], sc[1][3])};
      const bf16x8e pf = __builtin_bit_cast(bf16x8e, pu);
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const char* vr = Vt + ((size_t)(16 * db + ql) * vst + kc + 4 * g) * 2;
        const uint64_t lo = *(const uint64_t*)vr, hi = *(const uint64_t*)(vr + 32);
        const u32x4 vu = {(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
        acc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8e, vu), pf,
                                                          acc[db], 0, 0, 0);
      }
    }
    float lsum = lpart + __shfl_xor(lpart, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    // acc[db][v] = O^T[dim 16 db + 4 g + v][query q0 + ql]
    if (q0 + ql < L) {
      const float inv = 1.0f / lsum;
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const f32x4 o = acc[db] * inv;
        *(uint2*)(out16 + (int64_t)(t0 + q0 + ql) * ldo + h * DH + 16 * db + 4 * g) =
            uint2{pack_bf16_hw(o[0], o[1]), pack_bf16_hw(o[2], o[3])};
      }
    }
  }
}

// x3 attention: the fast kernel's structure (K / V^T staged with 16-B loads, HG heads of a
// sequence per block, two passes over the keys) on split-bf16 operands.  qkv arrives as the
// QKV GEMM's x3i interleaved rows (a head's 32 dims = one 32-block: 64 B hi then 64 B lo;
// Q of head h is block h, K block heads + h, V block 2 heads + h); each product is three
// bf16 MFMAs (hi.hi + lo.hi + hi.lo, as k_attn32_mfma<X3>): S = K Q^T and O^T = V^T P^T with
// P split in registers.  Pass 1 finds each query's row maximum from the hi.hi scores only (an
// offset for exp2's range; the softmax is exact for any offset), pass 2 the full scores, exp2
// and P.V.  The context goes out x3i interleaved (the Wo GEMM's A).
// LDS per head: K rows hi | lo (144 B) and V^T as two bf16 planes.
template <int HG>
__global__ __launch_bounds__(256 * HG) void k_attn32_x3(
    const uint16_t* __restrict__ qkv, int64_t ldq, const int32_t* __restrict__ cu,
    int H, int heads, float scale, uint16_t* __restrict__ out16, int64_t ldo) {
  constexpr int DH = 32, KROW = 2 * DH * 2 + 16;
  constexpr int WPH = 4, NT = 64 * HG * WPH;
  extern __shared__ __attribute__((aligned(16))) char sm[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int hh = w / WPH, wsub = w % WPH;
  const int g = lane >> 4, ql = lane & 15;
  const int groups = heads / HG;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int sq = lb / groups, h0 = (lb % groups) * HG, h = h0 + hh;
  const int t0 = cu[sq], L = cu[sq + 1] - t0;
  const int Lk = (L + 31) & ~31;
  const int vst = ((Lk + 127) & ~127) + 8;  // V^T row stride (bf16 elements)
  const size_t vplane = (size_t)32 * vst * 2;
  const size_t per_head = (size_t)Lk * KROW + 2 * vplane;
  char* Ks = sm + hh * per_head;
  char* Vt = Ks + (size_t)Lk * KROW;
  auto load_q = [&](int q0_, u32x4& qh, u32x4& qlo) __attribute__((always_inline)) {
    const int qr = q0_ + ql < L ? q0_ + ql : L - 1;
    const uint16_t* qp = qkv + (int64_t)(t0 + qr) * ldq + 64 * h + 8 * g;
    qh = *(const u32x4*)qp;
    qlo = *(const u32x4*)(qp + 32);
  };
  u32x4 qnh, qnl;
  load_q(16 * wsub < L ? 16 * wsub : 0, qnh, qnl);
  // item e = (key pair p, plane pl, head hs, 8-dim chunk c8), chunk fastest
  for (int e = tid; e < (Lk / 2) * 8 * HG; e += NT) {
    const int cc = e % (8 * HG), hs = (cc >> 2) % HG, pl = cc / (4 * HG);
    const int p = e / (8 * HG), c8 = 8 * (cc & 3), j = 2 * p;
    char* Ks_ = sm + hs * per_head;
    char* Vp = Ks_ + (size_t)Lk * KROW + pl * vplane;
    u32x4 k0 = {0u, 0u, 0u, 0u}, k1 = k0, v0 = k0, v1 = k0;
    const uint16_t* row = qkv + (int64_t)(t0 + j) * ldq + 64 * (h0 + hs) + 32 * pl + c8;
    if (j < L) {
      k0 = *(const u32x4*)(row + 2 * H);
      v0 = *(const u32x4*)(row + 4 * H);
    }
    if (j + 1 < L) {
      k1 = *(const u32x4*)(row + ldq + 2 * H);
      v1 = *(const u32x4*)(row + ldq + 4 * H);
    }
    *(u32x4*)(Ks_ + j * KROW + pl * 64 + c8 * 2) = k0;
    *(u32x4*)(Ks_ + (j + 1) * KROW + pl * 64 + c8 * 2) = k1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t a = (v0[i >> 1] >> (16 * (i & 1))) & 0xffffu;
      const uint32_t b = (v1[i >> 1] >> (16 * (i & 1))) & 0xffffu;
      // V^T column swizzle: the 16 lanes of a key pair write rows 8 apart of 4 planes -- one
      // bank (67% of the kernel's LDS cycles were conflicts) -- unless the pair's column is
      // XORed by 4 x (row group, plane); XOR by multiples of 4 keeps the readers' 4-key
      // groups contiguous and inside the row (< vst).  Encode -0.7% (B 256) / -0.8% (B 5120).
      const int jw = j ^ (4 * ((c8 >> 3) + 4 * (hs + HG * pl)));
      *(uint32_t*)(Vp + ((size_t)(c8 + i) * vst + jw) * 2) = a | (b << 16);
    }
  }
  __syncthreads();
  const float sl2 = scale * 1.4426950408889634f;  // scores in log2 units
  for (int q0 = 16 * wsub; q0 < L; q0 += 16 * WPH) {
    const bf16x8e qh = __builtin_bit_cast(bf16x8e, qnh), qlo = __builtin_bit_cast(bf16x8e, qnl);
    if (q0 + 16 * WPH < L) load_q(q0 + 16 * WPH, qnh, qnl);
    auto mask = [&](int kc, f32x4 (&sc)[2]) __attribute__((always_inline)) {
      if (kc + 32 > L) {
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int v = 0; v < 4; ++v)
            if (kc + 16 * b + 4 * g + v >= L) sc[b][v] = -__builtin_huge_valf();
      }
    };
    // pass 1: row maximum of the hi.hi scores (sc[b][v] = key kc + 16b + 4g + v, query ql)
    float m = -__builtin_huge_valf();
    for (int kc = 0; kc < Lk; kc += 32) {
      f32x4 sc[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const u32x4 kf = *(const u32x4*)(Ks + (kc + 16 * b + ql) * KROW + 16 * g);
        sc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8e, kf), qh,
                                                        f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      }
      mask(kc, sc);
      m = fmaxf(m, fmaxf(fmaxf(fmaxf(sc[0][0], sc[0][1]), fmaxf(sc[0][2], sc[0][3])),
                         fmaxf(fmaxf(sc[1][0], sc[1][1]), fmaxf(sc[1][2], sc[1][3]))));
    }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    const float m2 = m * sl2;
    float lpart = 0.0f;
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    for (int kc = 0; kc < Lk; kc += 32) {
      f32x4 sc[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const char* kr = Ks + (kc + 16 * b + ql) * KROW + 16 * g;
        const bf16x8e kh = __builtin_bit_cast(bf16x8e, *(const u32x4*)kr);
        const bf16x8e kl = __builtin_bit_cast(bf16x8e, *(const u32x4*)(kr + 64));
        f32x4 z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kh, qh, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kl, qh, z, 0, 0, 0);
        sc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kh, qlo, z, 0, 0, 0);
      }
      mask(kc, sc);
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          sc[b][v] = __builtin_amdgcn_exp2f(fmaf(sc[b][v], sl2, -m2));
          lpart += sc[b][v];
        }
      // P^T slots: j < 4 <-> key kc + 4g + j, j >= 4 <-> kc + 16 + 4g + (j - 4); split hi | lo
      bf16x8e ph, plo;
      split_bf16x8(__builtin_bit_cast(u32x4, sc[0]), __builtin_bit_cast(u32x4, sc[1]), ph, plo);
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const int d = 16 * db + ql;
        const char* vrow = Vt + (size_t)d * vst * 2;
        // hi / lo plane columns under the staging's swizzle
        const int sh = 4 * (((d >> 3) & 3) + 4 * hh), sl = sh + 16 * HG;
        const int c0 = (kc + 4 * g) ^ sh, c1 = (kc + 16 + 4 * g) ^ sh;
        const int e0 = (kc + 4 * g) ^ sl, e1 = (kc + 16 + 4 * g) ^ sl;
        const uint64_t a0 = *(const uint64_t*)(vrow + c0 * 2), a1 = *(const uint64_t*)(vrow + c1 * 2);
        const uint64_t b0 = *(const uint64_t*)(vrow + vplane + e0 * 2),
                       b1 = *(const uint64_t*)(vrow + vplane + e1 * 2);
        const bf16x8e vh = __builtin_bit_cast(
            bf16x8e, u32x4{(uint32_t)a0, (uint32_t)(a0 >> 32), (uint32_t)a1, (uint32_t)(a1 >> 32)});
        const bf16x8e vl = __builtin_bit_cast(
            bf16x8e, u32x4{(uint32_t)b0, (uint32_t)(b0 >> 32), (uint32_t)b1, (uint32_t)(b1 >> 32)});
        acc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vh, ph, acc[db], 0, 0, 0);
        acc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vl, ph, acc[db], 0, 0, 0);
        acc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vh, plo, acc[db], 0, 0, 0);
      }
    }
    float lsum = lpart + __shfl_xor(lpart, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    // acc[db][v] = O^T[dim 16 db + 4 g + v][query q0 + ql] -> the context, x3i interleaved
    // the two 16-dim blocks re-paired by v_permlane16_swap (partners share ql, so they are
    // valid together): lane g then holds dims 16 (g & 1) + 8 (g >> 1) .. + 7 -> one 16-B hi
    // and one 16-B lo store, a full 128-B x3i line per query row (was 8-B pieces)
    const float inv = 1.0f / lsum;
    uint32_t ph[2][2], pw[2][2];
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      const f32x4 o = acc[db] * inv;
      ph[db][0] = pack_bf16_hw(o[0], o[1]);
      ph[db][1] = pack_bf16_hw(o[2], o[3]);
      pw[db][0] = pack_bf16_hw(o[0] - __uint_as_float(ph[db][0] << 16),
                               o[1] - __uint_as_float(ph[db][0] & 0xffff0000u));
      pw[db][1] = pack_bf16_hw(o[2] - __uint_as_float(ph[db][1] << 16),
                               o[3] - __uint_as_float(ph[db][1] & 0xffff0000u));
    }
    const auto s0 = __builtin_amdgcn_permlane16_swap(ph[0][0], ph[1][0], false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(ph[0][1], ph[1][1], false, false);
    const auto u0 = __builtin_amdgcn_permlane16_swap(pw[0][0], pw[1][0], false, false);
    const auto u1 = __builtin_amdgcn_permlane16_swap(pw[0][1], pw[1][1], false, false);
    if (q0 + ql < L) {
      uint16_t* o16 = out16 + (int64_t)(t0 + q0 + ql) * ldo + 64 * h + 16 * (g & 1) + 8 * (g >> 1);
      *(u32x4*)o16 = u32x4{s0[0], s1[0], s0[1], s1[1]};
      *(u32x4*)(o16 + 32) = u32x4{u0[0], u1[0], u0[1], u1[1]};
    }
  }
}

size_t attn32_x3_smem(int max_len) {
  const int Lk = (max_len + 31) & ~31;
  const int vst = ((Lk + 127) & ~127) + 8;
  return (size_t)Lk * (2 * 32 * 2 + 16) + 2 * (size_t)32 * vst * 2;
}

size_t attn32_smem(int max_len, bool bf, bool x3 = false) {
  const int Lk = (max_len + 31) & ~31;
  const int vst = ((Lk + 127) & ~127) + (bf || x3 ? 8 : 4);
  // x3: K rows hi | lo (bf16, 144 B like f32), V^T as two bf16 planes (hi, lo)
  return (size_t)Lk * (32 * (bf ? 2 : 4) + 16) + (size_t)32 * vst * (bf ? 2 : 4);
}

// Mean pooling over each packed sequence: sum_t h[t] / max(L, 1e-9)  (ST Pooling, mean).
__global__ __launch_bounds__(256) void k_mean_pool(const float* __restrict__ x, int64_t ldx,
                                                   const int32_t* __restrict__ cu, int H,
                                                   float* __restrict__ out, int64_t ldo) {
  const int sq = blockIdx.x;
  const int t0 = cu[sq], t1 = cu[sq + 1];
  const float cnt = fmaxf((float)(t1 - t0), 1e-9f);
  for (int e = threadIdx.x; e < H; e += blockDim.x) {
    float s = 0.0f;
#pragma unroll 8
    for (int t = t0; t < t1; ++t) s += x[(int64_t)t * ldx + e];  // sequential sum, loads ahead
    out[(int64_t)sq * ldo + e] = s / cnt;
  }
}

// [pooled (Ht) | brand_table[bid] (C) | cat_table[cid] (C)] -> f32 rows (+bf16 copy);
// a null table (or negative id) contributes zeros (item_tower.py:158-159,168-169).
__global__ __launch_bounds__(256) void k_item_concat(const float* __restrict__ pooled,
                                                     int64_t ldp, int Ht,
                                                     const int32_t* __restrict__ bid,
                                                     const float* __restrict__ btab,
                                                     const int32_t* __restrict__ cid,
                                                     const float* __restrict__ ctab, int C,
                                                     float* __restrict__ out, int64_t ldo,
                                                     uint16_t* __restrict__ out16, int width) {
  const int r = blockIdx.x;
  for (int e = threadIdx.x; e < width; e += blockDim.x) {
    float v = 0.0f;
    if (e < Ht) v = pooled[(int64_t)r * ldp + e];
    else if (e < Ht + C) v = (btab && bid && bid[r] >= 0) ? btab[(int64_t)bid[r] * C + (e - Ht)] : 0.0f;
    else if (e < Ht + 2 * C) v = (ctab && cid && cid[r] >= 0) ? ctab[(int64_t)cid[r] * C + (e - Ht - C)] : 0.0f;
    out[(int64_t)r * ldo + e] = v;
    if (out16) out16[(int64_t)r * ldo + e] = f32_to_bf16_rne(v);
  }
}

}  // namespace tt

using namespace tt;

// ------------------------------------------------------------------------------- C ABI
namespace {
int enc_device_cus() {
  static const int cus = [] {
    int d = 0, v = 0;
    if (hipGetDevice(&d) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && v > 0)
      return v;
    return 256;
  }();
  return cus;
}
// TT_GEMM_BIG=0 in the environment keeps every bf16 GEMM on the 128x128 kernel (A/B timing)
bool gemm_ln_disabled() {  // TT_GEMM_LN=0: unfused GEMM + LayerNorm (timing builds only)
  static const bool off = env_switch("TT_GEMM_LN", 1) == 0;
  return off;
}
bool gemm_ln96_enabled() {  // TT_GEMM_LN96=0: 128-row k_gemm_ln tiles only (A/B timing)
  static const bool on = env_switch("TT_GEMM_LN96", 1) != 0;
  return on;
}
bool attn_fast_disabled() {  // TT_ATTN_FAST=0: the shared k_attn32_mfma for bf16 too
  static const bool off = env_switch("TT_ATTN_FAST", 1) == 0;
  return off;
}
bool gemm_wide_disabled() {  // TT_GEMM_WIDE=0: keep 256x128 tiles for the wide GEMMs too
  static const bool off = env_switch("TT_GEMM_WIDE", 1) == 0;
  return off;
}
bool x3c_enabled() {  // TT_X3C=0: the x3 path's split-in-loop GEMMs (timing builds: A/B)
  static const bool on = env_switch("TT_X3C", 1) != 0;
  return on;
}
int gemm_big_variant() {  // TT_GEMM_BIG: 0 = 128x128 tiles only, 1 = 256x128 ring (default),
                          // 2 = 128x128 ring, two blocks per CU, 3 = 256x256 ring
  static const int v = [] {
    const int e = env_switch("TT_GEMM_BIG", 1);
    return e >= 0 && e <= 3 ? e : 1;
  }();
  return v;
}
}  // namespace

// x3 GEMMs take the persistent ring kernel from this many 256x128 tiles (TT_X3_BIG_MIN=d,
// timing builds: d quarter-rounds of tiles per CU; 0 = never)
// (default 0: the ring kernel measured slower for x3 -- 84.7 vs 76.2 us mean per GEMM over the
// configs[1] encode; its 8 waves' on-the-fly splits are VALU-bound the same way)
static int x3_big_min_tiles(int ncu) {
  static const int d = env_switch("TT_X3_BIG_MIN", 0);
  return d == 0 ? 1 << 30 : ncu * d / 4;
}

static int gemm_f32_impl(const float* A, int64_t lda, const float* W, int64_t ldw,
                         const float* bias, const float* residual, int64_t ldr, float* C,
                         int64_t ldc, uint16_t* C_bf16, int64_t ldc16, int32_t M, int32_t N,
                         int32_t K, int32_t act, void* stream, bool x3,
                         const uint16_t* wx3 = nullptr, int64_t ldwx3 = 0) {
  if (wx3) {  // pre-split W (k_x3_split_w): the same 128-B rows per 32 k, as float units
    TT_REQUIRE(x3 && ldwx3 % 8 == 0 && ((uintptr_t)wx3 % 16) == 0,
               "pre-split W: 16-B aligned rows, ld % 8 == 0");
    W = (const float*)wx3;
    ldw = ldwx3 / 2;
  }
  TT_REQUIRE(M >= 0 && N >= 0 && K >= 0, "negative size");
  if (M == 0 || N == 0) return TT_OK;
  if (K % GemmElt<float>::BK != 0)
    return fail(TT_ERR_UNSUPPORTED, "tt_gemm_f32: need K % 32 == 0");
  TT_REQUIRE(A && W && (C || C_bf16), "null pointer");
  TT_REQUIRE(lda % 4 == 0 && ldw % 4 == 0 && ((uintptr_t)A % 16) == 0 && ((uintptr_t)W % 16) == 0,
             "A/W must be 16-B aligned with lda, ldw % 4 == 0");
  TT_REQUIRE(act >= 0 && act <= 2, "bad activation");
  const int nblk = ((M + GM_BM - 1) / GM_BM) * ((N + GM_BN - 1) / GM_BN);
  const int nbig = ((M + 255) / 256) * ((N + GB_BN - 1) / GB_BN), ncu = enc_device_cus();
  if (x3 && !wx3 && nbig >= x3_big_min_tiles(ncu)) {
    // the persistent 256x128 ring (3 slots, two stages ahead, one barrier per stage): the
    // 128x128 two-stage kernel left the MFMA pipes ~75% idle on DMA latency
    hipLaunchKernelGGL((k_gemm_big<256, 3, -1, false, float>), dim3(ncu), dim3(512), 0,
                       (hipStream_t)stream, A, lda, W, ldw, bias, residual, ldr, C, ldc, C_bf16,
                       ldc16, M, N, K, act);
    return check_launch("tt_gemm_x3(persistent)");
  }
  if (wx3)
    hipLaunchKernelGGL((k_gemm<float, 2>), dim3(nblk), dim3(256), 0, (hipStream_t)stream, A,
                       lda, W, ldw, bias, residual, ldr, C, ldc, C_bf16, ldc16, M, N, K, act, 0);
  else if (x3)
    hipLaunchKernelGGL((k_gemm<float, 1>), dim3(nblk), dim3(256), 0, (hipStream_t)stream, A,
                       lda, W, ldw, bias, residual, ldr, C, ldc, C_bf16, ldc16, M, N, K, act, 0);
  else
    hipLaunchKernelGGL((k_gemm<float, 0>), dim3(nblk), dim3(256), 0, (hipStream_t)stream, A,
                       lda, W, ldw, bias, residual, ldr, C, ldc, C_bf16, ldc16, M, N, K, act, 0);
  return check_launch(wx3 ? "tt_gemm_x3w" : x3 ? "tt_gemm_x3" : "tt_gemm_f32");
}

extern "C" int tt_gemm_f32(const float* A, int64_t lda, const float* W, int64_t ldw,
                           const float* bias, const float* residual, int64_t ldr, float* C,
                           int64_t ldc, uint16_t* C_bf16, int64_t ldc16, int32_t M, int32_t N,
                           int32_t K, int32_t act, void* stream) {
  return gemm_f32_impl(A, lda, W, ldw, bias, residual, ldr, C, ldc, C_bf16, ldc16, M, N, K, act,
                       stream, false);
}

extern "C" int tt_gemm_x3(const float* A, int64_t lda, const float* W, int64_t ldw,
                          const float* bias, const float* residual, int64_t ldr, float* C,
                          int64_t ldc, uint16_t* C_bf16, int64_t ldc16, int32_t M, int32_t N,
                          int32_t K, int32_t act, void* stream) {
  return gemm_f32_impl(A, lda, W, ldw, bias, residual, ldr, C, ldc, C_bf16, ldc16, M, N, K, act,
                       stream, true);
}

extern "C" int tt_x3_split_weights(const float* W, int64_t ldw, int32_t N, int32_t K,
                                   uint16_t* out, int64_t ld_out, void* stream) {
  TT_REQUIRE(N >= 0 && K >= 0, "negative size");
  if (N == 0 || K == 0) return TT_OK;
  if (K % 32 != 0) return fail(TT_ERR_UNSUPPORTED, "tt_x3_split_weights: need K % 32 == 0");
  TT_REQUIRE(W && out, "null pointer");
  TT_REQUIRE(ldw % 4 == 0 && ((uintptr_t)W % 16) == 0 && ld_out % 8 == 0 &&
                 ((uintptr_t)out % 16) == 0 && ld_out >= 2 * (int64_t)K,
             "W 16-B aligned rows (ldw % 4 == 0); out [N, >= 2K] 16-B aligned (ld % 8 == 0)");
  const int64_t n = (int64_t)N * (K / 32) * 4;
  hipLaunchKernelGGL(k_x3_split_w, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, W, ldw, N, K, out, ld_out);
  return check_launch("tt_x3_split_weights");
}

extern "C" int tt_x3i_weights(const float* W, int64_t ldw, int32_t N, int32_t K, uint16_t* out,
                              int64_t ld_out, void* stream) {
  TT_REQUIRE(N >= 0 && K >= 0, "negative size");
  if (N == 0 || K == 0) return TT_OK;
  if (K % 32 != 0) return fail(TT_ERR_UNSUPPORTED, "tt_x3i_weights: need K % 32 == 0");
  TT_REQUIRE(W && out && ldw >= K && ld_out >= 2 * (int64_t)K, "null pointer or ld too small");
  const int64_t n = (int64_t)N * K;
  hipLaunchKernelGGL(k_x3i_w, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, W, ldw, N, K, out, ld_out);
  return check_launch("tt_x3i_weights");
}

extern "C" int tt_gemm_x3w(const float* A, int64_t lda, const uint16_t* Wx3, int64_t ldwx3,
                           const float* bias, const float* residual, int64_t ldr, float* C,
                           int64_t ldc, uint16_t* C_bf16, int64_t ldc16, int32_t M, int32_t N,
                           int32_t K, int32_t act, void* stream) {
  TT_REQUIRE(Wx3 != nullptr, "null pointer");
  return gemm_f32_impl(A, lda, nullptr, 0, bias, residual, ldr, C, ldc, C_bf16, ldc16, M, N, K,
                       act, stream, true, Wx3, ldwx3);
}

// bf16 GEMM dispatch.  x3i: A [M, K] and W [N, K] are x3i interleaved rows (K = 2 x the
// product's K; k_gemm*<..., X3I>), and the result goes out split (x3i interleaved C_bf16 [M, 2N],
// C == NULL, residual == NULL).  split without x3i is not offered.
static int gemm_bf16_impl(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw,
                          const float* bias, const float* residual, int64_t ldr, float* C,
                          int64_t ldc, uint16_t* C_bf16, int64_t ldc16, int32_t M, int32_t N,
                          int32_t K, int32_t act, void* stream, bool x3i) {
  TT_REQUIRE(M >= 0 && N >= 0 && K >= 0, "negative size");
  if (M == 0 || N == 0) return TT_OK;
  if (K % GemmElt<uint16_t>::BK != 0)
    return fail(TT_ERR_UNSUPPORTED, "tt_gemm_bf16: need K % 64 == 0");
  TT_REQUIRE(A && W && (C || C_bf16), "null pointer");
  TT_REQUIRE(lda % 8 == 0 && ldw % 8 == 0 && ((uintptr_t)A % 16) == 0 && ((uintptr_t)W % 16) == 0,
             "A/W must be 16-B aligned with lda, ldw % 8 == 0");
  TT_REQUIRE(act >= 0 && act <= 2, "bad activation");
  TT_REQUIRE(!x3i || (!C && !residual && C_bf16 && N % 32 == 0 && ldc16 >= 2 * (int64_t)N &&
                      ldc16 % 8 == 0 && ((uintptr_t)C_bf16 % 16) == 0),
             "x3i output: C_bf16 only, N % 32 == 0, ldc16 >= 2N (16-B aligned rows)");
  // large M: the persistent 256x128 ring kernel (one block per CU) once there are at least
  // two tiles per CU
  const int nbig = ((M + 255) / 256) * ((N + GB_BN - 1) / GB_BN);
  const int ncu = enc_device_cus();
  const int variant = gemm_big_variant();
  if (nbig >= 2 * ncu && variant >= 1) {
    // specialisations: activation constant; bf16-only output (QKV, FFN1) without C / residual
    const bool bfo = !C && !residual && C_bf16 && ldc16 % 8 == 0 && ((uintptr_t)C_bf16 % 16) == 0;
    auto launch = [&](auto kern, int blocks, int threads) {
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, (hipStream_t)stream, A, lda, W, ldw,
                         bias, residual, ldr, C, ldc, C_bf16, ldc16, M, N, K, act);
      return check_launch("tt_gemm_bf16(persistent)");
    };
    // default: 256x256 tiles for the wide GEMMs (QKV N = 1152, FFN1 N = 1536: 534 / 747 us vs
    // 586 / 824 us with 256x128 at 370k tokens, bf16), 256x128 otherwise ... unless M is small
    // enough that 256x256 tiles quantise badly onto the CUs (at most two rounds): rounds x tile
    // cost with a 256x128 tile at 0.54 of a 256x256 one.  configs[1]'s QKV (~18k rows,
    // N = 1152): 360 wide tiles = 2 rounds vs 648 narrow = 3 x 0.54 (41.7 -> ~33 us); FFN1
    // (N = 1536) and the Mode A shapes (28+ rounds, where the wide tile measured faster: 546
    // vs 586 us QKV) stay wide.
    const int64_t mt = (M + 255) / 256, ntw = mt * ((N + 255) / 256), ntn = mt * ((N + 127) / 128);
    const bool narrow_pays =
        ntw <= 2 * ncu && ((ntn + ncu - 1) / ncu) * 54 < ((ntw + ncu - 1) / ncu) * 100;
    const bool wide = variant == 3 || (variant == 1 && N >= 1024 && !gemm_wide_disabled() &&
                                       !narrow_pays);
    if (x3i) {  // the x3 encoder's QKV (no activation) / FFN1 (GELU), split output
      if (wide) {
        if (act == ACT_GELU) return launch(k_gemm_wide<ACT_GELU, 2, true>, ncu, 512);
        if (act == ACT_NONE) return launch(k_gemm_wide<ACT_NONE, 2, true>, ncu, 512);
        return launch(k_gemm_wide<ACT_RELU, 2, true>, ncu, 512);
      }
      if (act == ACT_GELU) return launch(k_gemm_big<256, 3, ACT_GELU, 2, uint16_t, true>, ncu, 512);
      if (act == ACT_NONE) return launch(k_gemm_big<256, 3, ACT_NONE, 2, uint16_t, true>, ncu, 512);
      return launch(k_gemm_big<256, 3, ACT_RELU, 2, uint16_t, true>, ncu, 512);
    }
    if (variant == 3 || (wide && bfo)) {  // 256x256
      if (bfo && act == ACT_NONE) return launch(k_gemm_wide<ACT_NONE, true>, ncu, 512);
      if (bfo && act == ACT_GELU) return launch(k_gemm_wide<ACT_GELU, true>, ncu, 512);
      return launch(k_gemm_wide<-1, false>, ncu, 512);
    }
    if (variant == 2) {  // 128x128 tiles, two persistent blocks per CU
      if (bfo && act == ACT_NONE) return launch(k_gemm_big<128, 2, ACT_NONE, true>, 2 * ncu, 256);
      if (bfo && act == ACT_GELU) return launch(k_gemm_big<128, 2, ACT_GELU, true>, 2 * ncu, 256);
      return launch(k_gemm_big<128, 2, -1, false>, 2 * ncu, 256);
    }
    if (bfo && act == ACT_NONE) return launch(k_gemm_big<256, 3, ACT_NONE, true>, ncu, 512);
    if (bfo && act == ACT_GELU) return launch(k_gemm_big<256, 3, ACT_GELU, true>, ncu, 512);
    return launch(k_gemm_big<256, 3, -1, false>, ncu, 512);
  }
  const int nblk = ((M + GM_BM - 1) / GM_BM) * ((N + GM_BN - 1) / GM_BN);
  if (x3i)
    hipLaunchKernelGGL((k_gemm<uint16_t, 0, true>), dim3(nblk), dim3(256), 0, (hipStream_t)stream,
                       A, lda, W, ldw, bias, residual, ldr, C, ldc, C_bf16, ldc16, M, N, K, act,
                       N);
  else
    hipLaunchKernelGGL((k_gemm<uint16_t, 0>), dim3(nblk), dim3(256), 0, (hipStream_t)stream, A, lda,
                       W, ldw, bias, residual, ldr, C, ldc, C_bf16, ldc16, M, N, K, act, 0);
  return check_launch("tt_gemm_bf16");
}

extern "C" int tt_gemm_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw,
                            const float* bias, const float* residual, int64_t ldr, float* C,
                            int64_t ldc, uint16_t* C_bf16, int64_t ldc16, int32_t M, int32_t N,
                            int32_t K, int32_t act, void* stream) {
  return gemm_bf16_impl(A, lda, W, ldw, bias, residual, ldr, C, ldc, C_bf16, ldc16, M, N, K, act,
                        stream, false);
}

extern "C" int tt_gemm_x3i(const uint16_t* A2, int64_t lda2, const uint16_t* W2, int64_t ldw2,
                           const float* bias, uint16_t* C2, int64_t ldc2, int32_t M, int32_t N,
                           int32_t K, int32_t act, void* stream) {
  TT_REQUIRE(K > 0 && K % 32 == 0, "tt_gemm_x3i: need K % 32 == 0");
  return gemm_bf16_impl(A2, lda2, W2, ldw2, bias, nullptr, 0, nullptr, 0, C2, ldc2, M, N, 2 * K,
                        act, stream, true);
}

static int gemm_ln_impl(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw,
                        const float* bias, const float* gamma, const float* beta, float eps,
                        float* x, int64_t ldx, uint16_t* x_bf16, int64_t ldx16, int32_t M,
                        int32_t H, int32_t K, void* stream, bool x3i) {
  TT_REQUIRE(M >= 0 && K >= 0, "negative size");
  if (M == 0) return TT_OK;
  if (H != GL_H) return fail(TT_ERR_UNSUPPORTED, "tt_gemm_ln_bf16: H must be 384");
  if (K % 64 != 0 || K == 0) return fail(TT_ERR_UNSUPPORTED, "tt_gemm_ln_bf16: need K % 64 == 0");
  TT_REQUIRE(A && W && bias && gamma && beta && x && x_bf16, "null pointer");
  TT_REQUIRE(lda % 8 == 0 && ldw % 8 == 0 && ((uintptr_t)A % 16) == 0 && ((uintptr_t)W % 16) == 0,
             "A/W must be 16-B aligned with lda, ldw % 8 == 0");
  TT_REQUIRE(ldx % 4 == 0 && ldx16 % 4 == 0 && ((uintptr_t)x % 16) == 0 &&
                 ((uintptr_t)x_bf16 % 8) == 0 && ((uintptr_t)bias % 16) == 0 &&
                 ((uintptr_t)gamma % 16) == 0 && ((uintptr_t)beta % 16) == 0,
             "x / bias / gamma / beta must be 16-B aligned (x_bf16 8-B), ldx, ldx16 % 4 == 0");
  const int ncu = enc_device_cus();
  // cost of a tile height: rounds (ceil(tiles / CUs)) x (BM + ~32 rows of fixed cost); the
  // smallest cost wins, ties to the taller tile
  int bm = 128;
  int64_t best = ((M + 127) / 128 + ncu - 1) / ncu * (128 + 32);
  if (gemm_ln96_enabled())
    for (int c : {96, 80}) {
      const int64_t cost = (((M + c - 1) / c) + ncu - 1) / ncu * (c + 32);
      if (cost < best) {
        best = cost;
        bm = c;
      }
    }
  const int ntiles = (int)((M + bm - 1) / bm);
  const int grid = ntiles < ncu ? ntiles : ncu;
  // 16-B x16 stores (block pairs) when the copy's rows allow them
  const int st16 = ((uintptr_t)x_bf16 % 16) == 0 && ldx16 % 8 == 0;
  if (x3i) {
    TT_REQUIRE(ldx16 >= 2 * GL_H && ldx16 % 8 == 0, "x3i gemm_ln: x rows x3i interleaved (ldx16 >= 768)");
    auto kern = bm == 80 ? k_gemm_ln<80, true> : bm == 96 ? k_gemm_ln<96, true> : k_gemm_ln<128, true>;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, (hipStream_t)stream, A, lda, W, ldw, bias,
                       gamma, beta, eps, x, ldx, x_bf16, ldx16, M, K, st16);
    return check_launch("tt_gemm_ln_x3i");
  }
  auto kern = bm == 80 ? k_gemm_ln<80> : bm == 96 ? k_gemm_ln<96> : k_gemm_ln<128>;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, (hipStream_t)stream, A, lda, W, ldw, bias,
                     gamma, beta, eps, x, ldx, x_bf16, ldx16, M, K, st16);
  return check_launch("tt_gemm_ln_bf16");
}

extern "C" int tt_gemm_ln_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw,
                               const float* bias, const float* gamma, const float* beta,
                               float eps, float* x, int64_t ldx, uint16_t* x_bf16, int64_t ldx16,
                               int32_t M, int32_t H, int32_t K, void* stream) {
  return gemm_ln_impl(A, lda, W, ldw, bias, gamma, beta, eps, x, ldx, x_bf16, ldx16, M, H, K,
                      stream, false);
}

extern "C" int tt_gemm_ln_x3i(const uint16_t* A2, int64_t lda2, const uint16_t* W2, int64_t ldw2,
                              const float* bias, const float* gamma, const float* beta, float eps,
                              float* x, int64_t ldx, uint16_t* x2, int64_t ldx2, int32_t M,
                              int32_t H, int32_t K, void* stream) {
  TT_REQUIRE(K > 0 && K % 32 == 0, "tt_gemm_ln_x3i: need K % 32 == 0");
  return gemm_ln_impl(A2, lda2, W2, ldw2, bias, gamma, beta, eps, x, ldx, x2, ldx2, M, H, 2 * K,
                      stream, true);
}

extern "C" int tt_layernorm_f32(const float* x, int64_t ldx, const float* gamma,
                                const float* beta, float eps, float* y, int64_t ldy,
                                uint16_t* y_bf16, int64_t ldy16, int64_t rows, int32_t H,
                                void* stream) {
  TT_REQUIRE(rows >= 0 && H >= 1 && H <= 1024, "need rows >= 0, 1 <= H <= 1024");
  if (rows == 0) return TT_OK;
  TT_REQUIRE(x && gamma && beta && y, "null pointer");
  const int64_t b = (rows + 3) / 4;
  hipLaunchKernelGGL(k_layernorm, dim3((unsigned)(b < 8192 ? b : 8192)), dim3(256), 0,
                     (hipStream_t)stream, x, ldx, gamma, beta, eps, y, ldy, y_bf16, ldy16, rows, H);
  return check_launch("tt_layernorm_f32");
}

static int attention_varlen_impl(const float* qkv, int64_t ld_qkv, const int32_t* cu_seqlens,
                                 int32_t n_seq, int32_t max_len, int32_t H, int32_t heads,
                                 int32_t prec, float* out, int64_t ld_out, uint16_t* out_bf16,
                                 void* stream, int split16) {
  TT_REQUIRE(n_seq >= 0 && heads >= 1 && H % heads == 0, "bad n_seq / heads");
  TT_REQUIRE(prec == TT_PREC_F32 || prec == TT_PREC_BF16 || prec == TT_PREC_X3,
             "bad precision");
  if (n_seq == 0) return TT_OK;
  TT_REQUIRE(max_len >= 1 && max_len <= 512, "max_len must be in [1, 512]");
  TT_REQUIRE(qkv && cu_seqlens && (out || (split16 && out_bf16)), "null pointer");
  TT_REQUIRE(!split16 || (prec == TT_PREC_X3 && !out && ld_out >= 2 * (int64_t)H),
             "split context planes: x3 only, out_bf16 [T, >= 2H]");
  TT_REQUIRE(ld_qkv % 4 == 0 && ld_out % 4 == 0 && H % 4 == 0 && ((uintptr_t)qkv % 16) == 0 &&
                 ((uintptr_t)out % 16) == 0, "qkv/out must be 16-B aligned rows");
  if (H / heads != 32)
    return fail(TT_ERR_UNSUPPORTED, "tt_attention_varlen: MFMA path needs head dim 32");
  const bool bf = prec == TT_PREC_BF16, x3 = prec == TT_PREC_X3;
  const size_t smem = attn32_smem(max_len, bf, x3);
  const void* fn = bf   ? (const void*)k_attn32_mfma<true, float>
                   : x3 ? (const void*)k_attn32_mfma<false, float, true>
                        : (const void*)k_attn32_mfma<false, float>;
  if (smem > 64 * 1024 &&
      hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem) != hipSuccess)
    return fail(TT_ERR_LAUNCH, "hipFuncSetAttribute(max dynamic LDS)");
  const float scale = 1.0f / sqrtf(32.0f);
  const dim3 grid((unsigned)(n_seq * heads));
  if (bf)
    hipLaunchKernelGGL((k_attn32_mfma<true, float>), grid, dim3(256), smem, (hipStream_t)stream, qkv,
                       ld_qkv, cu_seqlens, H, heads, scale, out, ld_out, out_bf16, 0);
  else if (x3)
    hipLaunchKernelGGL((k_attn32_mfma<false, float, true>), grid, dim3(256), smem,
                       (hipStream_t)stream, qkv, ld_qkv, cu_seqlens, H, heads, scale, out, ld_out,
                       out_bf16, split16);
  else
    hipLaunchKernelGGL((k_attn32_mfma<false, float>), grid, dim3(256), smem, (hipStream_t)stream, qkv,
                       ld_qkv, cu_seqlens, H, heads, scale, out, ld_out, out_bf16, 0);
  return check_launch("tt_attention_varlen");
}

// x3 attention over x3i interleaved QKV rows (k_attn32_x3): qkv2 [T, ld >= 6H] bf16, context
// out2 [T, ld_out >= 2H] x3i interleaved
extern "C" int tt_attention_varlen_x3i(const uint16_t* qkv2, int64_t ld_qkv2,
                                       const int32_t* cu_seqlens, int32_t n_seq, int32_t max_len,
                                       int32_t H, int32_t heads, uint16_t* out2, int64_t ld_out2,
                                       void* stream) {
  TT_REQUIRE(n_seq >= 0 && heads >= 1 && H % heads == 0, "bad n_seq / heads");
  if (n_seq == 0) return TT_OK;
  TT_REQUIRE(max_len >= 1 && max_len <= 512, "max_len must be in [1, 512]");
  TT_REQUIRE(qkv2 && cu_seqlens && out2, "null pointer");
  if (H / heads != 32)
    return fail(TT_ERR_UNSUPPORTED, "tt_attention_varlen_x3i: head dim must be 32");
  TT_REQUIRE(ld_qkv2 >= 6 * (int64_t)H && ld_qkv2 % 8 == 0 && H % 8 == 0 &&
                 ld_out2 >= 2 * (int64_t)H && ld_out2 % 8 == 0 && ((uintptr_t)qkv2 % 16) == 0 &&
                 ((uintptr_t)out2 % 16) == 0,
             "qkv x3i rows [T, >= 6H] 16-B aligned; context x3i rows [T, >= 2H] 16-B aligned");
  const size_t smem = attn32_x3_smem(max_len);
  const bool h2 = heads % 2 == 0 && 2 * smem <= 160 * 1024;
  const void* fb = h2 ? (const void*)k_attn32_x3<2> : (const void*)k_attn32_x3<1>;
  const size_t sm = h2 ? 2 * smem : smem;
  if (sm > 160 * 1024) return fail(TT_ERR_UNSUPPORTED, "attention K/V exceed LDS");
  if (sm > 64 * 1024 &&
      hipFuncSetAttribute(fb, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm) != hipSuccess)
    return fail(TT_ERR_LAUNCH, "hipFuncSetAttribute(max dynamic LDS)");
  const float scale = 1.0f / sqrtf(32.0f);
  if (h2)
    hipLaunchKernelGGL(k_attn32_x3<2>, dim3((unsigned)(n_seq * heads / 2)), dim3(512), sm,
                       (hipStream_t)stream, qkv2, ld_qkv2, cu_seqlens, H, heads, scale, out2,
                       ld_out2);
  else
    hipLaunchKernelGGL(k_attn32_x3<1>, dim3((unsigned)(n_seq * heads)), dim3(256), sm,
                       (hipStream_t)stream, qkv2, ld_qkv2, cu_seqlens, H, heads, scale, out2,
                       ld_out2);
  return check_launch("tt_attention_varlen_x3i");
}

extern "C" int tt_attention_varlen(const float* qkv, int64_t ld_qkv, const int32_t* cu_seqlens,
                                   int32_t n_seq, int32_t max_len, int32_t H, int32_t heads,
                                   int32_t prec, float* out, int64_t ld_out, uint16_t* out_bf16,
                                   void* stream) {
  return attention_varlen_impl(qkv, ld_qkv, cu_seqlens, n_seq, max_len, H, heads, prec, out,
                               ld_out, out_bf16, stream, 0);
}

extern "C" int tt_attention_varlen_bf16(const uint16_t* qkv, int64_t ld_qkv,
                                        const int32_t* cu_seqlens, int32_t n_seq,
                                        int32_t max_len, int32_t H, int32_t heads, float* out,
                                        int64_t ld_out, uint16_t* out_bf16, void* stream) {
  TT_REQUIRE(n_seq >= 0 && heads >= 1 && H % heads == 0, "bad n_seq / heads");
  if (n_seq == 0) return TT_OK;
  TT_REQUIRE(max_len >= 1 && max_len <= 512, "max_len must be in [1, 512]");
  TT_REQUIRE(qkv && cu_seqlens && (out || out_bf16), "null pointer");
  TT_REQUIRE(ld_qkv % 8 == 0 && ld_out % 4 == 0 && H % 8 == 0 && ((uintptr_t)qkv % 16) == 0 &&
                 ((uintptr_t)out % 16) == 0 && ((uintptr_t)out_bf16 % 8) == 0,
             "qkv must be 16-B aligned rows (out 16-B, out_bf16 8-B aligned)");
  if (H / heads != 32)
    return fail(TT_ERR_UNSUPPORTED, "tt_attention_varlen_bf16: head dim must be 32");
  const size_t smem = attn32_smem(max_len, true);
  if (!out && out_bf16 && !attn_fast_disabled()) {  // bf16-only output: the fast kernel
    // two heads per block (a full 128-B line per row part; 1 / 3 / 4 heads: 285 / 329 / 332 us
    // per layer at 365k tokens vs 274 us)
    const bool h2 = heads % 2 == 0 && 2 * smem <= 160 * 1024;
    const void* fb = h2 ? (const void*)k_attn32_bf16<2> : (const void*)k_attn32_bf16<1>;
    const size_t sm = h2 ? 2 * smem : smem;
    if (sm > 64 * 1024 &&
        hipFuncSetAttribute(fb, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm) != hipSuccess)
      return fail(TT_ERR_LAUNCH, "hipFuncSetAttribute(max dynamic LDS)");
    if (h2)
      hipLaunchKernelGGL(k_attn32_bf16<2>, dim3((unsigned)(n_seq * heads / 2)), dim3(512), sm,
                         (hipStream_t)stream, qkv, ld_qkv, cu_seqlens, H, heads,
                         1.0f / sqrtf(32.0f), out_bf16, ld_out);
    else
      hipLaunchKernelGGL(k_attn32_bf16<1>, dim3((unsigned)(n_seq * heads)), dim3(256), sm,
                         (hipStream_t)stream, qkv, ld_qkv, cu_seqlens, H, heads,
                         1.0f / sqrtf(32.0f), out_bf16, ld_out);
    return check_launch("tt_attention_varlen_bf16");
  }
  const void* fn = (const void*)k_attn32_mfma<true, uint16_t>;
  if (smem > 64 * 1024 &&
      hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem) != hipSuccess)
    return fail(TT_ERR_LAUNCH, "hipFuncSetAttribute(max dynamic LDS)");
  hipLaunchKernelGGL((k_attn32_mfma<true, uint16_t>), dim3((unsigned)(n_seq * heads)), dim3(256),
                     smem, (hipStream_t)stream, qkv, ld_qkv, cu_seqlens, H, heads,
                     1.0f / sqrtf(32.0f), out, ld_out, out_bf16, 0);
  return check_launch("tt_attention_varlen_bf16");
}

extern "C" int tt_attention_varlen_f32(const float* qkv, int64_t ld_qkv, const int32_t* cu_seqlens,
                                       int32_t n_seq, int32_t max_len, int32_t H, int32_t heads,
                                       float* out, int64_t ld_out, uint16_t* out_bf16,
                                       void* stream) {
  TT_REQUIRE(n_seq >= 0 && heads >= 1 && H % heads == 0, "bad n_seq / heads");
  if (n_seq == 0) return TT_OK;
  const int dh = H / heads;
  TT_REQUIRE(max_len >= 1 && max_len <= 512, "max_len must be in [1, 512]");
  TT_REQUIRE(qkv && cu_seqlens && out, "null pointer");
  const size_t smem = (size_t)2 * max_len * dh * sizeof(float);
  if (smem > 160 * 1024) return fail(TT_ERR_UNSUPPORTED, "attention K/V exceed LDS");
  const float scale = 1.0f / sqrtf((float)dh);
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)(n_seq * heads));
  if (smem > 64 * 1024) {
    const void* fn = dh == 32 ? (const void*)k_attn<32> : (const void*)k_attn<64>;
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem) != hipSuccess)
      return fail(TT_ERR_LAUNCH, "hipFuncSetAttribute(max dynamic LDS)");
  }
  switch (dh) {
    case 32:
      hipLaunchKernelGGL(k_attn<32>, grid, dim3(128), smem, st, qkv, ld_qkv, cu_seqlens, H, heads,
                         scale, out, ld_out, out_bf16);
      break;
    case 64:
      hipLaunchKernelGGL(k_attn<64>, grid, dim3(128), smem, st, qkv, ld_qkv, cu_seqlens, H, heads,
                         scale, out, ld_out, out_bf16);
      break;
    default:
      return fail(TT_ERR_UNSUPPORTED, "attention head dim must be 32 or 64");
  }
  return check_launch("tt_attention_varlen_f32");
}

namespace {
size_t align_up(size_t b) { return (b + 255) / 256 * 256; }
struct EncWs {
  float *x, *qkv, *ctx, *y, *ff;
  uint16_t *x16, *ctx16, *ff16, *qkv16;
  size_t total;
};
EncWs enc_carve(char* base, int64_t T, int H, int I, bool bf16) {
  EncWs w{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += align_up(bytes);
    return p;
  };
  // f32 path: x, qkv, ctx, y, ff (f32).  bf16 path: x, y (f32 residual stream / LayerNorm)
  // and bf16 copies only where the consumer is a bf16 GEMM or the bf16 attention.
  w.x = (float*)take((size_t)T * H * 4);
  w.y = (float*)take((size_t)T * H * 4);
  if (bf16) {
    w.x16 = (uint16_t*)take((size_t)T * H * 2);
    w.qkv16 = (uint16_t*)take((size_t)T * 3 * H * 2);
    w.ctx16 = (uint16_t*)take((size_t)T * H * 2);
    w.ff16 = (uint16_t*)take((size_t)T * I * 2);
  } else {
    w.qkv = (float*)take((size_t)T * 3 * H * 4);
    w.ctx = (float*)take((size_t)T * H * 4);
    w.ff = (float*)take((size_t)T * I * 4);
  }
  w.total = off;
  return w;
}
}  // namespace

extern "C" int tt_bert_workspace_bytes(int64_t T, int32_t H, int32_t I, int32_t prec,
                                       int64_t* bytes) {
  TT_REQUIRE(bytes && T >= 0 && H > 0 && I > 0, "bad arguments");
  *bytes = (int64_t)enc_carve(nullptr, T, H, I, prec == TT_PREC_BF16).total;
  return TT_OK;
}

extern "C" int tt_bert_encode(const tt_bert_model* m, const int32_t* ids, const int32_t* cu_seqlens,
                              int32_t n_seq, int64_t T, int32_t max_len, int32_t prec,
                              float* out_pooled, int64_t ld_out, void* workspace,
                              int64_t workspace_bytes, void* stream) {
  TT_REQUIRE(m != nullptr, "model == NULL");
  TT_REQUIRE(prec == TT_PREC_F32 || prec == TT_PREC_BF16 || prec == TT_PREC_X3,
             "bad precision");
  TT_REQUIRE(n_seq >= 0 && T >= n_seq, "need T >= n_seq >= 0 (no empty sequences)");
  if (n_seq == 0) return TT_OK;
  const int H = m->hidden, I = m->intermediate, NL = m->layers;
  TT_REQUIRE(H > 0 && H <= 1024 && I > 0 && NL >= 0 && m->heads > 0, "bad model dims");
  TT_REQUIRE(max_len <= m->max_positions, "max_len > max_position_embeddings");
  const bool bf = prec == TT_PREC_BF16, x3 = prec == TT_PREC_X3;
  // the f32 path's GEMMs: f32 MFMA, or split-bf16 (x3) on the same f32 operands
  auto gemm32 = [&](const float* A, int64_t lda, const float* W, int64_t ldw, const float* bias,
                    const float* res, int64_t ldr, float* C, int64_t ldc, int32_t M, int32_t N,
                    int32_t K, int32_t act, const uint16_t* wx3) {
    return gemm_f32_impl(A, lda, W, ldw, bias, res, ldr, C, ldc, nullptr, 0, M, N, K, act,
                         stream, x3, x3 ? wx3 : nullptr, 2 * (int64_t)K);
  };
  // bf16 path at H = 384 with row tiles filling the chip: GEMM + LayerNorm fused (k_gemm_ln)
  const bool fuse_ln = bf && H == GL_H && I % 64 == 0 && !gemm_ln_disabled();
  // x3 at H = 384 with x3i weights (wqkv_x3i ...): every GEMM runs on the bf16 kernels with
  // x3i interleaved operands (three MFMAs per 32 k, no split VALU), Wo / W2 fused with their
  // LayerNorm; the producers (embedding LayerNorm, GEMM epilogues, attention) write their
  // outputs x3i interleaved
  bool x3fast = x3 && H == GL_H && I % 64 == 0 && H / m->heads == 32 && !gemm_ln_disabled() &&
                x3c_enabled();
  for (int l = 0; x3fast && l < NL; ++l)
    x3fast = m->layer[l].wqkv_x3i && m->layer[l].wo_x3i && m->layer[l].w1_x3i && m->layer[l].w2_x3i;
  EncWs w = enc_carve((char*)workspace, T, H, I, bf);
  if (!workspace || workspace_bytes < (int64_t)w.total)
    return fail(TT_ERR_WORKSPACE, "tt_bert_encode: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (x3fast) {
    // x3i rows alias the f32 path's buffers (same bytes: [T, 2H] bf16 == [T, H] f32)
    uint16_t* xs = (uint16_t*)w.y;
    uint16_t* cs = (uint16_t*)w.ctx;
    uint16_t* fs = (uint16_t*)w.ff;
    int rc = embed_ln_launch(m, ids, cu_seqlens, n_seq, T, max_len, w.x, xs, H, 1, st);
    if (rc) return rc;
    for (int l = 0; l < NL; ++l) {
      const tt_bert_layer& L = m->layer[l];
      uint16_t* qs = (uint16_t*)w.qkv;  // [T, 6H] x3i rows in the f32 path's [T, 3H] buffer
      rc = gemm_bf16_impl(xs, 2 * H, L.wqkv_x3i, 2 * H, L.bqkv, nullptr, 0, nullptr, 0, qs, 6 * H,
                          (int)T, 3 * H, 2 * H, ACT_NONE, stream, true);
      if (rc) return rc;
      rc = tt_attention_varlen_x3i(qs, 6 * H, cu_seqlens, n_seq, max_len, H, m->heads, cs, 2 * H,
                                   stream);
      if (rc) return rc;
      rc = gemm_ln_impl(cs, 2 * H, L.wo_x3i, 2 * H, L.bo, L.ln1_g, L.ln1_b, m->ln_eps, w.x, H, xs,
                        2 * H, (int)T, H, 2 * H, stream, true);
      if (rc) return rc;
      rc = gemm_bf16_impl(xs, 2 * H, L.w1_x3i, 2 * H, L.b1, nullptr, 0, nullptr, 0, fs, 2 * I,
                          (int)T, I, 2 * H, ACT_GELU, stream, true);
      if (rc) return rc;
      rc = gemm_ln_impl(fs, 2 * I, L.w2_x3i, 2 * I, L.b2, L.ln2_g, L.ln2_b, m->ln_eps, w.x, H, xs,
                        2 * H, (int)T, H, 2 * I, stream, true);
      if (rc) return rc;
    }
    hipLaunchKernelGGL(k_mean_pool, dim3((unsigned)n_seq), dim3(256), 0, st, w.x, (int64_t)H,
                       cu_seqlens, H, out_pooled, ld_out);
    return check_launch("k_mean_pool");
  }
  {
    int rc = embed_ln_launch(m, ids, cu_seqlens, n_seq, T, max_len, w.x, bf ? w.x16 : nullptr, H,
                             0, st);
    if (rc) return rc;
  }
  for (int l = 0; l < NL; ++l) {
    const tt_bert_layer& L = m->layer[l];
    int rc;
    // Q|K|V = x Wqkv^T + b
    rc = bf ? tt_gemm_bf16(w.x16, H, L.wqkv_bf16, H, L.bqkv, nullptr, 0, nullptr, 3 * H, w.qkv16,
                           3 * H, (int)T, 3 * H, H, ACT_NONE, stream)
            : gemm32(w.x, H, L.wqkv, H, L.bqkv, nullptr, 0, w.qkv, 3 * H, (int)T, 3 * H, H,
                     ACT_NONE, L.wqkv_x3);
    if (rc) return rc;
    if (bf && H / m->heads == 32)
      rc = tt_attention_varlen_bf16(w.qkv16, 3 * H, cu_seqlens, n_seq, max_len, H, m->heads,
                                    nullptr, H, w.ctx16, stream);
    else if (bf)
      return fail(TT_ERR_UNSUPPORTED, "tt_bert_encode: bf16 path needs head dim 32");
    else if (H / m->heads == 32)
      rc = tt_attention_varlen(w.qkv, 3 * H, cu_seqlens, n_seq, max_len, H, m->heads,
                               x3 ? TT_PREC_X3 : TT_PREC_F32, w.ctx, H, nullptr, stream);
    else
      rc = tt_attention_varlen_f32(w.qkv, 3 * H, cu_seqlens, n_seq, max_len, H, m->heads, w.ctx,
                                   H, nullptr, stream);
    if (rc) return rc;
    // y = ctx Wo^T + bo + x ; x = LN(y)
    if (fuse_ln) {
      rc = tt_gemm_ln_bf16(w.ctx16, H, L.wo_bf16, H, L.bo, L.ln1_g, L.ln1_b, m->ln_eps, w.x, H,
                           w.x16, H, (int)T, H, H, stream);
      if (rc) return rc;
    } else {
      rc = bf ? tt_gemm_bf16(w.ctx16, H, L.wo_bf16, H, L.bo, w.x, H, w.y, H, nullptr, 0, (int)T, H,
                             H, ACT_NONE, stream)
              : gemm32(w.ctx, H, L.wo, H, L.bo, w.x, H, w.y, H, (int)T, H, H, ACT_NONE, L.wo_x3);
      if (rc) return rc;
      rc = tt_layernorm_f32(w.y, H, L.ln1_g, L.ln1_b, m->ln_eps, w.x, H, bf ? w.x16 : nullptr, H,
                            T, H, stream);
      if (rc) return rc;
    }
    // ff = GELU(x W1^T + b1) ; y = ff W2^T + b2 + x ; x = LN(y)
    rc = bf ? tt_gemm_bf16(w.x16, H, L.w1_bf16, H, L.b1, nullptr, 0, nullptr, I, w.ff16, I, (int)T,
                           I, H, ACT_GELU, stream)
            : gemm32(w.x, H, L.w1, H, L.b1, nullptr, 0, w.ff, I, (int)T, I, H, ACT_GELU, L.w1_x3);
    if (rc) return rc;
    if (fuse_ln) {
      rc = tt_gemm_ln_bf16(w.ff16, I, L.w2_bf16, I, L.b2, L.ln2_g, L.ln2_b, m->ln_eps, w.x, H,
                           w.x16, H, (int)T, H, I, stream);
      if (rc) return rc;
    } else {
      rc = bf ? tt_gemm_bf16(w.ff16, I, L.w2_bf16, I, L.b2, w.x, H, w.y, H, nullptr, 0, (int)T, H,
                             I, ACT_NONE, stream)
              : gemm32(w.ff, I, L.w2, I, L.b2, w.x, H, w.y, H, (int)T, H, I, ACT_NONE, L.w2_x3);
      if (rc) return rc;
      rc = tt_layernorm_f32(w.y, H, L.ln2_g, L.ln2_b, m->ln_eps, w.x, H, bf ? w.x16 : nullptr, H,
                            T, H, stream);
      if (rc) return rc;
    }
  }
  hipLaunchKernelGGL(k_mean_pool, dim3((unsigned)n_seq), dim3(256), 0, st, w.x, (int64_t)H,
                     cu_seqlens, H, out_pooled, ld_out);
  return check_launch("k_mean_pool");
}

extern "C" int tt_item_concat(const float* pooled, int64_t ld_pooled, int32_t Ht,
                              const int32_t* brand_ids, const float* brand_table,
                              const int32_t* cat_ids, const float* cat_table, int32_t C, int64_t b,
                              float* out, int64_t ld_out, uint16_t* out_bf16, void* stream) {
  TT_REQUIRE(b >= 0 && Ht > 0 && C >= 0, "bad sizes");
  if (b == 0) return TT_OK;
  TT_REQUIRE(pooled && out && ld_out >= Ht + 2 * C, "null pointer or ld_out too small");
  hipLaunchKernelGGL(k_item_concat, dim3((unsigned)b), dim3(256), 0, (hipStream_t)stream, pooled,
                     ld_pooled, Ht, brand_ids, brand_table, cat_ids, cat_table, C, out, ld_out,
                     out_bf16, Ht + 2 * C);
  return check_launch("tt_item_concat");
}
