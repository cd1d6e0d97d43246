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
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = 1.0f - p * t * __expf(-z * z);  // erf(|x| / sqrt 2)
  return 0.5f * x * (1.0f + (x < 0.0f ? -e : e));
}

typedef __bf16 bf16x2e __attribute__((ext_vector_type(2)));
typedef float f32x2e __attribute__((ext_vector_type(2)));
// two floats -> packed bf16 (round to nearest even) in one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pack_bf16_hw(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2e{a, b}, bf16x2e));
}

// XCD-aware tile order: consecutive logical tiles (same A rows, all N tiles) on one XCD.
__device__ __forceinline__ int enc_xcd_remap(int bid, int nblk) {
  const int q = nblk / 8, r = nblk % 8, x = bid % 8, local = bid / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + local;
}

// Epilogue of one wave's 64x64 accumulator tile, stored straight from registers.  The MFMAs
// compute the TRANSPOSED block D = W . A^T, so lane (g = l >> 4, rl = l & 15) of block (i, j)
// holds C[m = mw0 + 16 i + rl][n = nw0 + 16 j + 4 g + v], v = 0..3: four consecutive columns of
// one row -> one 16-B (f32) / 8-B (bf16) store, bias and residual read as 16-B vectors; the
// 4 j-blocks of a row fill its 128-B (bf16) / 256-B (f32) span back to back.
// C or C16 may be NULL (write only the copy the consumer needs).
template <bool FAST>
__device__ __forceinline__ void gemm_wave_epilogue(f32x4 (&acc)[4][4], int mw0, int nw0,
                                                   int lane, int M, int N,
                                                   const float* __restrict__ bias,
                                                   const float* __restrict__ res, int64_t ldr,
                                                   float* __restrict__ C, int64_t ldc,
                                                   uint16_t* __restrict__ C16, int64_t ldc16,
                                                   int act) {
  const int g = lane >> 4, rl = lane & 15;
  const bool vec = (N % 4) == 0 && (ldc % 4) == 0 && (!res || (ldr % 4) == 0) &&
                   (!C16 || (ldc16 % 4) == 0) && ((uintptr_t)bias % 16) == 0 &&
                   ((uintptr_t)res % 16) == 0 && ((uintptr_t)C % 16) == 0 &&
                   ((uintptr_t)C16 % 8) == 0 && mw0 + 64 <= M && nw0 + 64 <= N;
  if (vec) {
    // full tile: every bias / residual load is issued before the first use, so their
    // latencies overlap (a load-use chain per 16x16 block serialises ~16 L2 round trips)
    f32x4 bv[4], rv[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bv[j] = bias ? *(const f32x4*)(bias + nw0 + 16 * j + 4 * g) : f32x4{0.f, 0.f, 0.f, 0.f};
    if (res) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          rv[i][j] = *(const f32x4*)(res + (int64_t)(mw0 + 16 * i + rl) * ldr + nw0 + 16 * j + 4 * g);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t m = mw0 + 16 * i + rl;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = nw0 + 16 * j + 4 * g;
        f32x4 y = acc[i][j] + bv[j];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (act == ACT_GELU) y[u] = FAST ? gelu_fast(y[u]) : gelu_erf(y[u]);
          else if (act == ACT_RELU) y[u] = y[u] > 0.0f ? y[u] : 0.0f;
        }
        if (res) y = y + rv[i][j];
        if (C) *(f32x4*)(C + m * ldc + n) = y;
        if (C16) *(uint2*)(C16 + m * ldc16 + n) = uint2{pack_bf16_hw(y[0], y[1]),
                                                        pack_bf16_hw(y[2], y[3])};
      }
    }
    return;
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
        if (C16) C16[(int64_t)m * ldc16 + n + u] = f32_to_bf16_rne(y);
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256, 2) void k_gemm(const T* __restrict__ A, int64_t lda,
                                                 const T* __restrict__ W, int64_t ldw,
                                                 const float* __restrict__ bias,
                                                 const float* __restrict__ res, int64_t ldr,
                                                 float* __restrict__ C, int64_t ldc,
                                                 uint16_t* __restrict__ C16, int64_t ldc16,
                                                 int M, int N, int K, int act) {
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
    const int64_t k0 = (int64_t)kt * BK;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = w + 4 * j;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(A + a_off[j] + k0),
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
    enc_lds_barrier();
  }

  gemm_wave_epilogue<sizeof(T) == 2>(acc, m0 + 64 * wm, n0 + 64 * wn, lane, M, N, bias, res, ldr,
                                     C, ldc, C16, ldc16, act);
}

// Large-M bf16 GEMM: persistent blocks (one per CU, 8 waves of 64x64 = 256x128 tiles), a
// 3-slot LDS ring (48 KB stages) fed two stages ahead, ONE barrier per k-stage.  The ring runs
// ACROSS tiles: the last two k-steps of a tile already load the first two stages of the
// block's next tile, so the epilogue's stores and the next tile's pipeline fill overlap
// instead of each launch-sized tile paying its DMA latency and store drain in full (measured:
// the 128x128 kernel spends ~3/4 of its time outside the MFMA loop at K = 384).
// DMA layout / swizzle / fragment reads / epilogue as k_gemm.
constexpr int GB_BM = 256, GB_BN = 128, GB_SLOTS = 3;
constexpr int GB_A_B = GB_BM * 128, GB_W_B = GB_BN * 128, GB_STAGE_B = GB_A_B + GB_W_B;
// timing-only experiment switches (results WRONG when set): tools/exp_filter.sh FILE=tt_encoder
#ifndef TT_GEXP_NOSTORE
#define TT_GEXP_NOSTORE 0  // skip the epilogue
#endif

__global__ __launch_bounds__(512, 1) void k_gemm_big(const uint16_t* __restrict__ A, int64_t lda,
                                                     const uint16_t* __restrict__ W, int64_t ldw,
                                                     const float* __restrict__ bias,
                                                     const float* __restrict__ res, int64_t ldr,
                                                     float* __restrict__ C, int64_t ldc,
                                                     uint16_t* __restrict__ C16, int64_t ldc16,
                                                     int M, int N, int K, int act) {
  constexpr int BK = 64, EPC = 8;
  __shared__ __attribute__((aligned(16))) char smem[GB_SLOTS * GB_STAGE_B];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int n_tn = (N + GB_BN - 1) / GB_BN;
  const int ntiles = ((M + GB_BM - 1) / GB_BM) * n_tn;
  const int nk = K / BK;
  // tile r of this block: logical tile (XCD-contiguous ranges; gridDim.x % 8 == 0 keeps a
  // block on one XCD's range)
  auto tile_of = [&](int r) { return enc_xcd_remap(blockIdx.x + r * gridDim.x, ntiles); };
  const int n_mine = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;

  // DMA: A = 32 pieces of 8 rows x 128 B, W = 16 pieces; wave w issues A pieces w + 8j
  // (j < 4) and W pieces w + 8j (j < 2).  Chunk swizzle as k_gemm.  Offsets of the current
  // (cur) and next (nxt) tile.
  struct Offs {
    int64_t a[4], w[2];
  };
  auto offsets = [&](int lt) __attribute__((always_inline)) {
    Offs o;
    const int m0 = (lt / n_tn) * GB_BM, n0 = (lt % n_tn) * GB_BN;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = 8 * (w + 8 * j) + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      int am = m0 + row;
      am = am < M ? am : M - 1;
      o.a[j] = (int64_t)am * lda + c * EPC;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = 8 * (w + 8 * j) + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      int wr = n0 + row;
      wr = wr < N ? wr : N - 1;
      o.w[j] = (int64_t)wr * ldw + c * EPC;
    }
    return o;
  };
  auto issue = [&](const Offs& o, int kt, int gs) __attribute__((always_inline)) {
    char* st = smem + (gs % GB_SLOTS) * GB_STAGE_B;
    const int64_t k0 = (int64_t)kt * BK;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(A + o.a[j] + k0),
          (__attribute__((address_space(3))) void*)(st + 1024 * (w + 8 * j)), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(W + o.w[j] + k0),
          (__attribute__((address_space(3))) void*)(st + GB_A_B + 1024 * (w + 8 * j)), 16, 0, 0);
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
  issue_next();
  issue_next();
  int gs = 0;  // global stage index of (tile r, k-step 0) = r * nk
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
      if ((kt == 0 && r > 0) || g_i <= gs + kt + 1) enc_wait_vm<0>();
      else enc_wait_vm<6>();
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
    if (!TT_GEXP_NOSTORE)
      gemm_wave_epilogue<true>(acc, (lt / n_tn) * GB_BM + 64 * wm, (lt % n_tn) * GB_BN + 64 * wn,
                               lane, M, N, bias, res, ldr, C, ldc, C16, ldc16, act);
    else if (acc[0][0][0] == 123.456f && acc[3][3][3] == 1.5f) C[0] = acc[1][1][1];
    gs += nk;
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
                                                  int H) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int64_t t = (int64_t)blockIdx.x * 4 + w; t < T; t += (int64_t)gridDim.x * 4) {
    int lo = 0, hi = n_seq;  // sequence: cu[lo] <= t < cu[lo+1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (cu[mid] <= t) lo = mid;
      else hi = mid;
    }
    const int p = (int)(t - cu[lo]);
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
        if (y16) y16[t * H + e] = f32_to_bf16_rne(o);
      }
    }
  }
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
// LDS: K [Lk][32] (rows padded to 144 B f32 / 80 B bf16) and V^T [32][vst] (vst = 128k + 4 f32
// / 128k + 8 bf16 elements): both fragment reads are bank-conflict-free.
template <bool BF, typename TI>
__global__ __launch_bounds__(256) void k_attn32_mfma(const TI* __restrict__ qkv, int64_t ldq,
                                                     const int32_t* __restrict__ cu, int H,
                                                     int heads, float scale,
                                                     float* __restrict__ out, int64_t ldo,
                                                     uint16_t* __restrict__ out16) {
  constexpr int DH = 32;
  constexpr int ES = BF ? 2 : 4;
  constexpr int KROW = DH * ES + 16;
  extern __shared__ __attribute__((aligned(16))) char sm[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, ql = lane & 15;
  const int sq = blockIdx.x / heads, h = blockIdx.x % heads;
  const int t0 = cu[sq], L = cu[sq + 1] - t0;
  const int Lk = (L + 31) & ~31;
  const int vst = ((Lk + 127) & ~127) + (BF ? 8 : 4);
  char* Ks = sm;
  char* Vt = sm + (size_t)Lk * KROW;
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
        if (out16) {
          uint16_t* o16 = out16 + (int64_t)(t0 + q0 + ql) * ldo + h * DH + 16 * db + 4 * g;
#pragma unroll
          for (int v = 0; v < 4; ++v) o16[v] = f32_to_bf16_rne(o[v]);
        }
      }
    }
  }
}

size_t attn32_smem(int max_len, bool bf) {
  const int Lk = (max_len + 31) & ~31;
  const int vst = ((Lk + 127) & ~127) + (bf ? 8 : 4);
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
    for (int t = t0; t < t1; ++t) s += x[(int64_t)t * ldx + e];
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
bool gemm_big_disabled() {
  static const bool off = [] {
    const char* e = getenv("TT_GEMM_BIG");
    return e && e[0] == '0';
  }();
  return off;
}
}  // namespace

extern "C" int tt_gemm_f32(const float* A, int64_t lda, const float* W, int64_t ldw,
                           const float* bias, const float* residual, int64_t ldr, float* C,
                           int64_t ldc, uint16_t* C_bf16, int64_t ldc16, int32_t M, int32_t N,
                           int32_t K, int32_t act, void* stream) {
  TT_REQUIRE(M >= 0 && N >= 0 && K >= 0, "negative size");
  if (M == 0 || N == 0) return TT_OK;
  if (K % GemmElt<float>::BK != 0)
    return fail(TT_ERR_UNSUPPORTED, "tt_gemm_f32: need K % 32 == 0");
  TT_REQUIRE(A && W && (C || C_bf16), "null pointer");
  TT_REQUIRE(lda % 4 == 0 && ldw % 4 == 0 && ((uintptr_t)A % 16) == 0 && ((uintptr_t)W % 16) == 0,
             "A/W must be 16-B aligned with lda, ldw % 4 == 0");
  TT_REQUIRE(act >= 0 && act <= 2, "bad activation");
  const int nblk = ((M + GM_BM - 1) / GM_BM) * ((N + GM_BN - 1) / GM_BN);
  hipLaunchKernelGGL(k_gemm<float>, dim3(nblk), dim3(256), 0, (hipStream_t)stream, A, lda, W, ldw,
                     bias, residual, ldr, C, ldc, C_bf16, ldc16, M, N, K, act);
  return check_launch("tt_gemm_f32");
}

extern "C" int tt_gemm_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw,
                            const float* bias, const float* residual, int64_t ldr, float* C,
                            int64_t ldc, uint16_t* C_bf16, int64_t ldc16, int32_t M, int32_t N,
                            int32_t K, int32_t act, void* stream) {
  TT_REQUIRE(M >= 0 && N >= 0 && K >= 0, "negative size");
  if (M == 0 || N == 0) return TT_OK;
  if (K % GemmElt<uint16_t>::BK != 0)
    return fail(TT_ERR_UNSUPPORTED, "tt_gemm_bf16: need K % 64 == 0");
  TT_REQUIRE(A && W && (C || C_bf16), "null pointer");
  TT_REQUIRE(lda % 8 == 0 && ldw % 8 == 0 && ((uintptr_t)A % 16) == 0 && ((uintptr_t)W % 16) == 0,
             "A/W must be 16-B aligned with lda, ldw % 8 == 0");
  TT_REQUIRE(act >= 0 && act <= 2, "bad activation");
  // large M: the persistent 256x128 ring kernel (one block per CU) once there are at least
  // two tiles per CU
  const int nbig = ((M + GB_BM - 1) / GB_BM) * ((N + GB_BN - 1) / GB_BN);
  const int ncu = enc_device_cus();
  if (nbig >= 2 * ncu && !gemm_big_disabled()) {
    hipLaunchKernelGGL(k_gemm_big, dim3(ncu), dim3(512), 0, (hipStream_t)stream, A, lda, W, ldw,
                       bias, residual, ldr, C, ldc, C_bf16, ldc16, M, N, K, act);
    return check_launch("tt_gemm_bf16(256x128)");
  }
  const int nblk = ((M + GM_BM - 1) / GM_BM) * ((N + GM_BN - 1) / GM_BN);
  hipLaunchKernelGGL(k_gemm<uint16_t>, dim3(nblk), dim3(256), 0, (hipStream_t)stream, A, lda, W,
                     ldw, bias, residual, ldr, C, ldc, C_bf16, ldc16, M, N, K, act);
  return check_launch("tt_gemm_bf16");
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

extern "C" int tt_attention_varlen(const float* qkv, int64_t ld_qkv, const int32_t* cu_seqlens,
                                   int32_t n_seq, int32_t max_len, int32_t H, int32_t heads,
                                   int32_t prec, float* out, int64_t ld_out, uint16_t* out_bf16,
                                   void* stream) {
  TT_REQUIRE(n_seq >= 0 && heads >= 1 && H % heads == 0, "bad n_seq / heads");
  TT_REQUIRE(prec == TT_PREC_F32 || prec == TT_PREC_BF16, "bad precision");
  if (n_seq == 0) return TT_OK;
  TT_REQUIRE(max_len >= 1 && max_len <= 512, "max_len must be in [1, 512]");
  TT_REQUIRE(qkv && cu_seqlens && out, "null pointer");
  TT_REQUIRE(ld_qkv % 4 == 0 && ld_out % 4 == 0 && H % 4 == 0 && ((uintptr_t)qkv % 16) == 0 &&
                 ((uintptr_t)out % 16) == 0, "qkv/out must be 16-B aligned rows");
  if (H / heads != 32)
    return fail(TT_ERR_UNSUPPORTED, "tt_attention_varlen: MFMA path needs head dim 32");
  const bool bf = prec == TT_PREC_BF16;
  const size_t smem = attn32_smem(max_len, bf);
  const void* fn = bf ? (const void*)k_attn32_mfma<true, float> : (const void*)k_attn32_mfma<false, float>;
  if (smem > 64 * 1024 &&
      hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem) != hipSuccess)
    return fail(TT_ERR_LAUNCH, "hipFuncSetAttribute(max dynamic LDS)");
  const float scale = 1.0f / sqrtf(32.0f);
  const dim3 grid((unsigned)(n_seq * heads));
  if (bf)
    hipLaunchKernelGGL((k_attn32_mfma<true, float>), grid, dim3(256), smem, (hipStream_t)stream, qkv,
                       ld_qkv, cu_seqlens, H, heads, scale, out, ld_out, out_bf16);
  else
    hipLaunchKernelGGL((k_attn32_mfma<false, float>), grid, dim3(256), smem, (hipStream_t)stream, qkv,
                       ld_qkv, cu_seqlens, H, heads, scale, out, ld_out, out_bf16);
  return check_launch("tt_attention_varlen");
}

extern "C" int tt_attention_varlen_bf16(const uint16_t* qkv, int64_t ld_qkv,
                                        const int32_t* cu_seqlens, int32_t n_seq,
                                        int32_t max_len, int32_t H, int32_t heads, float* out,
                                        int64_t ld_out, uint16_t* out_bf16, void* stream) {
  TT_REQUIRE(n_seq >= 0 && heads >= 1 && H % heads == 0, "bad n_seq / heads");
  if (n_seq == 0) return TT_OK;
  TT_REQUIRE(max_len >= 1 && max_len <= 512, "max_len must be in [1, 512]");
  TT_REQUIRE(qkv && cu_seqlens && (out || out_bf16), "null pointer");
  TT_REQUIRE(ld_qkv % 8 == 0 && ld_out % 4 == 0 && H % 8 == 0 && ((uintptr_t)qkv % 16) == 0,
             "qkv must be 16-B aligned rows");
  if (H / heads != 32)
    return fail(TT_ERR_UNSUPPORTED, "tt_attention_varlen_bf16: head dim must be 32");
  const size_t smem = attn32_smem(max_len, true);
  const void* fn = (const void*)k_attn32_mfma<true, uint16_t>;
  if (smem > 64 * 1024 &&
      hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem) != hipSuccess)
    return fail(TT_ERR_LAUNCH, "hipFuncSetAttribute(max dynamic LDS)");
  hipLaunchKernelGGL((k_attn32_mfma<true, uint16_t>), dim3((unsigned)(n_seq * heads)), dim3(256),
                     smem, (hipStream_t)stream, qkv, ld_qkv, cu_seqlens, H, heads,
                     1.0f / sqrtf(32.0f), out, ld_out, out_bf16);
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
  TT_REQUIRE(prec == TT_PREC_F32 || prec == TT_PREC_BF16, "bad precision");
  TT_REQUIRE(n_seq >= 0 && T >= n_seq, "need T >= n_seq >= 0 (no empty sequences)");
  if (n_seq == 0) return TT_OK;
  const int H = m->hidden, I = m->intermediate, NL = m->layers;
  TT_REQUIRE(H > 0 && H <= 1024 && I > 0 && NL >= 0 && m->heads > 0, "bad model dims");
  TT_REQUIRE(max_len <= m->max_positions, "max_len > max_position_embeddings");
  const bool bf = prec == TT_PREC_BF16;
  EncWs w = enc_carve((char*)workspace, T, H, I, bf);
  if (!workspace || workspace_bytes < (int64_t)w.total)
    return fail(TT_ERR_WORKSPACE, "tt_bert_encode: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  {
    const int64_t b = (T + 3) / 4;
    hipLaunchKernelGGL(k_embed_ln, dim3((unsigned)(b < 16384 ? b : 16384)), dim3(256), 0, st, ids,
                       cu_seqlens, n_seq, T, m->word_emb, m->vocab, m->pos_emb, m->type_emb,
                       m->emb_ln_g, m->emb_ln_b, m->ln_eps, w.x, bf ? w.x16 : nullptr, H);
    int rc = check_launch("k_embed_ln");
    if (rc) return rc;
  }
  for (int l = 0; l < NL; ++l) {
    const tt_bert_layer& L = m->layer[l];
    int rc;
    // Q|K|V = x Wqkv^T + b
    rc = bf ? tt_gemm_bf16(w.x16, H, L.wqkv_bf16, H, L.bqkv, nullptr, 0, nullptr, 3 * H, w.qkv16,
                           3 * H, (int)T, 3 * H, H, ACT_NONE, stream)
            : tt_gemm_f32(w.x, H, L.wqkv, H, L.bqkv, nullptr, 0, w.qkv, 3 * H, nullptr, 0, (int)T,
                          3 * H, H, ACT_NONE, stream);
    if (rc) return rc;
    if (bf && H / m->heads == 32)
      rc = tt_attention_varlen_bf16(w.qkv16, 3 * H, cu_seqlens, n_seq, max_len, H, m->heads,
                                    nullptr, H, w.ctx16, stream);
    else if (bf)
      return fail(TT_ERR_UNSUPPORTED, "tt_bert_encode: bf16 path needs head dim 32");
    else if (H / m->heads == 32)
      rc = tt_attention_varlen(w.qkv, 3 * H, cu_seqlens, n_seq, max_len, H, m->heads, prec, w.ctx,
                               H, nullptr, stream);
    else
      rc = tt_attention_varlen_f32(w.qkv, 3 * H, cu_seqlens, n_seq, max_len, H, m->heads, w.ctx,
                                   H, nullptr, stream);
    if (rc) return rc;
    // y = ctx Wo^T + bo + x ; x = LN(y)
    rc = bf ? tt_gemm_bf16(w.ctx16, H, L.wo_bf16, H, L.bo, w.x, H, w.y, H, nullptr, 0, (int)T, H, H,
                           ACT_NONE, stream)
            : tt_gemm_f32(w.ctx, H, L.wo, H, L.bo, w.x, H, w.y, H, nullptr, 0, (int)T, H, H,
                          ACT_NONE, stream);
    if (rc) return rc;
    rc = tt_layernorm_f32(w.y, H, L.ln1_g, L.ln1_b, m->ln_eps, w.x, H, bf ? w.x16 : nullptr, H, T,
                          H, stream);
    if (rc) return rc;
    // ff = GELU(x W1^T + b1) ; y = ff W2^T + b2 + x ; x = LN(y)
    rc = bf ? tt_gemm_bf16(w.x16, H, L.w1_bf16, H, L.b1, nullptr, 0, nullptr, I, w.ff16, I, (int)T,
                           I, H, ACT_GELU, stream)
            : tt_gemm_f32(w.x, H, L.w1, H, L.b1, nullptr, 0, w.ff, I, nullptr, 0, (int)T, I, H,
                          ACT_GELU, stream);
    if (rc) return rc;
    rc = bf ? tt_gemm_bf16(w.ff16, I, L.w2_bf16, I, L.b2, w.x, H, w.y, H, nullptr, 0, (int)T, H, I,
                           ACT_NONE, stream)
            : tt_gemm_f32(w.ff, I, L.w2, I, L.b2, w.x, H, w.y, H, nullptr, 0, (int)T, H, I, ACT_NONE,
                          stream);
    if (rc) return rc;
    rc = tt_layernorm_f32(w.y, H, L.ln2_g, L.ln2_b, m->ln_eps, w.x, H, bf ? w.x16 : nullptr, H, T,
                          H, stream);
    if (rc) return rc;
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
