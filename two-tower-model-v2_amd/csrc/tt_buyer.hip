// tt_buyer.hip -- buyer-tower aggregation kernels (gfx950).
//
// Replaces (reference file:line):
//   BuyerTower.weighted_average       src/models/buyer_tower.py:43-68
//   BuyerTower.attention_aggregation  src/models/buyer_tower.py:70-101 (MLP :32-36)
//   EmbeddingEncoder.encode_buyer Mode B (history rows gathered from the resident item
//   embedding table instead of re-encoded): src/inference/encoder.py:286-303
//
// Canonical order (oracle/tt_oracle.c restates it):
//   weighted avg: wsum = (((0+w0)+w1)+...)+1e-8f ; nw_s = w_s/wsum ;
//                 acc_e = (((0 + x0e*nw0) + x1e*nw1) + ...)   (products rounded, no fma)
//   attention:    h_j = relu(fmaf-chain_e(W1[j,e]*x_e) + b1_j); a = fmaf-chain_j(W2_j*h_j)+b2;
//                 c_s = a_s*w_s; m = max c; e_s = expf(c_s-m); Z = sequential sum;
//                 alpha_s = e_s/Z; acc_e = sequential sum_s x_se*alpha_s
//   then F.normalize: acc / max(sqrtf(pairwise_sumsq(acc)), 1e-12).
// One wave per buyer for the weighted average (memory-bound gather of s*d*4 bytes);
// one 256-thread block per buyer for attention.
#include "tt_common.hpp"

namespace tt {

constexpr int BY_MAXD = 1024;

__device__ __forceinline__ void normalize_store(float* row_s, int d, int depth, int lane,
                                                float* out) {
  float ss;
  if (depth >= 0) {
    ss = pw_sumsq_wave(row_s, d, depth, lane);
  } else {
    ss = lane == 0 ? pw_sumsq_serial(row_s, d) : 0.0f;
    ss = __shfl(ss, 0, 64);
  }
  const float den = norm_denom(ss, TT_NORM_MAX_EPS);
  for (int e = lane; e < d; e += 64) out[e] = __fdiv_rn(row_s[e], den);
}

// items: dense [b][s][d] (gather == false) or table rows selected by hist (gather == true).
// One wave per buyer; lane owns elements e = lane + 64 i, i < PER (PER = ceil(d / 64), a
// template so d = 384 holds 6 accumulators, not 16).  The s history rows are walked in order
// (canonical accumulation order), 64 at a time: lane j of a chunk computes that row's
// normalised weight and id once, and __shfl broadcasts them.  The loads of RU consecutive
// rows are issued before their FMAs (RU x PER coalesced 256-B wave loads in flight): one HBM
// round trip per RU rows instead of per row -- the gather was latency-bound (one row per
// round trip: 79 us for 10k buyers x 20 rows x 1.5 KB).  Arithmetic order is unchanged.
template <bool GATHER, int PER>
__global__ __launch_bounds__(256) void k_weighted_avg_l2(const float* __restrict__ src,
                                                         int64_t ld_src, int64_t n_table,
                                                         const int64_t* __restrict__ hist,
                                                         const float* __restrict__ w, int64_t b,
                                                         int s, int d, float* __restrict__ out,
                                                         int64_t ld_out, int depth) {
  constexpr int RU = PER <= 6 ? 4 : PER <= 12 ? 2 : 1;
  __shared__ float buf[4][BY_MAXD];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* row_s = buf[wv];
  for (int64_t bi = (int64_t)blockIdx.x * 4 + wv; bi < b; bi += (int64_t)gridDim.x * 4) {
    const float* wb = w + bi * s;
    float wsum = 0.0f;
    for (int j = 0; j < s; ++j) wsum = wsum + wb[j];
    wsum = wsum + 1e-8f;
    float acc[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) acc[i] = 0.0f;
    for (int j0 = 0; j0 < s; j0 += 64) {
      const int jn = s - j0 < 64 ? s - j0 : 64;
      float my_nw = 0.0f;
      int64_t my_r = -1;
      if (lane < jn) {
        my_nw = __fdiv_rn(wb[j0 + lane], wsum);
        if (GATHER) {
          const int64_t r = hist[bi * s + j0 + lane];
          my_r = (r >= 0 && r < n_table) ? r : -1;
        } else {
          my_r = bi * s + j0 + lane;
        }
      }
      for (int jj0 = 0; jj0 < jn; jj0 += RU) {
        float x[RU][PER], nw[RU];
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          const int jj = jj0 + u < jn ? jj0 + u : jn - 1;  // past jn: a repeat, never added
          nw[u] = __shfl(my_nw, jj, 64);
          const int64_t r = (int64_t)(((uint64_t)(uint32_t)__shfl((int)(my_r >> 32), jj, 64) << 32) |
                                      (uint32_t)__shfl((int)my_r, jj, 64));
          const float* xr = GATHER ? src + r * ld_src : src + r * (int64_t)d;
#pragma unroll
          for (int i = 0; i < PER; ++i) {
            const int e = lane + 64 * i;
            x[u][i] = (r >= 0 && e < d) ? xr[e] : 0.0f;
          }
        }
#pragma unroll
        for (int u = 0; u < RU; ++u)
          if (jj0 + u < jn)
#pragma unroll
            for (int i = 0; i < PER; ++i) acc[i] = acc[i] + __fmul_rn(x[u][i], nw[u]);
      }
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = lane + 64 * i;
      if (e < d) row_s[e] = acc[i];
    }
    wave_sync();
    normalize_store(row_s, d, depth, lane, out + bi * ld_out);
    for (int e = d + lane; e < ld_out; e += 64) out[bi * ld_out + e] = 0.0f;
    wave_sync();
  }
}

// launch k_weighted_avg_l2 with the smallest PER that covers d (d <= BY_MAXD)
template <bool GATHER>
static void launch_weighted_avg(hipStream_t st, const float* src, int64_t ld_src, int64_t n_table,
                                const int64_t* hist, const float* w, int64_t b, int s, int d,
                                float* out, int64_t ld_out, int depth, unsigned grid) {
  const int per = (d + 63) / 64;
#define TT_WAVG(P)                                                                       \
  hipLaunchKernelGGL((k_weighted_avg_l2<GATHER, P>), dim3(grid), dim3(256), 0, st, src, \
                     ld_src, n_table, hist, w, b, s, d, out, ld_out, depth)
  if (per <= 2) TT_WAVG(2);
  else if (per <= 6) TT_WAVG(6);
  else if (per <= 12) TT_WAVG(12);
  else TT_WAVG(16);
#undef TT_WAVG
}

// attention aggregation: one block (256 threads) per buyer; h <= 256, d <= BY_MAXD.
__global__ __launch_bounds__(256) void k_attn_agg_l2(const float* __restrict__ items, int64_t b,
                                                     int s, int d, const float* __restrict__ w,
                                                     const float* __restrict__ W1,
                                                     const float* __restrict__ b1, int h,
                                                     const float* __restrict__ W2,
                                                     const float* __restrict__ b2,
                                                     float* __restrict__ out, int64_t ld_out,
                                                     int depth) {
  __shared__ float xs[BY_MAXD];
  __shared__ float hs[256];
  __shared__ float cs[128];  // s <= 128 (max_interaction_history = 100, config.yaml:14)
  __shared__ float acc_s[BY_MAXD];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int64_t bi = blockIdx.x; bi < b; bi += gridDim.x) {
    const float* xb = items + bi * (int64_t)s * d;
    for (int j = 0; j < s; ++j) {
      for (int e = tid; e < d; e += 256) xs[e] = xb[(int64_t)j * d + e];
      __syncthreads();
      if (tid < h) {
        const float* wr = W1 + (int64_t)tid * d;
        float a = 0.0f;
        for (int e = 0; e < d; ++e) a = fmaf(wr[e], xs[e], a);
        a = a + b1[tid];
        hs[tid] = a > 0.0f ? a : 0.0f;
      }
      __syncthreads();
      if (tid == 0) {
        float a = 0.0f;
        for (int u = 0; u < h; ++u) a = fmaf(W2[u], hs[u], a);
        a = a + b2[0];
        cs[j] = __fmul_rn(a, w[bi * s + j]);
      }
      __syncthreads();
    }
    // softmax over s (every thread computes the same scalars from LDS)
    float m = -__builtin_huge_valf();
    for (int j = 0; j < s; ++j) m = fmaxf(m, cs[j]);
    float z = 0.0f;
    for (int j = 0; j < s; ++j) z = z + expf(cs[j] - m);
    for (int e = tid; e < d; e += 256) {
      float acc = 0.0f;
      for (int j = 0; j < s; ++j) {
        const float alpha = __fdiv_rn(expf(cs[j] - m), z);
        acc = acc + __fmul_rn(xb[(int64_t)j * d + e], alpha);
      }
      acc_s[e] = acc;
    }
    __syncthreads();
    if (wv == 0) {
      normalize_store(acc_s, d, depth, lane, out + bi * ld_out);
      for (int e = d + lane; e < ld_out; e += 64) out[bi * ld_out + e] = 0.0f;
    }
    __syncthreads();
  }
}

// Second stage of the batched attention aggregation (tt_attn_agg_l2_f32_ws): the first MLP
// layer H = relu(X W1^T + b1) [b*s, h] comes from tt_gemm_f32 (f32 MFMA: ~0.5 ms for 10k buyers
// x 20 rows x 768 -> 128, where the fused k_attn_agg_l2's per-buyer serial chains took 59 ms).
// Per buyer, as k_attn_agg_l2 from there on: a_s = fmaf-chain_u(W2_u H_su) + b2, c_s = a_s w_s,
// softmax over s, sum_s alpha_s x_s, F.normalize.
__global__ __launch_bounds__(256) void k_attn_pool_l2(const float* __restrict__ H, int h,
                                                      const float* __restrict__ items, int64_t b,
                                                      int s, int d, const float* __restrict__ w,
                                                      const float* __restrict__ W2,
                                                      const float* __restrict__ b2,
                                                      float* __restrict__ out, int64_t ld_out,
                                                      int depth) {
  __shared__ float cs[128];
  __shared__ float acc_s[BY_MAXD];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int64_t bi = blockIdx.x; bi < b; bi += gridDim.x) {
    const float* xb = items + bi * (int64_t)s * d;
    if (tid < s) {
      const float* hr = H + (bi * s + tid) * (int64_t)h;
      float a = 0.0f;
      for (int u = 0; u < h; ++u) a = fmaf(W2[u], hr[u], a);
      a = a + b2[0];
      cs[tid] = __fmul_rn(a, w[bi * s + tid]);
    }
    __syncthreads();
    float m = -__builtin_huge_valf();
    for (int j = 0; j < s; ++j) m = fmaxf(m, cs[j]);
    float z = 0.0f;
    for (int j = 0; j < s; ++j) z = z + expf(cs[j] - m);
    for (int e = tid; e < d; e += 256) {
      float acc = 0.0f;
      for (int j = 0; j < s; ++j) {
        const float alpha = __fdiv_rn(expf(cs[j] - m), z);
        acc = acc + __fmul_rn(xb[(int64_t)j * d + e], alpha);
      }
      acc_s[e] = acc;
    }
    __syncthreads();
    if (wv == 0) {
      normalize_store(acc_s, d, depth, lane, out + bi * ld_out);
      for (int e = d + lane; e < ld_out; e += 64) out[bi * ld_out + e] = 0.0f;
    }
    __syncthreads();
  }
}

static unsigned grid_for(int64_t units, int64_t per_block, int64_t cap) {
  int64_t g = (units + per_block - 1) / per_block;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (unsigned)g;
}

}  // namespace tt

using namespace tt;

extern "C" int tt_weighted_avg_l2_f32(const float* items, int64_t b, int32_t s, int32_t d,
                                      const float* w, float* out, int64_t ld_out,
                                      void* stream) {
  TT_REQUIRE(b >= 0 && s >= 1 && d >= 1 && ld_out >= d, "bad sizes");
  TT_REQUIRE(d <= BY_MAXD, "d > 1024");
  if (b == 0) return TT_OK;
  launch_weighted_avg<false>((hipStream_t)stream, items, (int64_t)d, (int64_t)0, nullptr, w, b,
                             s, d, out, ld_out, pw_perfect_depth(d), grid_for(b, 4, 16384));
  return check_launch("tt_weighted_avg_l2_f32");
}

extern "C" int tt_gather_weighted_avg_l2_f32(const float* table, int64_t n_table,
                                             int64_t ld_table, int32_t d, const int64_t* hist,
                                             const float* w, int64_t b, int32_t s, float* out,
                                             int64_t ld_out, void* stream) {
  TT_REQUIRE(b >= 0 && s >= 1 && d >= 1 && ld_out >= d && ld_table >= d, "bad sizes");
  TT_REQUIRE(d <= BY_MAXD, "d > 1024");
  if (b == 0) return TT_OK;
  launch_weighted_avg<true>((hipStream_t)stream, table, ld_table, n_table, hist, w, b, s, d,
                            out, ld_out, pw_perfect_depth(d), grid_for(b, 4, 16384));
  return check_launch("tt_gather_weighted_avg_l2_f32");
}

extern "C" int tt_attn_agg_l2_f32(const float* items, int64_t b, int32_t s, int32_t d,
                                  const float* w, const float* W1, const float* b1, int32_t h,
                                  const float* W2, const float* b2, float* out, int64_t ld_out,
                                  void* stream) {
  TT_REQUIRE(b >= 0 && s >= 1 && d >= 1 && ld_out >= d, "bad sizes");
  TT_REQUIRE(d <= BY_MAXD && h >= 1 && h <= 256 && s <= 128, "d>1024 or h>256 or s>128");
  if (b == 0) return TT_OK;
  hipLaunchKernelGGL(k_attn_agg_l2, dim3(grid_for(b, 1, 16384)), dim3(256), 0,
                     (hipStream_t)stream, items, b, s, d, w, W1, b1, h, W2, b2, out, ld_out,
                     pw_perfect_depth(d));
  return check_launch("tt_attn_agg_l2_f32");
}

extern "C" int tt_attn_agg_workspace_bytes(int64_t b, int32_t s, int32_t h, int64_t* bytes) {
  TT_REQUIRE(bytes != nullptr && b >= 0 && s >= 1 && h >= 1, "bad sizes");
  *bytes = (b * s * (int64_t)h * 4 + 255) / 256 * 256;
  return TT_OK;
}

extern "C" int tt_attn_agg_l2_f32_ws(const float* items, int64_t b, int32_t s, int32_t d,
                                     const float* w, const float* W1, const float* b1, int32_t h,
                                     const float* W2, const float* b2, float* out, int64_t ld_out,
                                     void* workspace, int64_t workspace_bytes, void* stream) {
  TT_REQUIRE(b >= 0 && s >= 1 && d >= 1 && ld_out >= d, "bad sizes");
  TT_REQUIRE(d <= BY_MAXD && h >= 1 && h <= 256 && s <= 128, "d>1024 or h>256 or s>128");
  if (b == 0) return TT_OK;
  if (d % 32 != 0)  // tt_gemm_f32 needs K % 32 == 0: the fused one-kernel form
    return tt_attn_agg_l2_f32(items, b, s, d, w, W1, b1, h, W2, b2, out, ld_out, stream);
  int64_t need = 0;
  tt_attn_agg_workspace_bytes(b, s, h, &need);
  if (workspace == nullptr || workspace_bytes < need)
    return fail(TT_ERR_WORKSPACE, "tt_attn_agg_l2_f32_ws: workspace too small");
  TT_REQUIRE(b * s <= 0x7fffffffLL, "b * s must fit int32");
  float* H = (float*)workspace;
  int rc = tt_gemm_f32(items, d, W1, d, b1, nullptr, 0, H, h, nullptr, 0, (int32_t)(b * s), h, d,
                       TT_ACT_RELU, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_attn_pool_l2, dim3(grid_for(b, 1, 16384)), dim3(256), 0,
                     (hipStream_t)stream, H, h, items, b, s, d, w, W2, b2, out, ld_out,
                     pw_perfect_depth(d));
  return check_launch("tt_attn_agg_l2_f32_ws");
}
