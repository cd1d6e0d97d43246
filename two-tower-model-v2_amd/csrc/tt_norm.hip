// tt_norm.hip -- row L2 normalisation with numpy-exact norms (gfx950).
//
// Replaces (reference file:line):
//   VectorDatabase.build_index   src/inference/vector_db.py:43-45  x / (||x|| + 1e-8)
//   VectorDatabase.retrieve      vector_db.py:151-153            (query re-normalisation)
//   VectorDatabase.retrieve_batch vector_db.py:188-190
//   F.normalize(p=2, dim=1)      src/models/item_tower.py:209, buyer_tower.py:66,99
//
// One wave per row: the row is staged once in LDS (coalesced 256-B loads), the sum of
// squares is evaluated in numpy's pairwise order (tt_common.hpp), then the row is divided
// by the canonical denominator and written (f32, optional bf16 copy).  HBM-bound:
// 4*d bytes read + 4*d (+2*d) written per row.
#include "tt_common.hpp"

namespace tt {

template <int MAXD>
__global__ __launch_bounds__(256) void k_l2norm_rows(const float* x, int64_t n,
                                                     int d, int64_t ldx, float* y,
                                                     int64_t ldy, uint16_t* yb, int mode,
                                                     int depth) {
  __shared__ float buf[4][MAXD];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* row_s = buf[w];
  for (int64_t row = (int64_t)blockIdx.x * 4 + w; row < n; row += (int64_t)gridDim.x * 4) {
    const float* xr = x + row * ldx;
    for (int i = lane; i < d; i += 64) row_s[i] = xr[i];
    wave_sync();
    float ss;
    if (depth >= 0) {
      ss = pw_sumsq_wave(row_s, d, depth, lane);
    } else {
      ss = lane == 0 ? pw_sumsq_serial(row_s, d) : 0.0f;
      ss = __shfl(ss, 0, 64);
    }
    const float den = norm_denom(ss, mode);
    float* yr = y + row * ldy;
    for (int i = lane; i < d; i += 64) {
      const float v = __fdiv_rn(row_s[i], den);
      yr[i] = v;
      if (yb) yb[row * ldy + i] = f32_to_bf16_rne(v);
    }
    for (int i = d + lane; i < ldy; i += 64) {  // keep the zero-padding invariant
      yr[i] = 0.0f;
      if (yb) yb[row * ldy + i] = 0;
    }
    wave_sync();
  }
}

}  // namespace tt

using namespace tt;

extern "C" int tt_l2norm_rows_f32(const float* x, int64_t n, int32_t d, int64_t ld_x, float* y,
                                  int64_t ld_y, uint16_t* y_bf16, int32_t mode, void* stream) {
  TT_REQUIRE(n >= 0, "n < 0");
  TT_REQUIRE(d >= 1, "d < 1");
  TT_REQUIRE(ld_x >= d && ld_y >= d, "leading dimension < d");
  TT_REQUIRE(mode == TT_NORM_ADD_EPS || mode == TT_NORM_MAX_EPS, "bad mode");
  if (n == 0) return TT_OK;
  TT_REQUIRE(x != nullptr && y != nullptr, "null pointer");
  const int depth = pw_perfect_depth(d);
  const int64_t blocks64 = (n + 3) / 4;
  const unsigned grid = (unsigned)(blocks64 < 8192 ? blocks64 : 8192);
  hipStream_t st = (hipStream_t)stream;
  if (d <= 1024) {
    hipLaunchKernelGGL(k_l2norm_rows<1024>, dim3(grid), dim3(256), 0, st, x, n, d, ld_x, y,
                       ld_y, y_bf16, mode, depth);
  } else if (d <= 4096) {
    hipLaunchKernelGGL(k_l2norm_rows<4096>, dim3(grid), dim3(256), 0, st, x, n, d, ld_x, y,
                       ld_y, y_bf16, mode, depth);
  } else {
    return fail(TT_ERR_UNSUPPORTED, "tt_l2norm_rows_f32: d > 4096");
  }
  return check_launch("tt_l2norm_rows_f32");
}

// ---------------------------------------------------------------------------------------
// Catalog bounds for the bf16 filter's error bound (tt_filter.hip): atomically max-combines
// into out2[0] an upper bound on max ||x_r|| and into out2[1] an upper bound on
// max ||x_r - bf16(x_r)|| over the n rows.  Sums are in any order; the f32 rounding of a
// d-term sum of squares is covered by the (1 + (d+2) 2^-23) factor.  NaN rows are skipped
// (their scores are NaN and never become candidates); Inf propagates (-> every query falls
// back to the exact scan).  One wave per row, HBM-bound (6 bytes per element).
namespace tt {
__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

__global__ __launch_bounds__(256) void k_bf16_bounds(const float* __restrict__ x,
                                                     const uint16_t* __restrict__ xb, int64_t n,
                                                     int d, int64_t ld, float* out2) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float mx = 0.0f, mr = 0.0f;
  for (int64_t row = (int64_t)blockIdx.x * 4 + w; row < n; row += (int64_t)gridDim.x * 4) {
    const float* xr = x + row * ld;
    const uint16_t* br = xb + row * ld;
    float sx = 0.0f, sr = 0.0f;
    for (int i = lane; i < d; i += 64) {
      const float v = xr[i], e = v - bf16_to_f32(br[i]);
      sx = fmaf(v, v, sx);
      sr = fmaf(e, e, sr);
    }
    for (int o = 32; o > 0; o >>= 1) {
      sx += __shfl_xor(sx, o, 64);
      sr += __shfl_xor(sr, o, 64);
    }
    if (sx == sx && sr == sr) {
      mx = fmaxf(mx, sx);
      mr = fmaxf(mr, sr);
    }
  }
  if (lane == 0) {
    const float grow = 1.0f + (float)(d + 2) * 1.1920929e-07f;
    const float bx = sqrtf(mx * grow) * (1.0f + 2.4e-7f), br = sqrtf(mr * grow) * (1.0f + 2.4e-7f);
    // non-negative floats order like their bit patterns
    atomicMax((unsigned int*)&out2[0], __float_as_uint(bx));
    atomicMax((unsigned int*)&out2[1], __float_as_uint(br));
  }
}
}  // namespace tt

extern "C" int tt_bf16_image_bounds(const float* x, const uint16_t* x_bf16, int64_t n,
                                    int32_t d, int64_t ld, float* out2, void* stream) {
  using namespace tt;
  TT_REQUIRE(n >= 0 && d >= 1 && ld >= d, "need n >= 0, 1 <= d <= ld");
  TT_REQUIRE(out2 != nullptr, "out2 == NULL");
  if (n == 0) return TT_OK;
  TT_REQUIRE(x != nullptr && x_bf16 != nullptr, "null pointer");
  const int64_t blocks64 = (n + 3) / 4;
  const unsigned grid = (unsigned)(blocks64 < 4096 ? blocks64 : 4096);
  hipLaunchKernelGGL(k_bf16_bounds, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, x_bf16, n,
                     d, ld, out2);
  return check_launch("tt_bf16_image_bounds");
}

// --------------------------------------------------------------------------- int8 image
// Catalog image of the int8 filter (tt_scan_topk_i8f32): x ~ c o n with per-dimension scales
// c (so that outlier dimensions do not widen every row's step) and n = rne(x / c) in
// [-127, 127].  The bound inputs are MEASURED on the image actually written, so any c is
// sound; c_i = max_r |x_ri| / 127 makes the residual smallest.
namespace tt {
// out[i] = max(out[i], max_r |x_ri|), i < d; NaN elements are skipped (fmaxf)
__global__ __launch_bounds__(256) void k_absmax_cols(const float* __restrict__ x, int64_t n,
                                                     int d, int64_t ld, int64_t rows_per_block,
                                                     float* out) {
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
  for (int i = threadIdx.x; i < d; i += blockDim.x) {
    float m = 0.0f;
    for (int64_t r = r0; r < r1; ++r) m = fmaxf(m, fabsf(x[r * ld + i]));
    atomicMax((unsigned int*)&out[i], __float_as_uint(m));  // non-negative: bit order = order
  }
}

// One wave per row: n = rne(x / c) (0 where c == 0 or x is NaN), padding columns [d, ep) = 0;
// max-combines out3 = {X >= max ||x||, R >= max ||x - c o n||, N >= max ||n||} over non-NaN rows.
__global__ __launch_bounds__(256) void k_quantize_i8(const float* __restrict__ x, int64_t n, int d,
                                                     int ep, int64_t ld,
                                                     const float* __restrict__ colscale,
                                                     int8_t* __restrict__ out, int64_t ld_out,
                                                     float* out3) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float mx = 0.0f, mr = 0.0f;
  int mn = 0;
  for (int64_t row = (int64_t)blockIdx.x * 4 + w; row < n; row += (int64_t)gridDim.x * 4) {
    const float* xr = x + row * ld;
    int8_t* orow = out + row * ld_out;
    float sx = 0.0f, sr = 0.0f;
    int sn = 0;
    for (int i0 = 4 * lane; i0 < ep; i0 += 256) {  // 4 columns per lane: one 32-bit store
      uint32_t packed = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u;
        int m = 0;
        if (i < d) {
          const float v = xr[i], c = colscale[i];
          if (c > 0.0f && v == v) {
            const float r = rintf(v / c);
            m = (int)fminf(127.0f, fmaxf(-127.0f, r));
          }
          const float e = fmaf(-c, (float)m, v);  // one rounding of x - c n
          sx = fmaf(v, v, sx);
          sr = fmaf(e, e, sr);
          sn += m * m;
        }
        packed |= (uint32_t)(uint8_t)(int8_t)m << (8 * u);
      }
      *(uint32_t*)(orow + i0) = packed;
    }
    for (int o = 32; o > 0; o >>= 1) {
      sx += __shfl_xor(sx, o, 64);
      sr += __shfl_xor(sr, o, 64);
      sn += __shfl_xor(sn, o, 64);
    }
    if (sx == sx && sr == sr) {
      mx = fmaxf(mx, sx);
      mr = fmaxf(mr, sr);
      mn = max(mn, sn);
    }
  }
  if (lane == 0) {
    const float grow = 1.0f + (float)(d + 3) * 1.1920929e-07f, up = 1.0f + 2.4e-7f;
    atomicMax((unsigned int*)&out3[0], __float_as_uint(sqrtf(mx * grow) * up));
    atomicMax((unsigned int*)&out3[1], __float_as_uint(sqrtf(mr * grow) * up));
    atomicMax((unsigned int*)&out3[2], __float_as_uint(sqrtf((float)mn) * up));  // mn < 2^24
  }
}
}  // namespace tt

extern "C" int tt_absmax_cols_f32(const float* x, int64_t n, int32_t d, int64_t ld, float* out,
                                  void* stream) {
  using namespace tt;
  TT_REQUIRE(n >= 0 && d >= 1 && ld >= d, "need n >= 0, 1 <= d <= ld");
  TT_REQUIRE(out != nullptr, "out == NULL");
  if (n == 0) return TT_OK;
  TT_REQUIRE(x != nullptr, "x == NULL");
  const int64_t rpb = n < 2048 ? 8 : (n + 2047) / 2048;  // <= 2048 blocks
  const unsigned grid = (unsigned)((n + rpb - 1) / rpb);
  hipLaunchKernelGGL(k_absmax_cols, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, n, d, ld,
                     rpb, out);
  return check_launch("tt_absmax_cols_f32");
}

extern "C" int tt_quantize_i8_rows(const float* x, int64_t n, int32_t d, int64_t ld,
                                   const float* colscale, int8_t* out, int64_t ld_out, float* out3,
                                   void* stream) {
  using namespace tt;
  const int ep = tt_padded_dim(d);
  TT_REQUIRE(ep > 0, "d > 768");
  TT_REQUIRE(n >= 0 && ld >= d && ld_out >= ep && ld_out % 4 == 0, "bad sizes / ld_out % 4");
  TT_REQUIRE(colscale != nullptr && out3 != nullptr, "null pointer");
  if (n == 0) return TT_OK;
  TT_REQUIRE(x != nullptr && out != nullptr && ((uintptr_t)out % 4) == 0, "x/out NULL or unaligned");
  const int64_t blocks64 = (n + 3) / 4;
  const unsigned grid = (unsigned)(blocks64 < 4096 ? blocks64 : 4096);
  hipLaunchKernelGGL(k_quantize_i8, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, n, d, ep, ld,
                     colscale, out, ld_out, out3);
  return check_launch("tt_quantize_i8_rows");
}
