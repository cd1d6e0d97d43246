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
