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
// int8 image of the catalog for the single-pass small-batch filter (tt_scan_topk_i8f32):
// per 64-row tile one scale s = max |x| / 127 over the tile's finite values, codes
// n = rint(x / s) in [-127, 127] (0 where s == 0 or x is not finite), padding columns zero.
// Bounds (max-combined into out3, every one rounded UP, accumulated in f64; rows with a
// non-finite value are skipped -- their scores are NaN and never returned):
//   out3[0] >= max_r ||x_r||, out3[1] >= max_r ||x_r - s n_r||, out3[2] >= max_r s ||n_r||.
// One block per tile: pass 1 the tile maximum, pass 2 one wave per row.
__global__ __launch_bounds__(256) void k_i8_image(const float* __restrict__ x, int64_t n, int d,
                                                  int64_t ld, int8_t* __restrict__ codes,
                                                  int64_t ldc, float* __restrict__ scales,
                                                  float* out3) {
  __shared__ float wmax[4];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t r0 = (int64_t)blockIdx.x * 64;
  const int nr = n - r0 < 64 ? (int)(n - r0) : 64;
  float m = 0.0f;
  for (int r = w; r < nr; r += 4) {
    const float* xr = x + (r0 + r) * ld;
    for (int i = lane; i < d; i += 64) {
      const float a = fabsf(xr[i]);
      if (a <= 3.4e38f) m = fmaxf(m, a);  // finite values only
    }
  }
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (lane == 0) wmax[w] = m;
  __syncthreads();
  m = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
  const float s = m / 127.0f;
  if (threadIdx.x == 0) scales[blockIdx.x] = s;
  double bx = 0.0, br = 0.0, bs = 0.0;
  for (int r = w; r < nr; r += 4) {
    const float* xr = x + (r0 + r) * ld;
    int8_t* cr = codes + (r0 + r) * ldc;
    double sx = 0.0, sr = 0.0, sn = 0.0;
    bool fin = true;
    for (int i = lane; i < ldc; i += 64) {
      int c = 0;
      if (i < d) {
        const float v = xr[i];
        fin &= fabsf(v) <= 3.4e38f;
        if (s > 0.0f && fabsf(v) <= 3.4e38f) {
          c = (int)rintf(v / s);
          c = c > 127 ? 127 : c < -127 ? -127 : c;
        }
        const double e = (double)v - (double)s * (double)c;
        sx += (double)v * (double)v;
        sr += e * e;
        sn += (double)c * (double)c;
      }
      cr[i] = (int8_t)c;
    }
    for (int o = 32; o > 0; o >>= 1) {
      sx += __shfl_xor(sx, o, 64);
      sr += __shfl_xor(sr, o, 64);
      sn += __shfl_xor(sn, o, 64);
    }
    if (__ballot(!fin) == 0ull) {
      bx = fmax(bx, sx);
      br = fmax(br, sr);
      bs = fmax(bs, (double)s * (double)s * sn);
    }
  }
  if (lane == 0) {
    // sqrt in f64 of sums of f64 squares (relative error ~1e-15), then rounded up, x1.000001
    atomicMax((unsigned int*)&out3[0], __float_as_uint(f64_up(sqrt(bx) * 1.000001)));
    atomicMax((unsigned int*)&out3[1], __float_as_uint(f64_up(sqrt(br) * 1.000001)));
    atomicMax((unsigned int*)&out3[2], __float_as_uint(f64_up(sqrt(bs) * 1.000001)));
  }
}

// The tiled int8 image (tt_i8_tile) for the register-fed single pass (k_filter_topm_i8r): per
// 16-row block KS = E / 64 pieces of 1 KB, piece s holding, for lane l = 16 g + col, row
// 16 b + col's bytes 64 s + 16 g .. + 15 -- one MFMA operand per 16-B load, 1 KB contiguous
// per wave instruction.  One thread per 16-B chunk; rows past n are zero.
__global__ __launch_bounds__(256) void k_i8_tile(const int8_t* __restrict__ codes, int64_t ldc,
                                                 int64_t n, int ep, int64_t chunks,
                                                 int8_t* __restrict__ tiled) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= chunks) return;
  const int64_t b = c / ep;  // 16-row block (ep chunks of 16 B each)
  const int wi = (int)(c - b * ep), s = wi >> 6, l = wi & 63;
  const int64_t row = 16 * b + (l & 15);
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (row < n) v = *(const uint4*)(codes + row * ldc + 64 * s + 16 * (l >> 4));
  *(uint4*)(tiled + 16 * c) = v;
}
}  // namespace tt

extern "C" int64_t tt_i8_tiled_bytes(int64_t n, int32_t d) {
  const int ep = tt_padded_dim(d);
  if (n < 0 || ep <= 0 || ep % 64 != 0) return -1;
  return (n + 15) / 16 * 16 * (int64_t)ep;
}

extern "C" int tt_i8_tile(const int8_t* codes, int64_t ld_codes, int64_t n, int32_t d,
                          int8_t* tiled, void* stream) {
  using namespace tt;
  const int ep = tt_padded_dim(d);
  TT_REQUIRE(n >= 0 && ep > 0 && ep % 64 == 0, "need n >= 0 and tt_padded_dim(d) % 64 == 0");
  if (n == 0) return TT_OK;
  TT_REQUIRE(codes != nullptr && tiled != nullptr, "null pointer");
  TT_REQUIRE(ld_codes >= ep && ld_codes % 16 == 0 && (uintptr_t)codes % 16 == 0 &&
                 (uintptr_t)tiled % 16 == 0,
             "ld_codes >= tt_padded_dim(d), multiple of 16; 16-B aligned buffers");
  const int64_t chunks = (n + 15) / 16 * ep;
  TT_REQUIRE((chunks + 255) / 256 < (1ll << 31), "too many rows");
  hipLaunchKernelGGL(k_i8_tile, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, codes, ld_codes, n, ep, chunks, tiled);
  return check_launch("tt_i8_tile");
}

extern "C" int tt_i8_image(const float* x, int64_t n, int32_t d, int64_t ld, int8_t* codes,
                           int64_t ld_codes, float* tile_scales, float* out3, void* stream) {
  using namespace tt;
  TT_REQUIRE(n >= 0 && d >= 1 && ld >= d && ld_codes >= d, "need n >= 0, 1 <= d <= ld, ld_codes");
  TT_REQUIRE(out3 != nullptr, "out3 == NULL");
  if (n == 0) return TT_OK;
  TT_REQUIRE(x != nullptr && codes != nullptr && tile_scales != nullptr, "null pointer");
  const int64_t tiles = (n + 63) / 64;
  TT_REQUIRE(tiles < (1ll << 31), "too many rows");
  hipLaunchKernelGGL(k_i8_image, dim3((unsigned)tiles), dim3(256), 0, (hipStream_t)stream, x, n,
                     d, ld, codes, ld_codes, tile_scales, out3);
  return check_launch("tt_i8_image");
}

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
