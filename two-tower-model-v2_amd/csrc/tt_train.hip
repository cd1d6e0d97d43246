// tt_train.hip -- backward / optimizer kernels of the configs[4] training step (gfx950).
//
// The reference trains the item-tower projection head + categorical embeddings and the
// buyer-tower attention MLP with InfoNCE (src/training/trainer.py:74-243 -> losses.py:20-79;
// the text encoder is frozen, item_tower.py:40-42) and Adam (trainer.py:49-52).  The GEMMs of
// forward and backward run on tt_gemm_f32 / tt_gemm_bf16 (tt_encoder.hip); this file holds
// the row-wise and reduction pieces between them:
//   tt_l2norm_backward_f32   F.normalize backward (item_tower.py:209, buyer_tower.py:99)
//   tt_transpose_f32         [rows, cols] -> [cols, ld] (zero-padded K for dW = dY^T X GEMMs)
//   tt_col_sum_f32           bias gradients (sum over rows)
//   tt_relu_backward_f32     dH *= (H > 0)
//   tt_attn_pool_fwd/bwd     the attention-aggregation head after the Linear(E,128)+ReLU
//                            GEMM: a = H.W2 + b2, c = a * w, softmax over S, sum alpha x, L2
//                            (buyer_tower.py:85-99), and its backward to dW2, db2, dH
//   tt_embedding_backward_f32  scatter-add of embedding-row gradients (padding_idx 0 skipped,
//                            nn.Embedding(padding_idx=0), item_tower.py:85-97)
//   tt_adam_f32              torch.optim.Adam step (bias-corrected, L2-free), fused
#include "tt_common.hpp"

namespace tt {

__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// dy = (dz - z (z . dz)) / ||y||  if ||y|| > eps, else dz / eps   (z = y / max(||y||, eps))
__global__ __launch_bounds__(256) void k_l2norm_bwd(const float* __restrict__ y, int64_t ldy,
                                                    const float* __restrict__ z, int64_t ldz,
                                                    const float* __restrict__ dz, int64_t lddz,
                                                    int64_t n, int d, float* __restrict__ dy,
                                                    int64_t lddy) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + w; r < n; r += (int64_t)gridDim.x * 4) {
    float ss = 0.0f, zd = 0.0f;
    for (int e = lane; e < d; e += 64) {
      const float yv = y[r * ldy + e];
      ss = fmaf(yv, yv, ss);
      zd = fmaf(z[r * ldz + e], dz[r * lddz + e], zd);
    }
    ss = wave_sum(ss);
    zd = wave_sum(zd);
    const float nrm = sqrtf(ss);
    for (int e = lane; e < d; e += 64) {
      const float g = dz[r * lddz + e];
      dy[r * lddy + e] = nrm > 1e-12f ? (g - z[r * ldz + e] * zd) / nrm : g / 1e-12f;
    }
  }
}

__global__ __launch_bounds__(256) void k_transpose(const float* __restrict__ x, int64_t ldx,
                                                   int rows, int cols, float* __restrict__ t,
                                                   int ldt) {
  __shared__ float tile[32][33];
  const int r0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int j = ty; j < 32; j += 8) {
    const int r = r0 + j, c = c0 + tx;
    tile[j][tx] = (r < rows && c < cols) ? x[(int64_t)r * ldx + c] : 0.0f;
  }
  __syncthreads();
  for (int j = ty; j < 32; j += 8) {
    const int c = c0 + j, r = r0 + tx;
    if (c < cols && r < ldt) t[(int64_t)c * ldt + r] = tile[tx][j];
  }
}

// out[c] (+)= sum_r x[r][c]: block per 64 columns, 4 row-strided waves
// Column sums (bias gradients, 1^T . dY): grid = (column blocks of 64, row chunks of
// CS_ROWS); a block reduces its chunk in LDS and adds the partial to out[c] with one float
// atomic per column (out pre-zeroed by the host unless accumulating).  A grid over columns
// only had 2-12 blocks for the head / attention shapes and walked 51k rows serially (1-5 ms);
// the atomics make the summation order run-dependent (ulp-level, within the tests' rtol).
constexpr int CS_ROWS = 256;
__global__ __launch_bounds__(256) void k_col_sum(const float* __restrict__ x, int64_t ldx,
                                                 int64_t rows, int cols, float* __restrict__ out) {
  __shared__ float part[4][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = blockIdx.x * 64 + lane;
  const int64_t r0 = (int64_t)blockIdx.y * CS_ROWS;
  const int64_t r1 = r0 + CS_ROWS < rows ? r0 + CS_ROWS : rows;
  float s = 0.0f;
  if (c < cols)
    for (int64_t r = r0 + w; r < r1; r += 4) s += x[r * ldx + c];
  part[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < cols)
    atomicAdd(out + c, (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]));
}

__global__ void k_relu_bwd(float* __restrict__ dh, const float* __restrict__ h, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    if (!(h[i] > 0.0f)) dh[i] = 0.0f;
}

// nn.Dropout(p) with a given keep mask (item_tower.py:61, active under model.train(),
// trainer.py:167): x[i] = keep[i] ? x[i] * scale : 0, scale = 1 / (1 - p).  The same call on
// the incoming gradient is the backward.
__global__ void k_dropout(float* __restrict__ x, const uint8_t* __restrict__ keep, float scale,
                          int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    x[i] = keep[i] ? x[i] * scale : 0.0f;
}

// Attention pooling, one block per buyer (S <= 128, hidden Hd <= 256, E <= 1024):
//   a_s = H_s . W2 + b2 ; c_s = a_s * w_s ; alpha = softmax(c) ; o = sum_s alpha_s x_s ;
//   z = o / max(||o||, 1e-12).  Saves alpha [B, S] and ||o|| [B] for the backward.
__global__ __launch_bounds__(256) void k_attn_pool_fwd(
    const float* __restrict__ H, int Hd, const float* __restrict__ W2, float b2,
    const float* __restrict__ w, const float* __restrict__ x, int S, int E,
    float* __restrict__ alpha, float* __restrict__ onorm, float* __restrict__ z, int64_t ldz) {
  __shared__ float cs[128];
  __shared__ float red[4];
  const int b = blockIdx.x, tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  for (int s = wv; s < S; s += 4) {  // wave per position
    const float* h = H + ((int64_t)b * S + s) * Hd;
    float a = 0.0f;
    for (int j = lane; j < Hd; j += 64) a = fmaf(h[j], W2[j], a);
    a = wave_sum(a);
    if (lane == 0) cs[s] = (a + b2) * w[(int64_t)b * S + s];
  }
  __syncthreads();
  float m = -__builtin_huge_valf();
  for (int s = 0; s < S; ++s) m = fmaxf(m, cs[s]);
  float sum = 0.0f;
  for (int s = 0; s < S; ++s) sum += expf(cs[s] - m);
  const float inv = 1.0f / sum;
  if (tid < S) alpha[(int64_t)b * S + tid] = expf(cs[tid] - m) * inv;
  // o = sum alpha x ; ||o||
  const float* xb = x + (int64_t)b * S * E;
  float ss = 0.0f;
  float ov[4];
  for (int i = 0; i < 4; ++i) {
    const int e = tid + 256 * i;
    float o = 0.0f;
    if (e < E)
      for (int s = 0; s < S; ++s) o = fmaf(expf(cs[s] - m) * inv, xb[(int64_t)s * E + e], o);
    ov[i] = o;
    ss = fmaf(o, o, ss);
  }
  ss = wave_sum(ss);
  if (lane == 0) red[wv] = ss;
  __syncthreads();
  const float nrm = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
  if (tid == 0) onorm[b] = nrm;
  const float den = fmaxf(nrm, 1e-12f);
  for (int i = 0; i < 4; ++i) {
    const int e = tid + 256 * i;
    if (e < E) z[(int64_t)b * ldz + e] = ov[i] / den;
  }
}

// Backward of k_attn_pool_fwd: block per buyer.  do = normalize backward(dz);
// dalpha_s = do . x_s ; dc_s = alpha_s (dalpha_s - sum_t alpha_t dalpha_t) ; da_s = dc_s w_s.
// Writes da [B*S] (dW2 = da^T H and db2 = sum da are reductions done after) and
// dH[bs][j] = da_bs * W2[j] (the ReLU mask is applied by tt_relu_backward_f32).
__global__ __launch_bounds__(256) void k_attn_pool_bwd(
    const float* __restrict__ dz, int64_t lddz, const float* __restrict__ z, int64_t ldz,
    const float* __restrict__ onorm, const float* __restrict__ alpha,
    const float* __restrict__ w, const float* __restrict__ x, int S, int E,
    const float* __restrict__ W2, int Hd, float* __restrict__ da, float* __restrict__ dH) {
  __shared__ float dov[1024];
  __shared__ float dal[128];
  __shared__ float red[4];
  const int b = blockIdx.x, tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const float nrm = onorm[b];
  float zd = 0.0f;
  for (int e = tid; e < E; e += 256) zd = fmaf(z[(int64_t)b * ldz + e], dz[(int64_t)b * lddz + e], zd);
  zd = wave_sum(zd);
  if (lane == 0) red[wv] = zd;
  __syncthreads();
  zd = (red[0] + red[1]) + (red[2] + red[3]);
  for (int e = tid; e < E; e += 256) {
    const float g = dz[(int64_t)b * lddz + e];
    dov[e] = nrm > 1e-12f ? (g - z[(int64_t)b * ldz + e] * zd) / nrm : g / 1e-12f;
  }
  __syncthreads();
  const float* xb = x + (int64_t)b * S * E;
  for (int s = wv; s < S; s += 4) {
    float d = 0.0f;
    for (int e = lane; e < E; e += 64) d = fmaf(dov[e], xb[(int64_t)s * E + e], d);
    d = wave_sum(d);
    if (lane == 0) dal[s] = d;
  }
  __syncthreads();
  float adot = 0.0f;
  for (int s = 0; s < S; ++s) adot = fmaf(alpha[(int64_t)b * S + s], dal[s], adot);
  for (int s = 0; s < S; ++s) {
    const float al = alpha[(int64_t)b * S + s];
    const float das = al * (dal[s] - adot) * w[(int64_t)b * S + s];
    if (tid == 0) da[(int64_t)b * S + s] = das;
    for (int j = tid; j < Hd; j += 256) dH[((int64_t)b * S + s) * Hd + j] = das * W2[j];
  }
}

// dW2[j] = sum_i da_i H_ij (rows strided over 4 waves, lane = column block of 64); db2 = sum da
__global__ __launch_bounds__(256) void k_weighted_col_sum(const float* __restrict__ H, int Hd,
                                                          const float* __restrict__ da,
                                                          int64_t rows, float* __restrict__ dW2,
                                                          float* __restrict__ db2) {
  // dW2[j] = sum_r da[r] H[r][j], db2 = sum_r da[r]; grid (column blocks, row chunks) with
  // float atomics, as k_col_sum (outputs pre-zeroed by the host)
  __shared__ float part[4][64];
  __shared__ float pb[4];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int j = blockIdx.x * 64 + lane;
  const int64_t r0 = (int64_t)blockIdx.y * CS_ROWS;
  const int64_t r1 = r0 + CS_ROWS < rows ? r0 + CS_ROWS : rows;
  float s = 0.0f, sb = 0.0f;
  for (int64_t r = r0 + w; r < r1; r += 4) {
    const float d = da[r];
    if (j < Hd) s = fmaf(d, H[r * Hd + j], s);
    sb += d;
  }
  part[w][lane] = s;
  if (lane == 0) pb[w] = sb;
  __syncthreads();
  if (w == 0 && j < Hd)
    atomicAdd(dW2 + j, (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]));
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(db2, (pb[0] + pb[1]) + (pb[2] + pb[3]));
}

__global__ void k_embedding_bwd(const float* __restrict__ g, int64_t ldg,
                                const int32_t* __restrict__ ids, int64_t n, int C,
                                float* __restrict__ table_grad) {
  const int64_t r = blockIdx.x;
  if (r >= n) return;
  const int id = ids[r];
  if (id <= 0) return;  // padding_idx 0 gets no gradient
  for (int c = threadIdx.x; c < C; c += blockDim.x)
    atomicAdd(&table_grad[(int64_t)id * C + c], g[r * ldg + c]);
}

// torch.optim.Adam (weight_decay 0, amsgrad False): m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2
// p -= lr * (m / (1 - b1^t)) / (sqrt(v / (1 - b2^t)) + eps)
__global__ void k_adam(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps,
                       float bc1, float bc2) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i];
    const float mi = b1 * m[i] + (1.0f - b1) * gi;
    const float vi = b2 * v[i] + (1.0f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    p[i] = p[i] - lr * (mi / bc1) / (sqrtf(vi / bc2) + eps);
  }
}

unsigned grid_for(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (unsigned)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

}  // namespace tt

using namespace tt;

extern "C" int tt_l2norm_backward_f32(const float* y, int64_t ldy, const float* z, int64_t ldz,
                                      const float* dz, int64_t lddz, int64_t n, int32_t d,
                                      float* dy, int64_t lddy, void* stream) {
  TT_REQUIRE(n >= 0 && d >= 1, "bad sizes");
  if (n == 0) return TT_OK;
  TT_REQUIRE(y && z && dz && dy, "null pointer");
  hipLaunchKernelGGL(k_l2norm_bwd, dim3(grid_for((n + 3) / 4 * 256)), dim3(256), 0,
                     (hipStream_t)stream, y, ldy, z, ldz, dz, lddz, n, d, dy, lddy);
  return check_launch("tt_l2norm_backward_f32");
}

extern "C" int tt_transpose_f32(const float* x, int64_t ldx, int32_t rows, int32_t cols, float* t,
                                int32_t ldt, void* stream) {
  TT_REQUIRE(rows >= 0 && cols >= 0 && ldt >= rows, "bad sizes (ldt < rows)");
  if (rows == 0 || cols == 0) return TT_OK;
  TT_REQUIRE(x && t, "null pointer");
  const dim3 g((unsigned)((ldt + 31) / 32), (unsigned)((cols + 31) / 32));
  hipLaunchKernelGGL(k_transpose, g, dim3(256), 0, (hipStream_t)stream, x, ldx, rows, cols, t, ldt);
  return check_launch("tt_transpose_f32");
}

extern "C" int tt_col_sum_f32(const float* x, int64_t ldx, int64_t rows, int32_t cols, float* out,
                              int32_t accumulate, void* stream) {
  TT_REQUIRE(rows >= 0 && cols >= 0, "bad sizes");
  if (cols == 0) return TT_OK;
  TT_REQUIRE(x && out, "null pointer");
  if (!accumulate && hipMemsetAsync(out, 0, (size_t)cols * 4, (hipStream_t)stream) != hipSuccess)
    return fail(TT_ERR_LAUNCH, "tt_col_sum_f32: hipMemsetAsync");
  if (rows == 0) return TT_OK;
  const int64_t chunks = (rows + CS_ROWS - 1) / CS_ROWS;
  TT_REQUIRE(chunks <= 65535, "rows > 65535 * 256");
  hipLaunchKernelGGL(k_col_sum, dim3((unsigned)((cols + 63) / 64), (unsigned)chunks), dim3(256), 0,
                     (hipStream_t)stream, x, ldx, rows, cols, out);
  return check_launch("tt_col_sum_f32");
}

extern "C" int tt_relu_backward_f32(float* dh, const float* h, int64_t n, void* stream) {
  TT_REQUIRE(n >= 0, "n < 0");
  if (n == 0) return TT_OK;
  TT_REQUIRE(dh && h, "null pointer");
  hipLaunchKernelGGL(k_relu_bwd, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, dh, h, n);
  return check_launch("tt_relu_backward_f32");
}

extern "C" int tt_dropout_apply_f32(float* x, const uint8_t* keep, float scale, int64_t n,
                                    void* stream) {
  TT_REQUIRE(n >= 0, "n < 0");
  if (n == 0) return TT_OK;
  TT_REQUIRE(x && keep, "null pointer");
  hipLaunchKernelGGL(k_dropout, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, keep,
                     scale, n);
  return check_launch("tt_dropout_apply_f32");
}

extern "C" int tt_attn_pool_fwd_f32(const float* H, int32_t Hd, const float* W2, float b2,
                                    const float* w, const float* x, int64_t B, int32_t S,
                                    int32_t E, float* alpha, float* onorm, float* z, int64_t ldz,
                                    void* stream) {
  TT_REQUIRE(B >= 0 && S >= 1 && S <= 128 && E >= 1 && E <= 1024 && Hd >= 1,
             "need 1 <= S <= 128, 1 <= E <= 1024");
  if (B == 0) return TT_OK;
  TT_REQUIRE(H && W2 && w && x && alpha && onorm && z, "null pointer");
  hipLaunchKernelGGL(k_attn_pool_fwd, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, H, Hd,
                     W2, b2, w, x, S, E, alpha, onorm, z, ldz);
  return check_launch("tt_attn_pool_fwd_f32");
}

extern "C" int tt_attn_pool_bwd_f32(const float* dz, int64_t lddz, const float* z, int64_t ldz,
                                    const float* onorm, const float* alpha, const float* w,
                                    const float* x, int64_t B, int32_t S, int32_t E,
                                    const float* H, const float* W2, int32_t Hd, float* dW2,
                                    float* db2, float* dH, float* da_ws, void* stream) {
  TT_REQUIRE(B >= 0 && S >= 1 && S <= 128 && E >= 1 && E <= 1024 && Hd >= 1,
             "need 1 <= S <= 128, 1 <= E <= 1024");
  if (B == 0) return TT_OK;
  TT_REQUIRE(dz && z && onorm && alpha && w && x && H && W2 && dW2 && db2 && dH && da_ws,
             "null pointer");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_attn_pool_bwd, dim3((unsigned)B), dim3(256), 0, st, dz, lddz, z, ldz,
                     onorm, alpha, w, x, S, E, W2, Hd, da_ws, dH);
  int rc = check_launch("k_attn_pool_bwd");
  if (rc) return rc;
  if (hipMemsetAsync(dW2, 0, (size_t)Hd * 4, st) != hipSuccess ||
      hipMemsetAsync(db2, 0, 4, st) != hipSuccess)
    return fail(TT_ERR_LAUNCH, "tt_attn_pool_bwd_f32: hipMemsetAsync");
  const int64_t chunks = (B * S + CS_ROWS - 1) / CS_ROWS;
  TT_REQUIRE(chunks <= 65535, "B * S > 65535 * 256");
  hipLaunchKernelGGL(k_weighted_col_sum, dim3((unsigned)((Hd + 63) / 64), (unsigned)chunks),
                     dim3(256), 0, st, H, Hd, da_ws, B * S, dW2, db2);
  return check_launch("k_weighted_col_sum");
}

extern "C" int tt_embedding_backward_f32(const float* g, int64_t ldg, const int32_t* ids,
                                         int64_t n, int32_t C, float* table_grad, void* stream) {
  TT_REQUIRE(n >= 0 && C >= 1, "bad sizes");
  if (n == 0) return TT_OK;
  TT_REQUIRE(g && ids && table_grad, "null pointer");
  hipLaunchKernelGGL(k_embedding_bwd, dim3((unsigned)n), dim3(64), 0, (hipStream_t)stream, g, ldg,
                     ids, n, C, table_grad);
  return check_launch("tt_embedding_backward_f32");
}

extern "C" int tt_adam_f32(float* p, const float* g, float* m, float* v, int64_t n, float lr,
                           float beta1, float beta2, float eps, int32_t step, void* stream) {
  TT_REQUIRE(n >= 0 && step >= 1, "need n >= 0, step >= 1");
  if (n == 0) return TT_OK;
  TT_REQUIRE(p && g && m && v, "null pointer");
  const float bc1 = 1.0f - powf(beta1, (float)step), bc2 = 1.0f - powf(beta2, (float)step);
  hipLaunchKernelGGL(k_adam, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n,
                     lr, beta1, beta2, eps, bc1, bc2);
  return check_launch("tt_adam_f32");
}
