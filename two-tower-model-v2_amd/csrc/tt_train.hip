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

typedef __bf16 tn_bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t tn_u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// dy = (dz - z (z . dz)) / ||y||  if ||y|| > eps, else dz / eps   (z = y / max(||y||, eps))
__global__ __launch_bounds__(256) void k_l2norm_bwd(const float* __restrict__ y, int64_t ldy,
                                                    const float* __restrict__ z, int64_t ldz,
                                                    const float* __restrict__ dz, int64_t lddz,
                                                    int64_t n, int d, float* __restrict__ dy,
                                                    int64_t lddy,
                                                    uint16_t* __restrict__ dy16 = nullptr,
                                                    int64_t lddy16 = 0) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool vec = d % 256 == 0 && d <= 1024 && ldy % 4 == 0 && ldz % 4 == 0 && lddz % 4 == 0 &&
                   lddy % 4 == 0 && (!dy16 || lddy16 % 4 == 0) && ((uintptr_t)y % 16) == 0 &&
                   ((uintptr_t)z % 16) == 0 && ((uintptr_t)dz % 16) == 0 &&
                   ((uintptr_t)dy % 16) == 0 && ((uintptr_t)dy16 % 8) == 0;
  if (vec) {  // a lane holds 4 consecutive columns per 256: one 16-B load per operand
    for (int64_t r = (int64_t)blockIdx.x * 4 + w; r < n; r += (int64_t)gridDim.x * 4) {
      f32x4 zv[4], gv[4];
      float ss = 0.0f, zd = 0.0f;
      const int nc = d / 256;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c >= nc) break;
        const int e = 256 * c + 4 * lane;
        const f32x4 yv = *(const f32x4*)(y + r * ldy + e);
        zv[c] = *(const f32x4*)(z + r * ldz + e);
        gv[c] = *(const f32x4*)(dz + r * lddz + e);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          ss = fmaf(yv[u], yv[u], ss);
          zd = fmaf(zv[c][u], gv[c][u], zd);
        }
      }
      ss = wave_sum(ss);
      zd = wave_sum(zd);
      const float nrm = sqrtf(ss);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c >= nc) break;
        const int e = 256 * c + 4 * lane;
        f32x4 o;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          o[u] = nrm > 1e-12f ? (gv[c][u] - zv[c][u] * zd) / nrm : gv[c][u] / 1e-12f;
        *(f32x4*)(dy + r * lddy + e) = o;
        if (dy16)
          *(tn_u32x2*)(dy16 + r * lddy16 + e) = tn_u32x2{
              (uint32_t)f32_to_bf16_rne(o[0]) | ((uint32_t)f32_to_bf16_rne(o[1]) << 16),
              (uint32_t)f32_to_bf16_rne(o[2]) | ((uint32_t)f32_to_bf16_rne(o[3]) << 16)};
      }
    }
    return;
  }
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
      const float v = nrm > 1e-12f ? (g - z[r * ldz + e] * zd) / nrm : g / 1e-12f;
      dy[r * lddy + e] = v;
      if (dy16) dy16[r * lddy16 + e] = f32_to_bf16_rne(v);
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
template <int NT>
__global__ __launch_bounds__(NT) void k_attn_pool_fwd(
    const float* __restrict__ H, int Hd, const float* __restrict__ W2, float b2,
    const float* __restrict__ b2p, const float* __restrict__ w, const float* __restrict__ x,
    int S, int E, float* __restrict__ alpha, float* __restrict__ onorm, float* __restrict__ z,
    int64_t ldz, uint16_t* __restrict__ z16 = nullptr) {
  constexpr int NW = NT / 64, PER = (1024 + NT - 1) / NT;
  __shared__ float cs[128], pal[128];
  __shared__ float red[NW];
  const int b = blockIdx.x, tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  if (b2p) b2 = *b2p;  // the bias read on the device (a graph-captured step: no host sync)
  // a_s = H_s . W2: 16 lanes per position, 16 positions per pass (the loads of all positions
  // in flight together; was one wave per position, five dependent rounds per wave)
  const int pl = tid & 15, pg = tid >> 4;
  for (int s0 = 0; s0 < S; s0 += NT / 16) {
    const int s = s0 + pg;
    float a = 0.0f;
    if (s < S) {
      const float* h = H + ((int64_t)b * S + s) * Hd;
      for (int j = pl; j < Hd; j += 16) a = fmaf(h[j], W2[j], a);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) a += __shfl_xor(a, o, 16);
    if (pl == 0 && s < S) cs[s] = (a + b2) * w[(int64_t)b * S + s];
  }
  __syncthreads();
  float m = -__builtin_huge_valf();
  for (int s = 0; s < S; ++s) m = fmaxf(m, cs[s]);
  float sum = 0.0f;
  for (int s = 0; s < S; ++s) sum += expf(cs[s] - m);
  const float inv = 1.0f / sum;
  if (tid < S) {
    const float al = expf(cs[tid] - m) * inv;
    pal[tid] = al;
    alpha[(int64_t)b * S + tid] = al;
  }
  __syncthreads();
  // o = sum alpha x ; ||o||
  const float* xb = x + (int64_t)b * S * E;
  float ss = 0.0f;
  float ov[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = tid + NT * i;
    float o = 0.0f;
    if (e < E)
      for (int s = 0; s < S; ++s) o = fmaf(pal[s], xb[(int64_t)s * E + e], o);
    ov[i] = o;
    ss = fmaf(o, o, ss);
  }
  ss = wave_sum(ss);
  if (lane == 0) red[wv] = ss;
  __syncthreads();
  float ssum = 0.0f;
#pragma unroll
  for (int i = 0; i < NW; ++i) ssum += red[i];
  const float nrm = sqrtf(ssum);
  if (tid == 0) onorm[b] = nrm;
  const float den = fmaxf(nrm, 1e-12f);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = tid + NT * i;
    if (e < E) {
      z[(int64_t)b * ldz + e] = ov[i] / den;
      if (z16) z16[(int64_t)b * ldz + e] = f32_to_bf16_rne(ov[i] / den);
    }
  }
}

// Backward of k_attn_pool_fwd: block per buyer.  do = normalize backward(dz);
// dalpha_s = do . x_s ; dc_s = alpha_s (dalpha_s - sum_t alpha_t dalpha_t) ; da_s = dc_s w_s.
// Writes da [B*S] (dW2 = da^T H and db2 = sum da are reductions done after) and
// dH[bs][j] = da_bs * W2[j] (the ReLU mask is applied by tt_relu_backward_f32).
template <int NT>
__global__ __launch_bounds__(NT) void k_attn_pool_bwd(
    const float* __restrict__ dz, int64_t lddz, const float* __restrict__ z, int64_t ldz,
    const float* __restrict__ onorm, const float* __restrict__ alpha,
    const float* __restrict__ w, const float* __restrict__ x, int S, int E,
    const float* __restrict__ W2, int Hd, float* __restrict__ da, float* __restrict__ dH,
    const float* __restrict__ H, bool relu_mask, float* __restrict__ part) {
  __shared__ float dov[1024];
  __shared__ float dal[128], sal[128], sw[128], sdas[128];
  constexpr int NW = NT / 64;
  __shared__ float red[NW];
  const int b = blockIdx.x, tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  if (tid < S) {  // the buyer's alpha and weights, loaded once (not per position in a loop)
    sal[tid] = alpha[(int64_t)b * S + tid];
    sw[tid] = w[(int64_t)b * S + tid];
  }
  const float nrm = onorm[b];
  float zd = 0.0f;
  for (int e = tid; e < E; e += NT) zd = fmaf(z[(int64_t)b * ldz + e], dz[(int64_t)b * lddz + e], zd);
  zd = wave_sum(zd);
  if (lane == 0) red[wv] = zd;
  __syncthreads();
  zd = 0.0f;
#pragma unroll
  for (int i = 0; i < NW; ++i) zd += red[i];
  for (int e = tid; e < E; e += NT) {
    const float g = dz[(int64_t)b * lddz + e];
    dov[e] = nrm > 1e-12f ? (g - z[(int64_t)b * ldz + e] * zd) / nrm : g / 1e-12f;
  }
  __syncthreads();
  const float* xb = x + (int64_t)b * S * E;
  // dalpha_s = do . x_s: 16 lanes per position, 16 positions per pass (all loads in flight)
  const int pl = tid & 15, pg = tid >> 4;
  for (int s0 = 0; s0 < S; s0 += NT / 16) {
    const int s = s0 + pg;
    float d = 0.0f;
    if (s < S)
      for (int e = pl; e < E; e += 16) d = fmaf(dov[e], xb[(int64_t)s * E + e], d);
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) d += __shfl_xor(d, o, 16);
    if (pl == 0 && s < S) dal[s] = d;
  }
  __syncthreads();
  float adot = 0.0f;
  for (int s = 0; s < S; ++s) adot = fmaf(sal[s], dal[s], adot);
  if (tid < S) {
    const float das = sal[tid] * (dal[tid] - adot) * sw[tid];
    sdas[tid] = das;
    da[(int64_t)b * S + tid] = das;
  }
  __syncthreads();
  const int64_t o0 = (int64_t)b * S * Hd;
  for (int i = tid; i < S * Hd; i += NT) {  // dH = da W2 (ReLU backward of H fused)
    const float v = sdas[i / Hd] * W2[i % Hd];
    dH[o0 + i] = relu_mask && !(H[o0 + i] > 0.0f) ? 0.0f : v;
  }
  if (part) {  // this buyer's part of dW2 = da^T H and db2 = sum da (k_attn_bwd_reduce sums)
    float* pb = part + (int64_t)b * (Hd + 1);
    for (int j = tid; j < Hd; j += NT) {
      float acc = 0.0f;
      for (int s2 = 0; s2 < S; ++s2) acc = fmaf(sdas[s2], H[o0 + (int64_t)s2 * Hd + j], acc);
      pb[j] = acc;
    }
    if (tid == 0) {
      float sd = 0.0f;
      for (int s2 = 0; s2 < S; ++s2) sd += sdas[s2];
      pb[Hd] = sd;
    }
  }
}

// dW2 [Hd] and db2 from the per-buyer parts [B][Hd + 1]: a block of 8 row groups x 128
// columns (a wave reads 64 consecutive columns of one row), each group a fixed contiguous
// range of buyers with all its loads in flight, then the 8 groups summed in order
// (deterministic; one launch, where 512 blocks' atomics on the same 129 addresses had
// serialised at the L2)
__global__ __launch_bounds__(1024) void k_attn_bwd_reduce(const float* __restrict__ part, int B,
                                                          int Hd, float* __restrict__ dW2,
                                                          float* __restrict__ db2) {
  __shared__ float gs[8][128];
  const int g = threadIdx.x >> 7, cl = threadIdx.x & 127;
  const int c = blockIdx.x * 128 + cl;
  const int per = (B + 7) / 8, r0 = g * per, r1 = min(B, r0 + per);
  float sacc = 0.0f;
  if (c <= Hd) {
    for (int rb = r0; rb < r1; rb += 32) {  // 32 loads in flight, then summed in row order
      float v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = rb + u < r1 ? part[(int64_t)(rb + u) * (Hd + 1) + c] : 0.0f;
#pragma unroll
      for (int u = 0; u < 32; ++u) sacc += v[u];
    }
  }
  gs[g][cl] = sacc;
  __syncthreads();
  if (g == 0 && c <= Hd) {
    float t = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += gs[i][cl];
    if (c < Hd) dW2[c] = t;
    else *db2 = t;
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

// ------------------------------------------------------------- C = A^T B  (weight gradients)
// dW [N, K] = dY^T X for row-major dY [M, N], X [M, K] f32: the reduction runs over the batch
// rows M (2.5k-10k) while N, K <= 768, so a tile grid over the output alone has 24-96 blocks.
// Each block takes one 64 x 64 output tile and one split of the rows and writes its partial
// tile to the workspace; k_tn_reduce then sums the splits of every output element in split
// order (deterministic; one thread per element, so the tail is parallel, not one block's).  No
// transposed copies: a 64-row chunk of dY and X is staged in LDS with m contiguous (a lane's
// coalesced column loads land as one 16-B write), and the next chunk's loads are in flight
// while this chunk's MFMAs run.  BF: operands rounded to bf16 (RNE) in registers,
// v_mfma_f32_16x16x32_bf16; else v_mfma_f32_16x16x4_f32.  Optional db [N] = column sums of
// dY (the bias gradient, from the same loads; f32, fixed order).
constexpr int TN_T = 64;
constexpr int TN_SMAX = 64;  // row splits per tile
__host__ __device__ constexpr int tn_pitch(bool bf) { return bf ? 64 + 8 : 64 + 4; }

template <bool BF>
__global__ __launch_bounds__(256) void k_gemm_tn(const float* __restrict__ A, int64_t lda,
                                                 const float* __restrict__ B, int64_t ldb, int M,
                                                 int N, int K, int mc, float* __restrict__ C,
                                                 int64_t ldc, float* __restrict__ db,
                                                 float* __restrict__ parts,
                                                 float* __restrict__ dbparts) {
  using E = typename std::conditional<BF, uint16_t, float>::type;
  constexpr int P = tn_pitch(BF);
  __shared__ __attribute__((aligned(16))) E sA[TN_T * P];
  __shared__ __attribute__((aligned(16))) E sB[TN_T * P];
  __shared__ float sdb[4][TN_T];
  const int kt = blockIdx.x, nt = blockIdx.y, s = blockIdx.z, S = gridDim.z;
  const int KT = gridDim.x, tile = nt * KT + kt;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int col = tid & 63, grp = tid >> 6;  // staging: column col, m-groups grp and grp + 4
  const int n0 = nt * TN_T, k0 = kt * TN_T;
  const int m_beg = s * mc, m_end = min(M, m_beg + mc);
  const bool na = n0 + col < N, kb = k0 + col < K;
  const bool want_db = db != nullptr && kt == 0;
  const int wn = w & 1, wk = w >> 1, r = lane & 15, q = lane >> 4;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbs = 0.0f;
  float av[2][8], bv[2][8];
  auto load = [&](int mc0) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int g8 = 8 * (grp + 4 * h);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = mc0 + g8 + j;
        const bool mv = m < m_end;
        av[h][j] = mv && na ? A[(int64_t)m * lda + n0 + col] : 0.0f;
        bv[h][j] = mv && kb ? B[(int64_t)m * ldb + k0 + col] : 0.0f;
      }
    }
  };
  if (m_beg < m_end) load(m_beg);
  for (int mc0 = m_beg; mc0 < m_end; mc0 += TN_T) {
    if (want_db) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 8; ++j) dbs += av[h][j];
    }
    __syncthreads();  // the previous chunk's fragment reads are done
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int g8 = 8 * (grp + 4 * h);
      if constexpr (BF) {
        uint32_t pa[4], pb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pa[j] = (uint32_t)f32_to_bf16_rne(av[h][2 * j]) |
                  ((uint32_t)f32_to_bf16_rne(av[h][2 * j + 1]) << 16);
          pb[j] = (uint32_t)f32_to_bf16_rne(bv[h][2 * j]) |
                  ((uint32_t)f32_to_bf16_rne(bv[h][2 * j + 1]) << 16);
        }
        *(u32x4_t*)&sA[col * P + g8] = u32x4_t{pa[0], pa[1], pa[2], pa[3]};
        *(u32x4_t*)&sB[col * P + g8] = u32x4_t{pb[0], pb[1], pb[2], pb[3]};
      } else {
        *(f32x4*)&sA[col * P + g8] = f32x4{av[h][0], av[h][1], av[h][2], av[h][3]};
        *(f32x4*)&sA[col * P + g8 + 4] = f32x4{av[h][4], av[h][5], av[h][6], av[h][7]};
        *(f32x4*)&sB[col * P + g8] = f32x4{bv[h][0], bv[h][1], bv[h][2], bv[h][3]};
        *(f32x4*)&sB[col * P + g8 + 4] = f32x4{bv[h][4], bv[h][5], bv[h][6], bv[h][7]};
      }
    }
    __syncthreads();
    if (mc0 + TN_T < m_end) load(mc0 + TN_T);  // next chunk in flight during the MFMAs
    if constexpr (BF) {
#pragma unroll
      for (int kk = 0; kk < TN_T; kk += 32) {
        tn_bf16x8 fa[2], fb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          fa[i] = *(const tn_bf16x8*)&sA[(32 * wn + 16 * i + r) * P + kk + 8 * q];
#pragma unroll
        for (int j = 0; j < 2; ++j)
          fb[j] = *(const tn_bf16x8*)&sB[(32 * wk + 16 * j + r) * P + kk + 8 * q];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < TN_T; kk += 4) {
        float fa[2], fb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) fa[i] = sA[(32 * wn + 16 * i + r) * P + kk + q];
#pragma unroll
        for (int j = 0; j < 2; ++j) fb[j] = sB[(32 * wk + 16 * j + r) * P + kk + q];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  // D lane layout: acc[i][j][v] = tile[n = 32 wn + 16 i + 4 q + v][k = 32 wk + 16 j + r]
  if (want_db) {
    sdb[grp][col] = dbs;
    __syncthreads();
  }
  if (S == 1) {  // no split: straight to C (and db)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int n = n0 + 32 * wn + 16 * i + 4 * q + v, k = k0 + 32 * wk + 16 * j + r;
          if (n < N && k < K) C[(int64_t)n * ldc + k] = acc[i][j][v];
        }
    if (want_db && tid < TN_T && n0 + tid < N)
      db[n0 + tid] = ((sdb[0][tid] + sdb[1][tid]) + sdb[2][tid]) + sdb[3][tid];
    return;
  }
  const int T = gridDim.x * gridDim.y;
  float* pt = parts + ((int64_t)s * T + tile) * (TN_T * TN_T);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 4; ++v)
        pt[(32 * wn + 16 * i + 4 * q + v) * TN_T + 32 * wk + 16 * j + r] = acc[i][j][v];
  if (want_db && tid < TN_T)
    dbparts[(int64_t)s * gridDim.y * TN_T + n0 + tid] =
        ((sdb[0][tid] + sdb[1][tid]) + sdb[2][tid]) + sdb[3][tid];
}

// The splits' sum, one thread per output element (and per bias-gradient entry), in split
// order; the S loads of a thread are independent, so they are all in flight at once.
__device__ __forceinline__ void tn_reduce_item(const float* __restrict__ parts,
                                               const float* __restrict__ dbparts, int S, int T,
                                               int KT, int NT, int N, int K,
                                               float* __restrict__ C, int64_t ldc,
                                               float* __restrict__ db, int64_t gid) {
  const int64_t ne = (int64_t)T * TN_T * TN_T;
  if (gid < ne) {
    const int tile = (int)(gid / (TN_T * TN_T)), e = (int)(gid % (TN_T * TN_T));
    const int n = (tile / KT) * TN_T + e / TN_T, k = (tile % KT) * TN_T + e % TN_T;
    if (n >= N || k >= K) return;
    float v[TN_SMAX];
#pragma unroll
    for (int u = 0; u < TN_SMAX; ++u) v[u] = u < S ? parts[(int64_t)u * ne + gid] : 0.0f;
    float sum = v[0];
#pragma unroll
    for (int u = 1; u < TN_SMAX; ++u)
      if (u < S) sum += v[u];
    C[(int64_t)n * ldc + k] = sum;
    return;
  }
  const int64_t i = gid - ne;  // bias gradient entries
  if (db == nullptr || i >= N) return;
  float v[TN_SMAX];
#pragma unroll
  for (int u = 0; u < TN_SMAX; ++u) v[u] = u < S ? dbparts[(int64_t)u * NT * TN_T + i] : 0.0f;
  float sum = v[0];
#pragma unroll
  for (int u = 1; u < TN_SMAX; ++u)
    if (u < S) sum += v[u];
  db[i] = sum;
}

__global__ __launch_bounds__(256) void k_tn_reduce(const float* __restrict__ parts,
                                                   const float* __restrict__ dbparts, int S,
                                                   int T, int KT, int NT, int N, int K,
                                                   float* __restrict__ C, int64_t ldc,
                                                   float* __restrict__ db) {
  tn_reduce_item(parts, dbparts, S, T, KT, NT, N, K, C, ldc, db,
                 (int64_t)blockIdx.x * 256 + threadIdx.x);
}

// Several GEMMs' split sums in one launch (tt_gemm_tn_reduce_many): job i owns the global
// items [start_i, start_{i+1}); the same per-item code and order as k_tn_reduce.
constexpr int TN_RED_MAX = 8;
struct TnRedJob {
  const float* parts;
  const float* dbparts;
  float* C;
  float* db;
  int64_t ldc, start;
  int S, T, KT, NT, N, K;
};
struct TnRedArgs {
  TnRedJob j[TN_RED_MAX];
  int n;
};
__global__ __launch_bounds__(256) void k_tn_reduce_many(TnRedArgs a) {
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int i = 0;
#pragma unroll
  for (int u = 1; u < TN_RED_MAX; ++u)
    if (u < a.n && gid >= a.j[u].start) i = u;
  const TnRedJob& J = a.j[i];
  tn_reduce_item(J.parts, J.dbparts, J.S, J.T, J.KT, J.NT, J.N, J.K, J.C, J.ldc, J.db,
                 gid - J.start);
}

// The training step's backward tail in ONE launch (tt_train_bwd_tail): blocks [0, nA) sum the
// deferred weight-gradient splits (k_tn_reduce_many's items), the next nB blocks the attention
// pooling's per-buyer dW2 / db2 parts (k_attn_bwd_reduce's order: 8 row groups, each summed in
// row order, then the groups in order -- the same bits), the rest scatter the embedding-row
// gradients (k_embedding_bwd2, one wave per row, atomics).
struct TailArgs {
  TnRedArgs tn;
  int64_t tn_items;
  int nA, nB;
  const float* part;  // attention parts [B][Hd + 1]
  int B, Hd;
  float *dW2, *db2;
  const float* g;  // embedding rows' gradients [n][ldg]: brand at 0, cat at C
  int64_t ldg, n;
  const int32_t *ids0, *ids1;
  int C;
  float *grad0, *grad1;
};
__global__ __launch_bounds__(256) void k_train_tail(TailArgs a) {
  const int bx = blockIdx.x, tid = threadIdx.x;
  if (bx < a.nA) {
    const int64_t gid = (int64_t)bx * 256 + tid;
    if (gid >= a.tn_items) return;
    int i = 0;
#pragma unroll
    for (int u = 1; u < TN_RED_MAX; ++u)
      if (u < a.tn.n && gid >= a.tn.j[u].start) i = u;
    const TnRedJob& J = a.tn.j[i];
    tn_reduce_item(J.parts, J.dbparts, J.S, J.T, J.KT, J.NT, J.N, J.K, J.C, J.ldc, J.db,
                   gid - J.start);
    return;
  }
  if (bx < a.nA + a.nB) {
    __shared__ float gs[8][32];
    const int g = tid >> 5, cl = tid & 31;
    const int c = (bx - a.nA) * 32 + cl, Hd = a.Hd, B = a.B;
    const int per = (B + 7) / 8, r0 = g * per, r1 = min(B, r0 + per);
    float sacc = 0.0f;
    if (c <= Hd) {
      for (int rb = r0; rb < r1; rb += 32) {
        float v[32];
#pragma unroll
        for (int u = 0; u < 32; ++u)
          v[u] = rb + u < r1 ? a.part[(int64_t)(rb + u) * (Hd + 1) + c] : 0.0f;
#pragma unroll
        for (int u = 0; u < 32; ++u) sacc += v[u];
      }
    }
    gs[g][cl] = sacc;
    __syncthreads();
    if (g == 0 && c <= Hd) {
      float t = 0.0f;
#pragma unroll
      for (int i = 0; i < 8; ++i) t += gs[i][cl];
      if (c < Hd) a.dW2[c] = t;
      else *a.db2 = t;
    }
    return;
  }
  const int64_t rr = (int64_t)(bx - a.nA - a.nB) * 4 + (tid >> 6), lane = tid & 63;
  if (rr >= 2 * a.n) return;
  const bool second = rr >= a.n;
  const int64_t r = second ? rr - a.n : rr;
  const int32_t* ids = second ? a.ids1 : a.ids0;
  if (ids == nullptr) return;
  const int id = ids[r];
  if (id <= 0) return;  // padding_idx 0 gets no gradient
  float* tg = second ? a.grad1 : a.grad0;
  const float* gr = a.g + r * a.ldg + (second ? a.C : 0);
  for (int c = (int)lane; c < a.C; c += 64) atomicAdd(&tg[(int64_t)id * a.C + c], gr[c]);
}

#ifndef TT_TN_BLOCKS
#define TT_TN_BLOCKS 1024  // blocks a split plan aims at (~4 per CU: the k-loop is latency-bound)
#endif
TT_CHECK_EXP(TT_TN_BLOCKS != 1024, "TT_TN_BLOCKS");
constexpr int TN_TARGET_BLOCKS = TT_TN_BLOCKS;
struct TnPlan {
  int NT, KT, S, mc;
  size_t parts, dbparts, total;
};
TnPlan tn_plan(int64_t M, int N, int K) {
  TnPlan p{};
  p.NT = (N + TN_T - 1) / TN_T;
  p.KT = (K + TN_T - 1) / TN_T;
  const int T = p.NT * p.KT;
  int64_t S = (TN_TARGET_BLOCKS + T - 1) / T;
  const int64_t maxS = (M + TN_T - 1) / TN_T;
  if (S > maxS) S = maxS;
  if (S > TN_SMAX) S = TN_SMAX;
  if (S < 1) S = 1;
  int64_t mc = (M + S - 1) / S;
  mc = (mc + TN_T - 1) / TN_T * TN_T;
  if (mc < TN_T) mc = TN_T;
  p.mc = (int)mc;
  p.S = (int)((M + mc - 1) / mc);
  if (p.S < 1) p.S = 1;
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  p.parts = 0;
  p.dbparts = p.S > 1 ? al((size_t)p.S * T * TN_T * TN_T * 4) : 0;
  p.total = p.S > 1 ? p.dbparts + al((size_t)p.S * p.NT * TN_T * 4) : 0;
  return p;
}

// ------------------------------------------------- fused elementwise pieces of the step
// nn.Dropout forward with a given keep mask plus the bf16 copy the next GEMM reads
__global__ void k_dropout_ex(float* __restrict__ x, const uint8_t* __restrict__ keep, float scale,
                             int64_t n, uint16_t* __restrict__ x16) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float v = keep[i] ? x[i] * scale : 0.0f;
    x[i] = v;
    if (x16) x16[i] = f32_to_bf16_rne(v);
  }
}

// nn.Dropout forward with the keep mask drawn in the kernel: element i of draw c is kept iff
// u(seed, c, i) >= p * 2^32, u = the high 32 bits of splitmix64(seed + (c << 40) + i) -- a
// counter-based generator, so a step replayed from a HIP graph draws fresh masks by reading
// the draw counter c from device memory (the caller advances it each step).  No mask is
// stored: the backward needs only h > 0 (k_relu_drop_bwd).
__device__ __forceinline__ uint32_t drop_u32(uint64_t seed, uint64_t c, uint64_t i) {
  uint64_t zz = seed + (c << 40) + i + 0x9e3779b97f4a7c15ull;
  zz = (zz ^ (zz >> 30)) * 0xbf58476d1ce4e5b9ull;
  zz = (zz ^ (zz >> 27)) * 0x94d049bb133111ebull;
  return (uint32_t)((zz ^ (zz >> 31)) >> 32);
}
__global__ void k_dropout_rng(float* __restrict__ x, int64_t n, uint32_t thresh, float scale,
                              uint64_t seed, const int64_t* __restrict__ ctr,
                              uint16_t* __restrict__ x16) {
  const uint64_t c = (uint64_t)*ctr;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float v = drop_u32(seed, c, (uint64_t)i) >= thresh ? x[i] * scale : 0.0f;
    x[i] = v;
    if (x16) x16[i] = f32_to_bf16_rne(v);
  }
}

// both embedding tables' row gradients in one launch: blocks [0, n) brand, [n, 2n) category
__global__ void k_embedding_bwd2(const float* __restrict__ g, int64_t ldg,
                                 const int32_t* __restrict__ ids0,
                                 const int32_t* __restrict__ ids1, int64_t n, int C,
                                 float* __restrict__ grad0, float* __restrict__ grad1) {
  const bool second = blockIdx.x >= n;
  const int64_t r = second ? blockIdx.x - n : blockIdx.x;
  const int32_t* ids = second ? ids1 : ids0;
  if (ids == nullptr) return;
  const int id = ids[r];
  if (id <= 0) return;  // padding_idx 0 gets no gradient
  float* tg = second ? grad1 : grad0;
  const float* gr = g + r * ldg + (second ? C : 0);
  for (int c = threadIdx.x; c < C; c += blockDim.x) atomicAdd(&tg[(int64_t)id * C + c], gr[c]);
}

// ReLU (+ Dropout) backward on the post-activation h: h > 0 iff the unit was kept and active,
// so dh = h > 0 ? dh * scale : 0 covers both (scale = 1 / (1 - p), 1 without dropout)
__global__ void k_relu_drop_bwd(float* __restrict__ dh, const float* __restrict__ h, float scale,
                                int64_t n, uint16_t* __restrict__ dh16,
                                int64_t* __restrict__ ctr_advance) {
  // (advances the dropout draw counter of tt_dropout_rng_f32 after this step's last use)
  if (ctr_advance && blockIdx.x == 0 && threadIdx.x == 0) *ctr_advance += 1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float v = h[i] > 0.0f ? dh[i] * scale : 0.0f;
    dh[i] = v;
    if (dh16) dh16[i] = f32_to_bf16_rne(v);
  }
}

constexpr int CV_RG = 4;  // row groups of 8 per non-transposed convert tile (32 rows)
struct tt_convert_batch_args {
  tt_convert_job jobs[TT_CONVERT_MAX_JOBS];
  int tile_off[TT_CONVERT_MAX_JOBS];
  int njobs;
};

// Batched operand preparation (one launch per step for all weight-derived GEMM operands and
// the bf16 copies of f32 inputs): job j copies src [rows, cols] to dst as f32 or bf16,
// optionally transposed (dst [cols, ld_dst], columns rows..ld_dst-1 zero-filled).
__global__ __launch_bounds__(256) void k_convert_batch(tt_convert_batch_args a) {
  int j = 0;
  while (j + 1 < a.njobs && (int)blockIdx.x >= a.tile_off[j + 1]) ++j;
  const tt_convert_job& jb = a.jobs[j];
  const int t = (int)blockIdx.x - a.tile_off[j];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  if (!jb.transpose) {  // 32 x 128 tiles: 4 row groups of 8, 4 consecutive elements per thread
    const int ct = (jb.cols + 127) / 128;
    const int c = (t % ct) * 128 + 4 * tx;
    if (c >= jb.cols) return;
    const bool full = c + 4 <= jb.cols;
#pragma unroll
    for (int k = 0; k < CV_RG; ++k) {
      const int r = (t / ct) * (8 * CV_RG) + 8 * k + ty;
      if (r >= jb.rows) break;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      const int sr = jb.row_ids ? jb.row_ids[r] : r;  // (gathered rows: a negative id is zeros)
      if (jb.src && sr >= 0) {
        const float* sp = jb.src + (int64_t)sr * jb.ld_src + c;
        if (full && ((uintptr_t)sp % 16) == 0) {
          const f32x4 q = *(const f32x4*)sp;
          v[0] = q[0], v[1] = q[1], v[2] = q[2], v[3] = q[3];
        } else {
          for (int u = 0; u < 4; ++u)
            if (c + u < jb.cols) v[u] = sp[u];
        }
      }
      if (jb.to_bf16) {
        uint16_t* dp = (uint16_t*)jb.dst + (int64_t)r * jb.ld_dst + c;
        if (full && ((uintptr_t)dp % 8) == 0) {
          *(tn_u32x2*)dp = tn_u32x2{
              (uint32_t)f32_to_bf16_rne(v[0]) | ((uint32_t)f32_to_bf16_rne(v[1]) << 16),
              (uint32_t)f32_to_bf16_rne(v[2]) | ((uint32_t)f32_to_bf16_rne(v[3]) << 16)};
        } else {
          for (int u = 0; u < 4; ++u)
            if (c + u < jb.cols) dp[u] = f32_to_bf16_rne(v[u]);
        }
      } else {
        float* dp = (float*)jb.dst + (int64_t)r * jb.ld_dst + c;
        if (full && ((uintptr_t)dp % 16) == 0) {
          *(f32x4*)dp = f32x4{v[0], v[1], v[2], v[3]};
        } else {
          for (int u = 0; u < 4; ++u)
            if (c + u < jb.cols) dp[u] = v[u];
        }
      }
    }
    return;
  }
  const int rr = (int)(jb.ld_dst > jb.rows ? jb.ld_dst : jb.rows);
  const int ct = (jb.cols + 31) / 32;
  const int r0 = (t / ct) * 32, c0 = (t % ct) * 32;
  __shared__ float tl[32][33];
  for (int y = ty; y < 32; y += 8) {
    const int r = r0 + y, c = c0 + tx;
    tl[y][tx] = (r < jb.rows && c < jb.cols) ? jb.src[(int64_t)r * jb.ld_src + c] : 0.0f;
  }
  __syncthreads();
  for (int y = ty; y < 32; y += 8) {
    const int c = c0 + y, r = r0 + tx;
    if (c < jb.cols && r < rr) {
      const float v = tl[tx][y];
      if (jb.to_bf16) ((uint16_t*)jb.dst)[(int64_t)c * jb.ld_dst + r] = f32_to_bf16_rne(v);
      else ((float*)jb.dst)[(int64_t)c * jb.ld_dst + r] = v;
    }
  }
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
  hipLaunchKernelGGL(k_attn_pool_fwd<256>, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, H,
                     Hd, W2, b2, (const float*)nullptr, w, x, S, E, alpha, onorm, z, ldz,
                     (uint16_t*)nullptr);
  return check_launch("tt_attn_pool_fwd_f32");
}

extern "C" int tt_attn_pool_fwd_f32_dev(const float* H, int32_t Hd, const float* W2,
                                        const float* b2, const float* w, const float* x, int64_t B,
                                        int32_t S, int32_t E, float* alpha, float* onorm, float* z,
                                        int64_t ldz, uint16_t* z_bf16, void* stream) {
  TT_REQUIRE(B >= 0 && S >= 1 && S <= 128 && E >= 1 && E <= 1024 && Hd >= 1,
             "need 1 <= S <= 128, 1 <= E <= 1024");
  if (B == 0) return TT_OK;
  TT_REQUIRE(H && W2 && b2 && w && x && alpha && onorm && z, "null pointer");
  hipLaunchKernelGGL(k_attn_pool_fwd<512>, dim3((unsigned)B), dim3(512), 0, (hipStream_t)stream, H,
                     Hd, W2, 0.0f, b2, w, x, S, E, alpha, onorm, z, ldz, z_bf16);
  return check_launch("tt_attn_pool_fwd_f32_dev");
}

namespace {
int attn_pool_bwd(const float* dz, int64_t lddz, const float* z, int64_t ldz, const float* onorm,
                  const float* alpha, const float* w, const float* x, int64_t B, int32_t S,
                  int32_t E, const float* H, const float* W2, int32_t Hd, float* dW2, float* db2,
                  float* dH, float* da_ws, bool relu_mask, bool fused, void* stream,
                  bool parts_only = false) {
  TT_REQUIRE(B >= 0 && S >= 1 && S <= 128 && E >= 1 && E <= 1024 && Hd >= 1,
             "need 1 <= S <= 128, 1 <= E <= 1024");
  if (B == 0) return TT_OK;
  TT_REQUIRE(dz && z && onorm && alpha && w && x && H && W2 && (parts_only || (dW2 && db2)) &&
                 dH && da_ws,
             "null pointer");
  hipStream_t st = (hipStream_t)stream;
  float* part = fused ? da_ws + (B * S + 63) / 64 * 64 : nullptr;  // [B][Hd + 1] after da
  hipLaunchKernelGGL(k_attn_pool_bwd<512>, dim3((unsigned)B), dim3(512), 0, st, dz, lddz, z, ldz,
                     onorm, alpha, w, x, S, E, W2, Hd, da_ws, dH, H, relu_mask, part);
  int rc = check_launch("k_attn_pool_bwd");
  if (rc || parts_only) return rc;
  if (fused) {
    hipLaunchKernelGGL(k_attn_bwd_reduce, dim3((unsigned)((Hd + 1 + 127) / 128)), dim3(1024), 0,
                       st, part, (int)B, Hd, dW2, db2);
    return check_launch("k_attn_bwd_reduce");
  }
  if (hipMemsetAsync(dW2, 0, (size_t)Hd * 4, st) != hipSuccess ||
      hipMemsetAsync(db2, 0, 4, st) != hipSuccess)
    return fail(TT_ERR_LAUNCH, "tt_attn_pool_bwd_f32: hipMemsetAsync");
  const int64_t chunks = (B * S + CS_ROWS - 1) / CS_ROWS;
  TT_REQUIRE(chunks <= 65535, "B * S > 65535 * 256");
  hipLaunchKernelGGL(k_weighted_col_sum, dim3((unsigned)((Hd + 63) / 64), (unsigned)chunks),
                     dim3(256), 0, st, H, Hd, da_ws, B * S, dW2, db2);
  return check_launch("k_weighted_col_sum");
}
}  // namespace

extern "C" int tt_attn_pool_bwd_f32(const float* dz, int64_t lddz, const float* z, int64_t ldz,
                                    const float* onorm, const float* alpha, const float* w,
                                    const float* x, int64_t B, int32_t S, int32_t E,
                                    const float* H, const float* W2, int32_t Hd, float* dW2,
                                    float* db2, float* dH, float* da_ws, void* stream) {
  return attn_pool_bwd(dz, lddz, z, ldz, onorm, alpha, w, x, B, S, E, H, W2, Hd, dW2, db2, dH,
                       da_ws, false, false, stream);
}

extern "C" int tt_attn_pool_bwd_relu_f32(const float* dz, int64_t lddz, const float* z,
                                         int64_t ldz, const float* onorm, const float* alpha,
                                         const float* w, const float* x, int64_t B, int32_t S,
                                         int32_t E, const float* H, const float* W2, int32_t Hd,
                                         float* dW2, float* db2, float* dH, float* da_ws,
                                         void* stream) {
  return attn_pool_bwd(dz, lddz, z, ldz, onorm, alpha, w, x, B, S, E, H, W2, Hd, dW2, db2, dH,
                       da_ws, true, true, stream);
}

extern "C" int tt_attn_pool_bwd_relu_parts_f32(const float* dz, int64_t lddz, const float* z,
                                               int64_t ldz, const float* onorm,
                                               const float* alpha, const float* w,
                                               const float* x, int64_t B, int32_t S, int32_t E,
                                               const float* H, const float* W2, int32_t Hd,
                                               float* dH, float* da_ws, void* stream) {
  return attn_pool_bwd(dz, lddz, z, ldz, onorm, alpha, w, x, B, S, E, H, W2, Hd, nullptr,
                       nullptr, dH, da_ws, true, true, stream, true);
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

extern "C" int tt_gemm_tn_workspace_bytes(int64_t M, int32_t N, int32_t K, int64_t* bytes) {
  TT_REQUIRE(bytes && M >= 0 && N >= 0 && K >= 0, "bad arguments");
  *bytes = (int64_t)tn_plan(M, N, K).total;
  return TT_OK;
}

namespace {
// the GEMM launch of tt_gemm_tn; *pending = 1 when its split sums still have to be reduced
int gemm_tn_launch(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M,
                   int32_t N, int32_t K, int32_t prec, float* C, int64_t ldc, float* db,
                   void* workspace, int64_t workspace_bytes, void* stream, int* pending) {
  *pending = 0;
  TT_REQUIRE(M >= 0 && N >= 0 && K >= 0 && M <= 0x7fffffffLL, "bad sizes");
  TT_REQUIRE(prec == TT_PREC_F32 || prec == TT_PREC_BF16, "prec must be TT_PREC_F32 / BF16");
  if (N == 0 || K == 0) return TT_OK;
  TT_REQUIRE(C && ldc >= K && lda >= N && ldb >= K, "null C or ld too small");
  hipStream_t st = (hipStream_t)stream;
  if (M == 0) {  // empty reduction: zeros
    if (hipMemset2DAsync(C, (size_t)ldc * 4, 0, (size_t)K * 4, (size_t)N, st) != hipSuccess ||
        (db && hipMemsetAsync(db, 0, (size_t)N * 4, st) != hipSuccess))
      return fail(TT_ERR_LAUNCH, "tt_gemm_tn: hipMemset");
    return TT_OK;
  }
  TT_REQUIRE(A && B, "null operand");
  const TnPlan p = tn_plan(M, N, K);
  TT_REQUIRE(p.NT <= 65535, "N too large");
  if (p.S > 1 && (!workspace || workspace_bytes < (int64_t)p.total))
    return fail(TT_ERR_WORKSPACE, "tt_gemm_tn: workspace too small (tt_gemm_tn_workspace_bytes)");
  char* ws = (char*)workspace;
  float* parts = p.S > 1 ? (float*)(ws + p.parts) : nullptr;
  float* dbparts = p.S > 1 ? (float*)(ws + p.dbparts) : nullptr;
  const dim3 grid((unsigned)p.KT, (unsigned)p.NT, (unsigned)p.S);
  if (prec == TT_PREC_BF16)
    hipLaunchKernelGGL(k_gemm_tn<true>, grid, dim3(256), 0, st, A, lda, B, ldb, (int)M, N, K,
                       p.mc, C, ldc, db, parts, dbparts);
  else
    hipLaunchKernelGGL(k_gemm_tn<false>, grid, dim3(256), 0, st, A, lda, B, ldb, (int)M, N, K,
                       p.mc, C, ldc, db, parts, dbparts);
  int rc = check_launch("k_gemm_tn");
  if (!rc) *pending = p.S > 1;
  return rc;
}
}  // namespace

extern "C" int tt_gemm_tn(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M,
                          int32_t N, int32_t K, int32_t prec, float* C, int64_t ldc, float* db,
                          void* workspace, int64_t workspace_bytes, void* stream) {
  int pending = 0;
  int rc = gemm_tn_launch(A, lda, B, ldb, M, N, K, prec, C, ldc, db, workspace, workspace_bytes,
                          stream, &pending);
  if (rc || !pending) return rc;
  const TnPlan p = tn_plan(M, N, K);
  const int T = p.NT * p.KT;
  const int64_t items = (int64_t)T * TN_T * TN_T + (db ? N : 0);
  char* ws = (char*)workspace;
  hipLaunchKernelGGL(k_tn_reduce, dim3((unsigned)((items + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const float*)(ws + p.parts),
                     (const float*)(ws + p.dbparts), p.S, T, p.KT, p.NT, N, K, C, ldc, db);
  return check_launch("k_tn_reduce");
}

extern "C" int tt_gemm_tn_partial(const float* A, int64_t lda, const float* B, int64_t ldb,
                                  int64_t M, int32_t N, int32_t K, int32_t prec, float* C,
                                  int64_t ldc, float* db, void* workspace,
                                  int64_t workspace_bytes, void* stream) {
  int pending = 0;
  return gemm_tn_launch(A, lda, B, ldb, M, N, K, prec, C, ldc, db, workspace, workspace_bytes,
                        stream, &pending);
}

namespace {
int fill_tn_jobs(const tt_tn_pending* jobs, int32_t n, TnRedArgs& a, int64_t* total_out) {
  TT_REQUIRE(n >= 0 && n <= TN_RED_MAX && (n == 0 || jobs), "0 <= n <= 8 jobs");
  int64_t total = 0;
  for (int i = 0; i < n; ++i) {
    const tt_tn_pending& q = jobs[i];
    TT_REQUIRE(q.M >= 0 && q.N >= 0 && q.K >= 0, "bad sizes");
    if (q.M == 0 || q.N == 0 || q.K == 0) continue;
    const TnPlan p = tn_plan(q.M, q.N, q.K);
    if (p.S == 1) continue;  // (that GEMM wrote C directly)
    TT_REQUIRE(q.workspace && q.C, "null workspace / C");
    TnRedJob& J = a.j[a.n++];
    const char* ws = (const char*)q.workspace;
    J.parts = (const float*)(ws + p.parts);
    J.dbparts = (const float*)(ws + p.dbparts);
    J.C = q.C;
    J.db = q.db;
    J.ldc = q.ldc;
    J.start = total;
    J.S = p.S;
    J.T = p.NT * p.KT;
    J.KT = p.KT;
    J.NT = p.NT;
    J.N = q.N;
    J.K = q.K;
    total += (int64_t)J.T * TN_T * TN_T + (q.db ? q.N : 0);
  }
  *total_out = total;
  return TT_OK;
}
}  // namespace

extern "C" int tt_gemm_tn_reduce_many(const tt_tn_pending* jobs, int32_t n, void* stream) {
  TnRedArgs a{};
  int64_t total = 0;
  int rc = fill_tn_jobs(jobs, n, a, &total);
  if (rc) return rc;
  if (a.n == 0) return TT_OK;
  hipLaunchKernelGGL(k_tn_reduce_many, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, a);
  return check_launch("k_tn_reduce_many");
}

extern "C" int tt_train_bwd_tail(const tt_tn_pending* jobs, int32_t njobs,
                                 const float* attn_parts, int64_t B, int32_t Hd, float* dW2,
                                 float* db2, const float* g_emb, int64_t ldg,
                                 const int32_t* ids0, const int32_t* ids1, int64_t n_emb,
                                 int32_t C, float* grad0, float* grad1, void* stream) {
  TailArgs a{};
  int rc = fill_tn_jobs(jobs, njobs, a.tn, &a.tn_items);
  if (rc) return rc;
  a.nA = (int)((a.tn_items + 255) / 256);
  TT_REQUIRE(B >= 0 && Hd >= 0 && n_emb >= 0 && C >= 0, "bad sizes");
  if (attn_parts && B > 0) {
    TT_REQUIRE(dW2 && db2 && Hd >= 1, "attention: null dW2 / db2");
    a.part = attn_parts, a.B = (int)B, a.Hd = Hd, a.dW2 = dW2, a.db2 = db2;
    a.nB = (Hd + 1 + 31) / 32;
  }
  int nC = 0;
  if (g_emb && n_emb > 0 && (ids0 || ids1)) {
    TT_REQUIRE(C >= 1 && ldg >= 2 * C && (!ids0 || grad0) && (!ids1 || grad1),
               "embedding: bad ldg / null grads");
    a.g = g_emb, a.ldg = ldg, a.n = n_emb, a.ids0 = ids0, a.ids1 = ids1, a.C = C;
    a.grad0 = grad0, a.grad1 = grad1;
    nC = (int)((2 * n_emb + 3) / 4);
  }
  const int64_t blocks = (int64_t)a.nA + a.nB + nC;
  if (blocks == 0) return TT_OK;
  hipLaunchKernelGGL(k_train_tail, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("k_train_tail");
}

extern "C" int tt_dropout_apply_ex(float* x, const uint8_t* keep, float scale, int64_t n,
                                   uint16_t* x_bf16, void* stream) {
  TT_REQUIRE(n >= 0, "n < 0");
  if (n == 0) return TT_OK;
  TT_REQUIRE(x && keep, "null pointer");
  hipLaunchKernelGGL(k_dropout_ex, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, keep,
                     scale, n, x_bf16);
  return check_launch("tt_dropout_apply_ex");
}

extern "C" int tt_dropout_rng_f32(float* x, int64_t n, float p, uint64_t seed,
                                  const int64_t* counter, uint16_t* x_bf16, void* stream) {
  TT_REQUIRE(n >= 0 && p >= 0.0f && p < 1.0f, "need n >= 0, 0 <= p < 1");
  if (n == 0) return TT_OK;
  TT_REQUIRE(x && counter, "null pointer");
  const double th = (double)p * 4294967296.0;
  const uint32_t thresh = th >= 4294967295.0 ? 0xffffffffu : (uint32_t)th;
  hipLaunchKernelGGL(k_dropout_rng, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, n,
                     thresh, 1.0f / (1.0f - p), seed, counter, x_bf16);
  return check_launch("tt_dropout_rng_f32");
}

extern "C" int tt_embedding_backward2_f32(const float* g, int64_t ldg, const int32_t* ids0,
                                          const int32_t* ids1, int64_t n, int32_t C,
                                          float* grad0, float* grad1, void* stream) {
  TT_REQUIRE(n >= 0 && C >= 1, "bad sizes");
  if (n == 0 || (!ids0 && !ids1)) return TT_OK;
  TT_REQUIRE(g && (!ids0 || grad0) && (!ids1 || grad1) && ldg >= 2 * C, "null pointer / ldg");
  hipLaunchKernelGGL(k_embedding_bwd2, dim3((unsigned)(2 * n)), dim3(64), 0, (hipStream_t)stream,
                     g, ldg, ids0, ids1, n, C, grad0, grad1);
  return check_launch("tt_embedding_backward2_f32");
}

extern "C" int tt_relu_dropout_backward_f32(float* dh, const float* h, float scale, int64_t n,
                                            uint16_t* dh_bf16, int64_t* counter_advance,
                                            void* stream) {
  TT_REQUIRE(n >= 0, "n < 0");
  if (n == 0) return TT_OK;
  TT_REQUIRE(dh && h, "null pointer");
  hipLaunchKernelGGL(k_relu_drop_bwd, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, dh, h,
                     scale, n, dh_bf16, counter_advance);
  return check_launch("tt_relu_dropout_backward_f32");
}

extern "C" int tt_convert_batch(const tt_convert_job* jobs, int32_t njobs, void* stream) {
  TT_REQUIRE(jobs && njobs >= 0 && njobs <= TT_CONVERT_MAX_JOBS, "need 0 <= njobs <= 16");
  tt_convert_batch_args a{};
  int tiles = 0, nj = 0;
  for (int j = 0; j < njobs; ++j) {
    const tt_convert_job& jb = jobs[j];
    TT_REQUIRE(jb.dst && jb.rows >= 0 && jb.cols >= 0 && (!jb.src || jb.ld_src >= jb.cols),
               "bad job");
    TT_REQUIRE(jb.src || !jb.transpose, "a zero-fill job (src NULL) cannot transpose");
    TT_REQUIRE(!jb.row_ids || !jb.transpose, "a gather job (row_ids) cannot transpose");
    TT_REQUIRE(jb.transpose ? jb.ld_dst >= jb.rows : jb.ld_dst >= jb.cols, "bad job ld_dst");
    if (jb.rows == 0 || jb.cols == 0) continue;
    a.jobs[nj] = jb;
    a.tile_off[nj] = tiles;
    if (jb.transpose) {
      const int64_t rr = jb.ld_dst > jb.rows ? jb.ld_dst : jb.rows;
      tiles += (int)(((rr + 31) / 32) * ((jb.cols + 31) / 32));
    } else {
      tiles += (int)(((jb.rows + 8 * CV_RG - 1) / (8 * CV_RG)) * ((jb.cols + 127) / 128));
    }
    ++nj;
  }
  a.njobs = nj;
  if (tiles == 0) return TT_OK;
  hipLaunchKernelGGL(k_convert_batch, dim3((unsigned)tiles), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("tt_convert_batch");
}

extern "C" int tt_l2norm_backward_ex(const float* y, int64_t ldy, const float* z, int64_t ldz,
                                     const float* dz, int64_t lddz, int64_t n, int32_t d,
                                     float* dy, int64_t lddy, uint16_t* dy_bf16, int64_t lddy16,
                                     void* stream) {
  TT_REQUIRE(n >= 0 && d >= 1, "bad sizes");
  if (n == 0) return TT_OK;
  TT_REQUIRE(y && z && dz && dy, "null pointer");
  hipLaunchKernelGGL(k_l2norm_bwd, dim3(grid_for((n + 3) / 4 * 256)), dim3(256), 0,
                     (hipStream_t)stream, y, ldy, z, ldz, dz, lddz, n, d, dy, lddy, dy_bf16,
                     lddy16);
  return check_launch("tt_l2norm_backward_ex");
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
