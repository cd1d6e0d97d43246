// tt_loss.hip -- InfoNCE loss with in-batch negatives, forward + backward (gfx950).
//
// Replaces InfoNCELoss.forward (src/training/losses.py:20-79) and its autograd backward.
// Row i of the logits (all / tau):  [ b_i.p_i | b_i.n_ij (j < N) | b_i.p_k (k < B, k != i:
// the diagonal is -inf, :64-65) ];  loss = mean_i( logsumexp(row_i) - b_i.p_i / tau ).
// The reference materialises the expanded [B, B, E] positives (:55-61); here the in-batch
// block is one GEMM S = b p^T on MFMA, and the backward is two more GEMMs:
//   c = 1 / (tau B),  P = softmax(row),  P0 = P[positive], Pn = P[negatives], Pb = P[in-batch]
//   dL/db_i  = c [ (P0_i - 1) p_i + sum_j Pn_ij n_ij + (Pb p)_i ]
//   dL/dp_k  = c [ (P0_k - 1) b_k + (Pb^T b)_k ]
//   dL/dn_ij = c Pn_ij b_i
// GEMMs (prec f32 / bf16 MFMA): S = b p^T on tt_gemm_f32 / tt_gemm_bf16; the backward's
// Pb . p = (Pb^T)^T p and Pb^T . b on tt_gemm_tn (A^T B from the row-major Pb^T / Pb the row
// kernel writes: no transposed or bf16 operand copies).  The row kernel (logits, softmax,
// per-row loss) and the gradient assembly are HBM/latency-bound and tiny.
#include "tt_common.hpp"

extern "C" int tt_gemm_f32(const float* A, int64_t lda, const float* W, int64_t ldw,
                           const float* bias, const float* residual, int64_t ldr, float* C,
                           int64_t ldc, uint16_t* C_bf16, int64_t ldc16, int32_t M, int32_t N,
                           int32_t K, int32_t act, void* stream);
extern "C" int tt_gemm_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw,
                            const float* bias, const float* residual, int64_t ldr, float* C,
                            int64_t ldc, uint16_t* C_bf16, int64_t ldc16, int32_t M, int32_t N,
                            int32_t K, int32_t act, void* stream);
extern "C" int tt_gemm_tn_workspace_bytes(int64_t M, int32_t N, int32_t K, int64_t* bytes);
extern "C" int tt_gemm_tn(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M,
                          int32_t N, int32_t K, int32_t prec, float* C, int64_t ldc, float* db,
                          void* workspace, int64_t workspace_bytes, void* stream);

namespace tt {

__device__ __forceinline__ float block_sum(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.0f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;
}
__device__ __forceinline__ float block_max(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = -__builtin_huge_valf();
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s = fmaxf(s, red[i]);
  return s;
}

__global__ __launch_bounds__(256) void k_to_bf16(const float* __restrict__ x, int64_t ldx,
                                                 int rows, int E, uint16_t* __restrict__ y,
                                                 int64_t ldy) {
  const int64_t n = (int64_t)rows * E;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / E, e = i % E;
    y[r * ldy + e] = f32_to_bf16_rne(x[r * ldx + e]);
  }
}

// One block per row i: logits, softmax, per-row loss; writes P0[i], Pn[i][j], Pb[i][k]
// (row-major [B, ldp], diagonal and padding 0) and Pb^T (so the backward GEMMs read
// row-major A operands), f32 and/or bf16.
__global__ __launch_bounds__(256) void k_infonce_rows(
    const float* __restrict__ b, int64_t ldb, const float* __restrict__ p, int64_t ldp_in,
    const float* __restrict__ n, int64_t ldn_row, int64_t ldn_item, const float* __restrict__ S,
    int64_t lds, int B, int N, int E, float inv_tau, float* __restrict__ row_loss,
    float* __restrict__ P0, float* __restrict__ Pn, float* __restrict__ Pb,
    float* __restrict__ PbT, uint16_t* __restrict__ Pb16, uint16_t* __restrict__ PbT16, int ldp) {
  __shared__ float red[8];
  __shared__ float lg[1 + 64];  // positive + up to 64 explicit negatives
  const int i = blockIdx.x, tid = threadIdx.x;
  const float* bi = b + (int64_t)i * ldb;
  // the positive and the explicit negatives' logits, 8 dot products per pass (one reduction
  // round for all 8: their loads in flight together)
  __shared__ float red8[8][8];
  for (int j0 = 0; j0 <= N; j0 += 8) {
    float sv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + u;
      float acc = 0.0f;
      if (j <= N) {
        const float* y = j == 0 ? p + (int64_t)i * ldp_in
                                : n + (int64_t)i * ldn_row + (int64_t)(j - 1) * ldn_item;
        for (int e = tid; e < E; e += 256) acc = fmaf(bi[e], y[e], acc);
      }
      for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
      sv[u] = acc;
    }
    if ((tid & 63) == 0)
#pragma unroll
      for (int u = 0; u < 8; ++u) red8[tid >> 6][u] = sv[u];
    __syncthreads();
    if (tid < 8 && j0 + tid <= N) {
      float t = 0.0f;
      for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red8[w][tid];
      lg[j0 + tid] = t * inv_tau;
    }
    __syncthreads();
  }
  const float* Si = S + (int64_t)i * lds;
  float mx = -__builtin_huge_valf();
  for (int j = tid; j <= N; j += 256) mx = fmaxf(mx, lg[j]);
  for (int k = tid; k < B; k += 256)
    if (k != i) mx = fmaxf(mx, Si[k] * inv_tau);
  mx = block_max(mx, red);
  float se = 0.0f;
  for (int j = tid; j <= N; j += 256) se += expf(lg[j] - mx);
  for (int k = tid; k < B; k += 256)
    if (k != i) se += expf(Si[k] * inv_tau - mx);
  se = block_sum(se, red);
  const float lse = mx + logf(se);
  if (tid == 0) row_loss[i] = lse - lg[0];
  const float inv_se = 1.0f / se;
  if (P0 && tid == 0) P0[i] = expf(lg[0] - mx) * inv_se;
  if (Pn)
    for (int j = tid; j < N; j += 256) Pn[(int64_t)i * N + j] = expf(lg[j + 1] - mx) * inv_se;
  if (Pb || Pb16)
    for (int k = tid; k < ldp; k += 256) {
      const float v = (k < B && k != i) ? expf(Si[k] * inv_tau - mx) * inv_se : 0.0f;
      if (Pb) Pb[(int64_t)i * ldp + k] = v;
      if (PbT && k < B) PbT[(int64_t)k * ldp + i] = v;
      if (Pb16) Pb16[(int64_t)i * ldp + k] = f32_to_bf16_rne(v);
      if (PbT16 && k < B) PbT16[(int64_t)k * ldp + i] = f32_to_bf16_rne(v);
    }
}

__global__ __launch_bounds__(256) void k_mean(const float* __restrict__ v, int n, float* out) {
  __shared__ float red[8];
  float s = 0.0f;
  for (int i = threadIdx.x; i < n; i += 256) s += v[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) *out = s / (float)n;
}

// gradient assembly, block per row i
__global__ __launch_bounds__(256) void k_infonce_grads(
    const float* __restrict__ b, int64_t ldb, const float* __restrict__ p, int64_t ldp_in,
    const float* __restrict__ n, int64_t ldn_row, int64_t ldn_item, int B, int N, int E, float c,
    const float* __restrict__ P0, const float* __restrict__ Pn, const float* __restrict__ G1,
    const float* __restrict__ G2, int64_t ldg, float* __restrict__ gb, int64_t ldgb,
    float* __restrict__ gp, int64_t ldgp, float* __restrict__ gn, int64_t ldgn_row,
    int64_t ldgn_item, const float* __restrict__ row_loss, float* __restrict__ loss) {
  const int i = blockIdx.x;
  if (i == 0 && loss) {  // the mean loss (k_mean's sum, in the same order), no launch of its own
    __shared__ float red[8];
    float sl = 0.0f;
    for (int r = threadIdx.x; r < B; r += 256) sl += row_loss[r];
    sl = block_sum(sl, red);
    if (threadIdx.x == 0) *loss = sl / (float)B;
  }
  const float a0 = P0[i] - 1.0f;
  const float* bi = b + (int64_t)i * ldb;
  const float* pi = p + (int64_t)i * ldp_in;
  for (int e = threadIdx.x; e < E; e += 256) {
    if (gb) {
      float v = a0 * pi[e];
      for (int j = 0; j < N; ++j)
        v = fmaf(Pn[(int64_t)i * N + j], n[(int64_t)i * ldn_row + (int64_t)j * ldn_item + e], v);
      gb[(int64_t)i * ldgb + e] = c * (v + G1[(int64_t)i * ldg + e]);
    }
    if (gp) gp[(int64_t)i * ldgp + e] = c * (a0 * bi[e] + G2[(int64_t)i * ldg + e]);
    if (gn)
      for (int j = 0; j < N; ++j)
        gn[(int64_t)i * ldgn_row + (int64_t)j * ldgn_item + e] = c * Pn[(int64_t)i * N + j] * bi[e];
  }
}

}  // namespace tt

using namespace tt;

namespace {
size_t al(size_t b) { return (b + 255) / 256 * 256; }
struct NceWs {
  float *S, *row_loss, *P0, *Pn, *Pb, *PbT, *G1, *G2;
  uint16_t *b16, *p16;
  char *tn, *tn2;
  int64_t tn_bytes;
  size_t total;
};
NceWs nce_carve(char* base, int B, int N, int E, bool bf, bool grads) {
  NceWs w{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* r = base ? base + off : nullptr;
    off += al(bytes);
    return r;
  };
  const int Bp = (B + 63) / 64 * 64;
  w.S = (float*)take((size_t)B * B * 4);
  w.row_loss = (float*)take((size_t)B * 4);
  if (bf) {
    w.b16 = (uint16_t*)take((size_t)B * E * 2);
    w.p16 = (uint16_t*)take((size_t)B * E * 2);
  }
  if (grads) {
    w.P0 = (float*)take((size_t)B * 4);
    w.Pn = (float*)take((size_t)B * (N > 0 ? N : 1) * 4);
    w.G1 = (float*)take((size_t)B * E * 4);
    w.G2 = (float*)take((size_t)B * E * 4);
    w.Pb = (float*)take((size_t)B * Bp * 4);
    w.PbT = (float*)take((size_t)B * Bp * 4);
    int64_t tb = 0;
    tt_gemm_tn_workspace_bytes(B, B, E, &tb);
    w.tn_bytes = tb;
    w.tn = take((size_t)tb);
    w.tn2 = take((size_t)tb);  // G2's splits (both products are reduced in one launch)
  }
  w.total = off;
  return w;
}
}  // namespace

extern "C" int tt_infonce_workspace_bytes(int32_t B, int32_t N, int32_t E, int32_t prec,
                                          int32_t with_grads, int64_t* bytes) {
  TT_REQUIRE(bytes && B >= 1 && N >= 0 && E >= 1, "bad arguments");
  *bytes = (int64_t)nce_carve(nullptr, B, N, E, prec == TT_PREC_BF16, with_grads != 0).total;
  return TT_OK;
}

namespace {
int infonce(const float* b, int64_t ldb, const float* p, int64_t ldp, const float* n,
            int64_t ldn_row, int64_t ldn_item, int32_t B, int32_t N, int32_t E, float temperature,
            int32_t prec, float* loss, float* grad_b, float* grad_p, float* grad_n,
            void* workspace, int64_t workspace_bytes, const uint16_t* b16_in, int64_t ldb16,
            const uint16_t* p16_in, int64_t ldp16, void* stream);
}

extern "C" int tt_infonce_f32(const float* b, int64_t ldb, const float* p, int64_t ldp,
                              const float* n, int64_t ldn_row, int64_t ldn_item, int32_t B,
                              int32_t N, int32_t E, float temperature, int32_t prec,
                              float* loss, float* grad_b, float* grad_p, float* grad_n,
                              void* workspace, int64_t workspace_bytes, void* stream) {
  return infonce(b, ldb, p, ldp, n, ldn_row, ldn_item, B, N, E, temperature, prec, loss, grad_b,
                 grad_p, grad_n, workspace, workspace_bytes, nullptr, 0, nullptr, 0, stream);
}

extern "C" int tt_infonce_ex(const float* b, int64_t ldb, const float* p, int64_t ldp,
                             const float* n, int64_t ldn_row, int64_t ldn_item, int32_t B,
                             int32_t N, int32_t E, float temperature, int32_t prec, float* loss,
                             float* grad_b, float* grad_p, float* grad_n, void* workspace,
                             int64_t workspace_bytes, const uint16_t* b_bf16, int64_t ldb16,
                             const uint16_t* p_bf16, int64_t ldp16, void* stream) {
  return infonce(b, ldb, p, ldp, n, ldn_row, ldn_item, B, N, E, temperature, prec, loss, grad_b,
                 grad_p, grad_n, workspace, workspace_bytes, b_bf16, ldb16, p_bf16, ldp16,
                 stream);
}

namespace {
int infonce(const float* b, int64_t ldb, const float* p, int64_t ldp, const float* n,
            int64_t ldn_row, int64_t ldn_item, int32_t B, int32_t N, int32_t E, float temperature,
            int32_t prec, float* loss, float* grad_b, float* grad_p, float* grad_n,
            void* workspace, int64_t workspace_bytes, const uint16_t* b16_in, int64_t ldb16,
            const uint16_t* p16_in, int64_t ldp16, void* stream) {
  TT_REQUIRE(B >= 1 && N >= 0 && N <= 64 && E >= 1, "need B >= 1, 0 <= N <= 64, E >= 1");
  TT_REQUIRE(temperature > 0.0f, "temperature must be > 0");
  TT_REQUIRE(prec == TT_PREC_F32 || prec == TT_PREC_BF16, "bad precision");
  TT_REQUIRE(b && p && loss && (N == 0 || n), "null pointer");
  const bool bf = prec == TT_PREC_BF16;
  const int BK = bf ? 64 : 32;
  if (E % BK != 0) return fail(TT_ERR_UNSUPPORTED, "tt_infonce_f32: E must be a multiple of 32 (f32) / 64 (bf16)");
  const bool grads = grad_b || grad_p || grad_n;
  NceWs w = nce_carve((char*)workspace, B, N, E, bf, grads);
  if (!workspace || workspace_bytes < (int64_t)w.total)
    return fail(TT_ERR_WORKSPACE, "tt_infonce_f32: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const float inv_tau = 1.0f / temperature;
  const int Bp = (B + 63) / 64 * 64;
  int rc;
  // S = b p^T  [B, B]
  if (bf) {  // bf16 operands: the caller's copies (tt_infonce_ex) or converted here
    const unsigned g = (unsigned)(((int64_t)B * E + 255) / 256 < 4096 ? ((int64_t)B * E + 255) / 256 : 4096);
    const uint16_t *b16 = b16_in, *p16 = p16_in;
    if (!b16) {
      hipLaunchKernelGGL(k_to_bf16, dim3(g), dim3(256), 0, st, b, ldb, B, E, w.b16, (int64_t)E);
      b16 = w.b16, ldb16 = E;
    }
    if (!p16) {
      hipLaunchKernelGGL(k_to_bf16, dim3(g), dim3(256), 0, st, p, ldp, B, E, w.p16, (int64_t)E);
      p16 = w.p16, ldp16 = E;
    }
    rc = tt_gemm_bf16(b16, ldb16, p16, ldp16, nullptr, nullptr, 0, w.S, B, nullptr, 0, B, B, E, 0,
                      stream);
  } else {
    rc = tt_gemm_f32(b, ldb, p, ldp, nullptr, nullptr, 0, w.S, B, nullptr, 0, B, B, E, 0, stream);
  }
  if (rc) return rc;
  hipLaunchKernelGGL(k_infonce_rows, dim3(B), dim3(256), 0, st, b, ldb, p, ldp, n, ldn_row,
                     ldn_item, w.S, (int64_t)B, B, N, E, inv_tau, w.row_loss, w.P0,
                     N > 0 ? w.Pn : nullptr, w.Pb, w.PbT, (uint16_t*)nullptr,
                     (uint16_t*)nullptr, Bp);
  if ((rc = check_launch("k_infonce_rows"))) return rc;
  if (!grads) {
    hipLaunchKernelGGL(k_mean, dim3(1), dim3(256), 0, st, w.row_loss, B, loss);
    return check_launch("k_mean");
  }
  // G1 = Pb . p = (Pb^T)^T p;  G2 = Pb^T . b   (row-major Pb^T / Pb as the A^T operands)
  // (the two products' split sums reduced by one launch)
  rc = tt_gemm_tn_partial(w.PbT, Bp, p, ldp, B, B, E, prec, w.G1, E, nullptr, w.tn, w.tn_bytes,
                          stream);
  if (!rc)
    rc = tt_gemm_tn_partial(w.Pb, Bp, b, ldb, B, B, E, prec, w.G2, E, nullptr, w.tn2, w.tn_bytes,
                            stream);
  if (!rc) {
    const tt_tn_pending jobs[2] = {{w.tn, B, B, E, w.G1, E, nullptr},
                                   {w.tn2, B, B, E, w.G2, E, nullptr}};
    rc = tt_gemm_tn_reduce_many(jobs, 2, stream);
  }
  if (rc) return rc;
  hipLaunchKernelGGL(k_infonce_grads, dim3(B), dim3(256), 0, st, b, ldb, p, ldp, n, ldn_row,
                     ldn_item, B, N, E, inv_tau / (float)B, w.P0, w.Pn, w.G1, w.G2, (int64_t)E,
                     grad_b, (int64_t)E, grad_p, (int64_t)E, grad_n, (int64_t)N * E, (int64_t)E,
                     w.row_loss, loss);
  return check_launch("k_infonce_grads");
}

}  // namespace

extern "C" int tt_f32_to_bf16(const float* x, int64_t ldx, int32_t rows, int32_t cols, uint16_t* y,
                              int64_t ldy, void* stream) {
  TT_REQUIRE(rows >= 0 && cols >= 0, "bad sizes");
  if (rows == 0 || cols == 0) return TT_OK;
  TT_REQUIRE(x && y, "null pointer");
  const int64_t n = (int64_t)rows * cols;
  const unsigned g = (unsigned)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192);
  hipLaunchKernelGGL(k_to_bf16, dim3(g), dim3(256), 0, (hipStream_t)stream, x, ldx, rows, cols, y,
                     ldy);
  return check_launch("tt_f32_to_bf16");
}
