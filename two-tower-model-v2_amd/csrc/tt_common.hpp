// tt_common.hpp -- shared device/host helpers for libtwotower_hip.so (gfx950 only).
//
// Canonical float32 numerics shared by every kernel (restated on the CPU in
// oracle/tt_oracle.c; DESIGN.md "Canonical numerics"):
//   * pairwise_sumsq: numpy's float32 pairwise sum of x*x (loops_utils.h pairwise_sum:
//     n<8 sequential, n<=128 eight interleaved accumulators, else split at
//     n/2 - (n/2)%8).  np.linalg.norm(axis=1) == sqrtf(pairwise_sumsq) bit-for-bit.
//   * dot (scan score): fmaf chain, d = 16t + 4g + i visited in (t, i, g) order --
//     exactly what a chain of v_mfma_f32_16x16x4_f32 computes when lane-group g holds
//     dims 16t+4g..16t+4g+3 (see tt_scan.hip).
//   * top-k order: score descending, ties -> lower row; NaN never selected.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string>

#include "../../include/twotower_hip.h"

#include <type_traits>
namespace tt {

// ----------------------------------------------------------------------------- errors
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int check_launch(const char* what);

#define TT_REQUIRE(cond, msg)                                                     \
  do {                                                                            \
    if (!(cond)) return ::tt::fail(TT_ERR_INVALID, std::string(__func__) + ": " + (msg)); \
  } while (0)

// ----------------------------------------------------------------------------- A/B switches
// Alternate kernel paths kept for A/B timing are chosen from the environment ONLY in a
// timing build (-DTT_TIMING_BUILD, tools/exp_*.sh).  The shipped library ignores the
// environment and always runs the default path -- the one the GPU tests cover.
#ifdef TT_TIMING_BUILD
inline int env_switch(const char* name, int dflt) {
  const char* e = getenv(name);
  return e && e[0] >= '0' && e[0] <= '9' ? e[0] - '0' : dflt;
}
#else
inline int env_switch(const char*, int dflt) { return dflt; }
#endif
// A compile-time experiment macro that changes results (or the tested schedule) may only be
// set in a timing build: `#error` otherwise (see the users of TT_CHECK_EXP).
#ifdef TT_TIMING_BUILD
#define TT_CHECK_EXP(cond, what)
#else
#define TT_CHECK_EXP(cond, what) static_assert(!(cond), what " is a timing-only switch: build with -DTT_TIMING_BUILD")
#endif

// ----------------------------------------------------------------------------- device utils
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

// a float >= v (v >= 0, finite): rounding UP of an f64 bound
__device__ __forceinline__ float f64_up(double v) {
  const float f = (float)v;
  return (double)f >= v ? f : __uint_as_float(__float_as_uint(f) + 1u);
}

// XCD-aware block id: blocks b and b+8 run on the same XCD (observed placement, speed only).
// Give every XCD a contiguous range of logical ids so that blocks sharing data (the slabs of
// a filter level, the heads of one sequence in attention) share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int q = nblk / 8, r = nblk % 8, x = bid % 8, local = bid / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + local;
}

// Orders LDS traffic between lanes of ONE wave (no workgroup barrier: waves of a block
// run independent control flow in the scan kernel).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave64 scans / reductions on DPP lane moves (VALU, a few cycles per step).  __shfl is a
// ds_bpermute through the LDS pipe: ~100+ cycles of latency per dependent step, which is what
// a one-block latency-bound kernel (the small-batch final) spends its time on.
// Inclusive prefix sum over lanes 0..63: row_shr 1/2/4/8 within rows of 16, then row_bcast 15
// (row r's total into row r + 1, rows 1 and 3) and row_bcast 31 (rows 0-1's total into rows
// 2 and 3).  Lanes whose source is outside the row read 0 (old = 0, bound_ctrl off).
__device__ __forceinline__ int wave_incl_sum(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
  return x;
}
__device__ __forceinline__ int wave_sum(int x) {
  return __builtin_amdgcn_readlane(wave_incl_sum(x), 63);
}
// max over the wave of unsigned values (0 = identity), same DPP pattern
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  int x = (int)v;
  auto mx = [](int a, int b) { return (int)((uint32_t)a > (uint32_t)b ? (uint32_t)a : (uint32_t)b); };
  x = mx(x, __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false));
  x = mx(x, __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false));
  x = mx(x, __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false));
  x = mx(x, __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false));
  x = mx(x, __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false));
  x = mx(x, __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false));
  return (uint32_t)__builtin_amdgcn_readlane(x, 63);
}
// sum over aligned lane quads (lanes 4i .. 4i + 3), result in every lane of the quad
__device__ __forceinline__ int quad_sum(int x) {
  x += __builtin_amdgcn_mov_dpp(x, 0xb1, 0xf, 0xf, false);  // quad_perm [1, 0, 3, 2]
  x += __builtin_amdgcn_mov_dpp(x, 0x4e, 0xf, 0xf, false);  // quad_perm [2, 3, 0, 1]
  return x;
}

// Monotone map float -> uint32 (larger float -> larger key).  -0 is folded to +0 so that
// equal scores compare equal; NaN maps to 0 (below every finite value and -inf).
__device__ __forceinline__ uint32_t float_key(float f) {
  if (f != f) return 0u;
  f = f + 0.0f;  // -0 -> +0 under round-to-nearest
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_float(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}
// 64-bit sort key: high word = score key, low word = ~row (lower row wins a tie).
__device__ __forceinline__ uint64_t make_key(float score, uint32_t row) {
  return ((uint64_t)float_key(score) << 32) | (uint64_t)(0xffffffffu - row);
}
__device__ __forceinline__ float key_score(uint64_t k) { return key_float((uint32_t)(k >> 32)); }
__device__ __forceinline__ uint32_t key_row(uint64_t k) { return 0xffffffffu - (uint32_t)k; }

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  lo = __shfl_xor(lo, m, 64);
  hi = __shfl_xor(hi, m, 64);
  return ((uint64_t)hi << 32) | lo;
}

// Value of lane (lane ^ M): DPP for M < 16 (quad_perm, or a row shift left / right picked by
// the lane's bit M: VALU moves, a few cycles), ds_bpermute (__shfl_xor) for M = 16, 32.  The
// whole wave must be active (a DPP read of a disabled lane does not return its register).
template <int M>
__device__ __forceinline__ uint32_t lane_xor_u32(uint32_t x, int lane) {
  if constexpr (M == 1) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xb1, 0xf, 0xf, false);  // [1,0,3,2]
  } else if constexpr (M == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4e, 0xf, 0xf, false);  // [2,3,0,1]
  } else if constexpr (M == 4 || M == 8) {
    const uint32_t up = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x100 + M, 0xf, 0xf, false);
    const uint32_t dn = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x110 + M, 0xf, 0xf, false);
    return (lane & M) ? dn : up;  // row_shl M: lane i reads i + M; row_shr M: i - M
  } else {
    return (uint32_t)__shfl_xor((int)x, M, 64);
  }
}
template <int M>
__device__ __forceinline__ uint64_t lane_xor_u64(uint64_t v, int lane) {
  const uint32_t lo = lane_xor_u32<M>((uint32_t)v, lane);
  const uint32_t hi = lane_xor_u32<M>((uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

// Bitonic sort, descending, of 64*PER keys held PER per lane (element e = lane*PER + r), the
// whole wave active.  Stages unrolled at compile time so the lane exchanges (lane ^ stride/PER)
// are DPP moves except for partner distances 16 and 32 (3 of the 21 cross-lane stages at
// PER = 4): the ds_bpermute exchange of every stage (~100+ cycles of latency each) made a
// 256-key sort ~2.5 us.
template <int PER, int SIZE, int STRIDE>
__device__ __forceinline__ void bitonic_steps(uint64_t (&key)[PER], int lane) {
  if constexpr (STRIDE >= PER) {
    constexpr int LM = STRIDE / PER;
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      const int e = lane * PER + r;
      const uint64_t o = lane_xor_u64<LM>(key[r], lane);
      const bool up = (e & SIZE) == 0;
      const bool lower = (e & STRIDE) == 0;
      const bool keep_max = (lower == up);
      const uint64_t mx = key[r] > o ? key[r] : o;
      const uint64_t mn = key[r] > o ? o : key[r];
      key[r] = keep_max ? mx : mn;
    }
  } else {
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      if ((r & STRIDE) == 0) {
        const int r2 = r | STRIDE;
        const int e = lane * PER + r;
        const bool up = (e & SIZE) == 0;
        const uint64_t a = key[r], b = key[r2];
        const uint64_t mx = a > b ? a : b, mn = a > b ? b : a;
        key[r] = up ? mx : mn;
        key[r2] = up ? mn : mx;
      }
    }
  }
  if constexpr (STRIDE > 1) bitonic_steps<PER, SIZE, STRIDE / 2>(key, lane);
}
template <int PER, int SIZE>
__device__ __forceinline__ void bitonic_sizes(uint64_t (&key)[PER], int lane) {
  bitonic_steps<PER, SIZE, SIZE / 2>(key, lane);
  if constexpr (SIZE < 64 * PER) bitonic_sizes<PER, SIZE * 2>(key, lane);
}
template <int PER>
__device__ __forceinline__ void bitonic_desc(uint64_t (&key)[PER], int lane) {
  bitonic_sizes<PER, 2>(key, lane);
}

// Sort each row of 16 lanes (one key per lane) descending: the bitonic network of 16 on DPP
// exchanges only (10 stages).  Row 0 (lanes 0..15) comes out descending; the other rows are
// sorted too, in either direction (callers use row 0).
__device__ __forceinline__ void bitonic_desc16_rows(uint64_t& key, int lane) {
  auto step = [&](auto size_, auto stride_) __attribute__((always_inline)) {
    constexpr int SIZE = decltype(size_)::value, STRIDE = decltype(stride_)::value;
    const uint64_t o = lane_xor_u64<STRIDE>(key, lane);
    const bool keep_max = ((lane & STRIDE) == 0) == ((lane & SIZE) == 0);
    const uint64_t mx = key > o ? key : o, mn = key > o ? o : key;
    key = keep_max ? mx : mn;
  };
  using std::integral_constant;
  step(integral_constant<int, 2>{}, integral_constant<int, 1>{});
  step(integral_constant<int, 4>{}, integral_constant<int, 2>{});
  step(integral_constant<int, 4>{}, integral_constant<int, 1>{});
  step(integral_constant<int, 8>{}, integral_constant<int, 4>{});
  step(integral_constant<int, 8>{}, integral_constant<int, 2>{});
  step(integral_constant<int, 8>{}, integral_constant<int, 1>{});
  step(integral_constant<int, 16>{}, integral_constant<int, 8>{});
  step(integral_constant<int, 16>{}, integral_constant<int, 4>{});
  step(integral_constant<int, 16>{}, integral_constant<int, 2>{});
  step(integral_constant<int, 16>{}, integral_constant<int, 1>{});
}

// Top 16 of the nonzero keys held PER per lane (whole wave active), without sorting them
// all: the 16th largest high word x is built MSB-first (32 steps; a step counts the keys with
// hi >= candidate by ballot + scalar popcount), ties at x resolved by the same search on the
// low word among them; the <= 16 winners are placed by ballot prefix into lanes 0..15 through
// `scratch` (LDS, 16 entries; the caller orders it against other LDS use) and sorted there
// (bitonic_desc16_rows).  Returns lane i < n's key (i-th largest), 0 in the other lanes;
// *n_out = min(16, #nonzero).  (A full bitonic sort of 128-256 64-bit keys per compaction:
// ~2-3.6 us of one wave; this: a few hundred scalar-heavy instructions.)
template <int PER>
__device__ __forceinline__ uint64_t wave_top16(const uint64_t (&key)[PER], int lane,
                                               uint64_t* scratch, int* n_out) {
  int total = 0;
#pragma unroll
  for (int r = 0; r < PER; ++r) total += __popcll(__ballot(key[r] != 0ull));
  uint32_t x = 0u, xl = 0u;  // select: hi > x, or hi == x and lo >= xl
  if (total > 16) {
#pragma unroll 1
    for (int bit = 31; bit >= 0; --bit) {
      const uint32_t cand = x | (1u << bit);
      int c = 0;
#pragma unroll
      for (int r = 0; r < PER; ++r) c += __popcll(__ballot((uint32_t)(key[r] >> 32) >= cand));
      if (c >= 16) x = cand;
    }
    int gt = 0, eq = 0;
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      const uint32_t h = (uint32_t)(key[r] >> 32);
      gt += __popcll(__ballot(h > x));
      eq += __popcll(__ballot(h == x));
    }
    const int need = 16 - gt;  // >= 1 ties to take
    if (eq > need) {
#pragma unroll 1
      for (int bit = 31; bit >= 0; --bit) {
        const uint32_t cand = xl | (1u << bit);
        int c = 0;
#pragma unroll
        for (int r = 0; r < PER; ++r)
          c += __popcll(__ballot((uint32_t)(key[r] >> 32) == x && (uint32_t)key[r] >= cand));
        if (c >= need) xl = cand;
      }
    }
  } else {
    x = 1u;  // every nonzero key (a real key's high word is >= 1)
  }
  int base = 0;
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const uint32_t h = (uint32_t)(key[r] >> 32);
    const bool sel = key[r] != 0ull && (h > x || (h == x && (uint32_t)key[r] >= xl));
    const uint64_t bm = __ballot(sel);
    const int pos = base + (int)__builtin_amdgcn_mbcnt_hi(
                               (uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
    if (sel) scratch[pos] = key[r];
    base += __popcll(bm);
  }
  wave_sync();
  const int n = base < 16 ? base : 16;
  uint64_t k = lane < n ? scratch[lane] : 0ull;
  wave_sync();
  bitonic_desc16_rows(k, lane);
  *n_out = n;
  return lane < 16 ? k : 0ull;
}

// numpy pairwise float32 sum of v[i]*v[i] (i < n, stride 1), sequential in ONE lane.
// Recursion is unrolled into an explicit post-order walk (depth <= 24).
__device__ __forceinline__ float pw_leaf_sumsq(const float* a, int n) {
  if (n < 8) {
    float res = 0.0f;
    for (int i = 0; i < n; ++i) res = res + __fmul_rn(a[i], a[i]);
    return res;
  }
  float r0 = __fmul_rn(a[0], a[0]), r1 = __fmul_rn(a[1], a[1]);
  float r2 = __fmul_rn(a[2], a[2]), r3 = __fmul_rn(a[3], a[3]);
  float r4 = __fmul_rn(a[4], a[4]), r5 = __fmul_rn(a[5], a[5]);
  float r6 = __fmul_rn(a[6], a[6]), r7 = __fmul_rn(a[7], a[7]);
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
    r0 = r0 + __fmul_rn(a[i + 0], a[i + 0]);
    r1 = r1 + __fmul_rn(a[i + 1], a[i + 1]);
    r2 = r2 + __fmul_rn(a[i + 2], a[i + 2]);
    r3 = r3 + __fmul_rn(a[i + 3], a[i + 3]);
    r4 = r4 + __fmul_rn(a[i + 4], a[i + 4]);
    r5 = r5 + __fmul_rn(a[i + 5], a[i + 5]);
    r6 = r6 + __fmul_rn(a[i + 6], a[i + 6]);
    r7 = r7 + __fmul_rn(a[i + 7], a[i + 7]);
  }
  float res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res = res + __fmul_rn(a[i], a[i]);
  return res;
}

__device__ __forceinline__ float pw_sumsq_serial(const float* a, int n) {
  if (n <= 128) return pw_leaf_sumsq(a, n);
  // explicit stack: entries are (start, len) to expand, or len == -1 meaning "combine".
  int st_s[48], st_n[48];
  float val[24];
  int sp = 0, vp = 0;
  st_s[sp] = 0; st_n[sp] = n; ++sp;
  while (sp > 0) {
    --sp;
    const int s = st_s[sp], len = st_n[sp];
    if (len < 0) {
      const float b = val[--vp];
      const float a0 = val[--vp];
      val[vp++] = a0 + b;
    } else if (len <= 128) {
      val[vp++] = pw_leaf_sumsq(a + s, len);
    } else {
      int n2 = len / 2;
      n2 -= n2 % 8;
      st_s[sp] = 0; st_n[sp] = -1; ++sp;           // combine after both halves
      st_s[sp] = s + n2; st_n[sp] = len - n2; ++sp;  // right half (processed second)
      st_s[sp] = s; st_n[sp] = n2; ++sp;             // left half (processed first)
    }
  }
  return val[0];
}

// Wave-parallel version for a row held in LDS: valid when numpy's recursion tree is a
// perfect binary tree of depth D <= 3 (true for d = 384, 768 and most d <= 1024).  Leaf
// b (of 2^D) is found by walking the split rule; lane 8b+j owns accumulator r_j of leaf b.
// Returns the sum in every lane.  `depth` < 0 means "not perfect": caller uses the serial path.
__host__ __device__ inline int pw_perfect_depth(int n) {
  // returns D if the split tree is perfect with D <= 3, else -1
  int lens[8] = {n, 0, 0, 0, 0, 0, 0, 0};
  int cnt = 1;
  for (int D = 0; D <= 3; ++D) {
    bool all_leaf = true, any_leaf = false;
    for (int i = 0; i < cnt; ++i) {
      if (lens[i] <= 128) any_leaf = true; else all_leaf = false;
    }
    if (all_leaf) return D;
    if (any_leaf || D == 3) return -1;
    int nl[8];
    for (int i = 0; i < cnt; ++i) {
      int n2 = lens[i] / 2;
      n2 -= n2 % 8;
      nl[2 * i] = n2;
      nl[2 * i + 1] = lens[i] - n2;
    }
    cnt *= 2;
    for (int i = 0; i < cnt; ++i) lens[i] = nl[i];
  }
  return -1;
}

__device__ __forceinline__ float pw_sumsq_wave(const float* row, int n, int depth, int lane) {
  const int leaf = lane >> 3, j = lane & 7;
  float r = 0.0f;
  int s = 0, len = n;
  const bool active = leaf < (1 << depth);
  if (active) {
    for (int lvl = depth - 1; lvl >= 0; --lvl) {
      int n2 = len / 2;
      n2 -= n2 % 8;
      if ((leaf >> lvl) & 1) { s += n2; len -= n2; } else { len = n2; }
    }
  }
  const float* a = row + s;
  const bool small = len < 8;
  if (active && !small) {
    r = __fmul_rn(a[j], a[j]);
    for (int i = 8 + j; i < len - (len % 8); i += 8) r = r + __fmul_rn(a[i], a[i]);
  }
  // ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)): the xor butterfly reproduces it (each + commutes)
  r = r + __shfl_xor(r, 1, 64);
  r = r + __shfl_xor(r, 2, 64);
  r = r + __shfl_xor(r, 4, 64);
  if (active) {
    if (small) {
      r = 0.0f;
      for (int i = 0; i < len; ++i) r = r + __fmul_rn(a[i], a[i]);
    } else {
      for (int i = len - (len % 8); i < len; ++i) r = r + __fmul_rn(a[i], a[i]);
    }
  }
  // inter-leaf tree: pw(left) + pw(right), perfect tree -> butterfly over leaf groups
  for (int lvl = 0; lvl < depth; ++lvl) r = r + __shfl_xor(r, 8 << lvl, 64);
  return __shfl(r, 0, 64);
}

// F.normalize / vector_db denominators (canonical: IEEE sqrt + IEEE div, no fast math)
__device__ __forceinline__ float norm_denom(float sumsq, int mode) {
  const float nrm = sqrtf(sumsq);  // correctly rounded (__fsqrt_rn lowers to the 1-ulp v_sqrt_f32)
  return mode == TT_NORM_ADD_EPS ? nrm + 1e-8f : fmaxf(nrm, 1e-12f);
}

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}


typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
// Hand-issued LDS reads with counted waits (the compiler drains lgkmcnt(0) before every use
// of its own reads).  lds_wait<N> waits until at most N LDS operations are outstanding;
// reg_tie pins a consumer below the wait that made its register valid.
template <int OFF>
__device__ __forceinline__ u32x4_t lds_read128(uint32_t addr) {
  u32x4_t r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
  return r;
}
template <int N>
__device__ __forceinline__ void lds_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N));
}
__device__ __forceinline__ void reg_tie(u32x4_t& r) { asm volatile("" : "+v"(r)); }
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

}  // namespace tt
