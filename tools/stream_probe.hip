// Streaming probe (timing only, not product code): how fast can 256 blocks read a 1M x 384
// int8 image straight into VGPRs, as a register-fed form of the int8 single pass would, with
// the lane mapping the MFMA operand wants (lane (g, col) = row col of a 16-row block) instead
// of the fully coalesced one?  Each wave streams its own 16-row blocks (6 KB), D blocks in
// flight, no LDS and no barrier.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stream_probe.hip -o tools/bin/stream_probe
//   ./tools/bin/stream_probe            (prints one line per variant)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);           \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

constexpr int E = 384, KS = 6;

// MAP 0: coalesced (instruction s: lane i reads bytes s*1024 + 16 i of the 6-KB block)
// MAP 1: lane (g, col) reads row col, bytes 96 g + 16 s (contiguous 96 B per lane)
// MAP 2: lane (g, col) reads row col, bytes 64 s + 16 g (the ring kernel's MFMA layout)
template <int MAP>
__device__ __forceinline__ uint32_t lane_off(int lane, int s) {
  const int col = lane & 15, g = lane >> 4;
  if (MAP == 0) return (uint32_t)(s * 1024 + 16 * lane);
  if (MAP == 1) return (uint32_t)(col * E + 96 * g + 16 * s);
  return (uint32_t)(col * E + 64 * s + 16 * g);
}

typedef int32_t v4i __attribute__((ext_vector_type(4)));

// asm loads with explicit counted waits: the compiler neither tracks nor waits for them, so
// slot d is consumed after vmcnt((D - 1) * KS) -- the younger slots stay in flight
template <int MAP, int D, int NW, int MF>
__global__ __launch_bounds__(64 * NW, 1) void k_probe_asm(const int8_t* __restrict__ x,
                                                          int64_t n, int rows_per_blk,
                                                          uint32_t* out) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t j0 = (int64_t)blockIdx.x * rows_per_blk;
  int64_t j1 = j0 + rows_per_blk;
  j1 = j1 < n ? j1 : n;
  const int nb = j0 < j1 ? (int)((j1 - j0) / 16) : 0;
  const uint64_t base = (uint64_t)(x + j0 * E);
  v4i rs;
  rs[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)base);
  rs[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(base >> 32) & 0xffff);
  rs[2] = __builtin_amdgcn_readfirstlane(j0 < j1 ? (int)((j1 - j0) * E) : 0);
  rs[3] = 0x00020000;
  uint32_t off[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) off[s] = lane_off<MAP>(lane, s);
  u32x4 buf[D][KS];
  i32x4 acc = {0, 0, 0, 0};
  const u32x4 qf = {0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u};
  auto load = [&](int slot, int b) __attribute__((always_inline)) {
    const uint32_t bo = (uint32_t)b * 16u * E;
#pragma unroll
    for (int s = 0; s < KS; ++s)
      asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen nt"
                   : "=v"(buf[slot][s])
                   : "v"(bo + off[s]), "s"(rs)
                   : "memory");
  };
  int b = w;
#pragma unroll
  for (int d = 0; d < D; ++d) load(d, b + d * NW);
  for (; b < nb; b += D * NW) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int bb = b + d * NW;
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * KS) : "memory");
#pragma unroll
      for (int s = 0; s < KS; ++s) asm volatile("" : "+v"(buf[d][s]));
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if (MF)
          acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, buf[d][s]),
                                                      __builtin_bit_cast(i32x4, qf), acc, 0, 0,
                                                      0);
        else
          acc += __builtin_bit_cast(i32x4, buf[d][s]);
      }
      __builtin_amdgcn_sched_barrier(0);
      load(d, bb + D * NW);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int d = 0; d < D; ++d)
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" : "+v"(buf[d][s]));
  const int32_t v = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
  if (v == 0x12345678) out[blockIdx.x] = v;
}

template <int MAP, int D, int NW, int MF>
__global__ __launch_bounds__(64 * NW, 1) void k_probe(const int8_t* __restrict__ x, int64_t n,
                                                      int rows_per_blk, uint32_t* out) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t j0 = (int64_t)blockIdx.x * rows_per_blk;
  int64_t j1 = j0 + rows_per_blk;
  j1 = j1 < n ? j1 : n;
  const int nb = j0 < j1 ? (int)((j1 - j0) / 16) : 0;  // 16-row blocks of the slab
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(x + j0 * E), 0, j0 < j1 ? (int)((j1 - j0) * E) : 0, 0x00020000);
  uint32_t off[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) off[s] = lane_off<MAP>(lane, s);
  u32x4 buf[D][KS];
  i32x4 acc = {0, 0, 0, 0};
  const u32x4 qf = {0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u};
  // wave w takes blocks w, w + NW, ...
  auto load = [&](int slot, int b) __attribute__((always_inline)) {
    const uint32_t base = (uint32_t)b * 16u * E;
#pragma unroll
    for (int s = 0; s < KS; ++s)
      buf[slot][s] = __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, base + off[s], 0, 2));
  };
  int b = w;
#pragma unroll
  for (int d = 0; d < D; ++d) load(d, b + d * NW);
  for (; b < nb; b += D * NW) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int bb = b + d * NW;
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if (MF)
          acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, buf[d][s]),
                                                      __builtin_bit_cast(i32x4, qf), acc, 0, 0,
                                                      0);
        else
          acc += __builtin_bit_cast(i32x4, buf[d][s]);
      }
      __builtin_amdgcn_sched_barrier(0);
      load(d, bb + D * NW);  // past the slab end: bounded resource reads 0
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  const int32_t v = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
  if (v == 0x12345678) out[blockIdx.x] = v;  // keeps the loads live
}

template <int MAP, int D, int NW, int MF, bool ASM = false>
int run(const int8_t* x, int64_t n, uint32_t* out, const char* name) {
  const int G = 256;
  int rpb = (int)((n + G - 1) / G);
  rpb = (rpb + 63) / 64 * 64;
  hipEvent_t a, c;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&c));
  auto launch = [&]() {
    if (ASM)
      k_probe_asm<MAP, D, NW, MF><<<G, 64 * NW>>>(x, n, rpb, out);
    else
      k_probe<MAP, D, NW, MF><<<G, 64 * NW>>>(x, n, rpb, out);
  };
  for (int i = 0; i < 5; ++i) launch();
  CK(hipDeviceSynchronize());
  const int R = 50;
  CK(hipEventRecord(a));
  for (int i = 0; i < R; ++i) launch();
  CK(hipEventRecord(c));
  CK(hipEventSynchronize(c));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, c));
  const double us = ms * 1e3 / R, bytes = (double)n * E;
  printf("%-28s %7.1f us  %5.2f TB/s  frac %.3f\n", name, us, bytes / us * 1e-6,
         bytes / us * 1e-6 / 8.0);
  return 0;
}

__global__ void k_fill(uint32_t* x, int64_t nw) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nw; i += (int64_t)gridDim.x * 256) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    x[i] = (uint32_t)(z ^ (z >> 31));
  }
}

int main() {
  const int64_t n = 1000000;
  int8_t* x;
  uint32_t* out;
  CK(hipMalloc(&x, n * E + 4096));
  CK(hipMalloc(&out, 4096));
  CK(hipMemset(x, 3, n * E));
  int rc = 0;
  rc |= run<0, 4, 8, 0>(x, n, out, "coalesced D4 W8 (memset 3)");
  rc |= run<0, 4, 8, 0, true>(x, n, out, "asm coalesced D4 W8 (memset 3)");
  k_fill<<<4096, 256>>>((uint32_t*)x, n * E / 4);  // random bytes from here on
  CK(hipDeviceSynchronize());
  rc |= run<0, 4, 8, 0>(x, n, out, "coalesced D4 W8");
  rc |= run<1, 4, 8, 0>(x, n, out, "row96 D4 W8");
  rc |= run<2, 4, 8, 0>(x, n, out, "rowmfma D4 W8");
  rc |= run<1, 2, 8, 0>(x, n, out, "row96 D2 W8");
  rc |= run<1, 3, 8, 0>(x, n, out, "row96 D3 W8");
  rc |= run<1, 6, 8, 0>(x, n, out, "row96 D6 W8");
  rc |= run<1, 8, 4, 0>(x, n, out, "row96 D8 W4");
  rc |= run<0, 8, 4, 0>(x, n, out, "coalesced D8 W4");
  rc |= run<1, 4, 16, 0>(x, n, out, "row96 D4 W16");
  rc |= run<1, 4, 8, 1>(x, n, out, "row96 D4 W8 mfma");
  rc |= run<1, 3, 8, 1>(x, n, out, "row96 D3 W8 mfma");
  rc |= run<1, 6, 8, 1>(x, n, out, "row96 D6 W8 mfma");
  rc |= run<0, 4, 8, 0, true>(x, n, out, "asm coalesced D4 W8");
  rc |= run<1, 4, 8, 0, true>(x, n, out, "asm row96 D4 W8");
  rc |= run<2, 4, 8, 0, true>(x, n, out, "asm rowmfma D4 W8");
  rc |= run<1, 3, 8, 0, true>(x, n, out, "asm row96 D3 W8");
  rc |= run<1, 2, 8, 0, true>(x, n, out, "asm row96 D2 W8");
  rc |= run<1, 6, 8, 0, true>(x, n, out, "asm row96 D6 W8");
  rc |= run<1, 8, 4, 0, true>(x, n, out, "asm row96 D8 W4");
  rc |= run<1, 4, 16, 0, true>(x, n, out, "asm row96 D4 W16");
  rc |= run<1, 4, 8, 1, true>(x, n, out, "asm row96 D4 W8 mfma");
  rc |= run<1, 3, 8, 1, true>(x, n, out, "asm row96 D3 W8 mfma");
  rc |= run<0, 4, 8, 0>(x, n, out, "coalesced D4 W8 (again)");
  CK(hipFree(x));
  CK(hipFree(out));
  return rc;
}
