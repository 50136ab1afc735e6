// Round-6 probe: a 256 x 256 x 64 bf16 GEMM main loop with ONE wave per SIMD (4 waves, 512
// registers per lane: 64 accumulator tiles in AGPRs), software-pipelined inside each wave
// (the next k-step's fragment reads and the next K-tile's LDS-DMA issued between this k-step's
// MFMAs) and one barrier per K-tile, against the product's 8-wave ping-pong loop (two waves per
// SIMD, 4-8 barriers per K-tile). C[M][N] = A[M][K] . W[N][K]^T, bf16 in / bf16 out, M, N
// multiples of 256, K of 64. Not part of the product library.
//
//   hipcc -O3 --offload-arch=gfx950 -shared -fPIC scripts/probe/gemm4w.hip -o scripts/probe/libgemm4w.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#define LDS __attribute__((address_space(3)))

namespace {
constexpr int ROWB = 128, TILE = 256 * ROWB, STAGE = 2 * TILE;

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, local = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
}

// two 1-KiB LDS-DMA pieces 1 KiB apart in LDS under one M0 (instruction offset on both addresses)
__device__ __forceinline__ void glds_pair(const void* sbase, uint32_t v0, uint32_t v1, uint32_t m) {
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %2\n\t"
               "global_load_lds_dwordx4 %1, %2 offset:1024"
               :: "v"(v0), "v"(v1), "s"(sbase), "s"(m) : "memory", "m0");
}

__device__ __forceinline__ f32x4 mma(const u32x4& w, const u32x4& a, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, w),
                                                 __builtin_bit_cast(bf16x8, a), c, 0, 0, 0);
}

// VAR 0: reads / DMA placed by the compiler; VAR 1: sched_group_barrier interleave (4 MFMA : 1
// ds_read, the DMA pieces spread over the first k-step)
template <int VAR>
__global__ __launch_bounds__(256, 1) void gemm4w_kernel(const __bf16* A, const __bf16* W,
                                                        __bf16* C, int M, int N, int K, int store) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int ntn = N / 256;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / ntn, tn = tile - tm * ntn;
  const int m0 = tm * 256, n0 = tn * 256;
  const int nk = K / 64;
  const int srow = lane >> 3, sslot = lane & 7;
  const uint32_t swz = (uint32_t)((sslot ^ srow) << 4);
  const uint32_t ldb = (uint32_t)K * 2;
  // DMA: wave w stages A rows [64 w, 64 w + 64) and W rows [64 w, 64 w + 64): 4 pairs each
  uint32_t va[4][2], vw[4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r0 = wave * 64 + q * 16 + srow;
    va[q][0] = (uint32_t)r0 * ldb + swz + 1024;
    va[q][1] = (uint32_t)(r0 + 8) * ldb + swz;
    vw[q][0] = va[q][0];
    vw[q][1] = va[q][1];
  }
  const char* abase = (const char*)A + (int64_t)m0 * ldb - 1024;
  const char* wbase = (const char*)W + (int64_t)n0 * ldb - 1024;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(LDS char*)smem;
  auto dma = [&](int kt, int q) {  // pair q of A then of W for K-tile kt
    const uint32_t st = lds0 + (kt & 1) * STAGE;
    const uint32_t row = wave * 64 + q * 16;
    glds_pair(abase + kt * ROWB, va[q][0], va[q][1], st + row * ROWB);
    glds_pair(wbase + kt * ROWB, vw[q][0], vw[q][1], st + TILE + row * ROWB);
  };
  const int frow = lane & 15, fsw = lane & 7, fg = lane >> 4;
  auto rd = [&](int buf, int row, int ks) {
    const LDS char* S = (const LDS char*)smem + buf * STAGE;
    return *(const LDS u32x4*)(S + row * ROWB + (((fg + 4 * ks) ^ fsw) << 4));
  };
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // A fragments double-buffered by k-step parity (fa[0] / fa[1]); B fragments rotate in place:
  // fb[j] of the next k-step is read right after the 8 MFMAs that consume the current fb[j]
  u32x4 fa[2][8], fb[8];

  // prologue: K-tile 0 -> buffer 0, visible; reads of (0, ks0)
#pragma unroll
  for (int q = 0; q < 4; ++q) dma(0, q);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) fa[0][i] = rd(0, wm * 128 + 16 * i + frow, 0);
#pragma unroll
  for (int j = 0; j < 8; ++j) fb[j] = rd(0, 256 + wn * 128 + 16 * j + frow, 0);

  for (int t = 0; t < nk; ++t) {
    const int b = t & 1;
    const bool more = t + 1 < nk;
    // ---- k-step 0 of K-tile t: DMA of K-tile t + 1, reads of (t, ks1)
    if (more) {
#pragma unroll
      for (int q = 0; q < 4; ++q) dma(t + 1, q);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[1][i] = rd(b, wm * 128 + 16 * i + frow, 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[j][i] = mma(fb[j], fa[0][i], acc[j][i]);
      fb[j] = rd(b, 256 + wn * 128 + 16 * j + frow, 1);
      if constexpr (VAR == 1) {
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
        if (j == 0) __builtin_amdgcn_sched_group_barrier(0x100, 9, 0);
        else __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    }
    // ---- k-step 1, B fragments 0-3
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[j][i] = mma(fb[j], fa[1][i], acc[j][i]);
    // K-tile t + 1 landed (every wave's pieces) and every read of buffer b retired, then the
    // barrier: buffer b ^ 1 is readable, buffer b may be restaged
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (more) {
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[0][i] = rd(b ^ 1, wm * 128 + 16 * i + frow, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = rd(b ^ 1, 256 + wn * 128 + 16 * j + frow, 0);
    }
#pragma unroll
    for (int j = 4; j < 8; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[j][i] = mma(fb[j], fa[1][i], acc[j][i]);
      if (more) fb[j] = rd(b ^ 1, 256 + wn * 128 + 16 * j + frow, 0);
      if constexpr (VAR == 1) {
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 1);
        if (j == 4) __builtin_amdgcn_sched_group_barrier(0x100, 13, 1);
        else __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
      }
    }
  }
  if (!store) return;
  // acc[j][i][r] = C[m0 + wm 128 + 16 i + (lane & 15)][n0 + wn 128 + 16 j + 4 (lane >> 4) + r]
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wm * 128 + 16 * i + frow, n = n0 + wn * 128 + 16 * j + 4 * fg;
      const bf16x4 o = {(__bf16)acc[j][i][0], (__bf16)acc[j][i][1], (__bf16)acc[j][i][2],
                        (__bf16)acc[j][i][3]};
      *(bf16x4*)(C + (int64_t)m * N + n) = o;
    }
}
}  // namespace

extern "C" int gemm4w_launch(const void* A, const void* W, void* C, int M, int N, int K, int var,
                             int store, void* stream) {
  if (M % 256 || N % 256 || K % 64 || K < 128) return -1;
  const dim3 grid((M / 256) * (N / 256));
  if (var == 1)
    hipLaunchKernelGGL(gemm4w_kernel<1>, grid, dim3(256), 0, (hipStream_t)stream,
                       (const __bf16*)A, (const __bf16*)W, (__bf16*)C, M, N, K, store);
  else
    hipLaunchKernelGGL(gemm4w_kernel<0>, grid, dim3(256), 0, (hipStream_t)stream,
                       (const __bf16*)A, (const __bf16*)W, (__bf16*)C, M, N, K, store);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
