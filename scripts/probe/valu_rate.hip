// VALU issue rate probe (gfx950): cycles per wave-instruction of the ops the GELU / LayerNorm
// epilogues are built from, measured with 1, 2 and 4 waves per SIMD issuing 8 independent chains
// of the op (s_memtime around an unrolled loop; cycles per instruction per SIMD = elapsed cycles x
// waves per SIMD / instructions per wave). Each op's result feeds its own next instance, 8 chains
// deep, so dependency latency is hidden at >= 2 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC scripts/probe/valu_rate.hip -o scripts/probe/valu_rate.so
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CHAIN8(OP)                                                                     \
  asm volatile(OP " %0, %0, %8, %9\n" OP " %1, %1, %8, %9\n" OP " %2, %2, %8, %9\n"     \
               OP " %3, %3, %8, %9\n" OP " %4, %4, %8, %9\n" OP " %5, %5, %8, %9\n"     \
               OP " %6, %6, %8, %9\n" OP " %7, %7, %8, %9\n"                            \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
               : "v"(b), "v"(c))
#define CHAIN8_2(OP)                                                                   \
  asm volatile(OP " %0, %0, %8\n" OP " %1, %1, %8\n" OP " %2, %2, %8\n"                 \
               OP " %3, %3, %8\n" OP " %4, %4, %8\n" OP " %5, %5, %8\n"                 \
               OP " %6, %6, %8\n" OP " %7, %7, %8\n"                                    \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
               : "v"(b))
#define CHAIN8_1(OP)                                                                   \
  asm volatile(OP " %0, %0\n" OP " %1, %1\n" OP " %2, %2\n" OP " %3, %3\n"               \
               OP " %4, %4\n" OP " %5, %5\n" OP " %6, %6\n" OP " %7, %7\n"               \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7))

template <int OPK>
__global__ __launch_bounds__(1024) void valu_kernel(unsigned long long* out, int iters) {
  // 32-bit ops work on one VGPR per chain, 64-bit packed-f32 ops on a pair
  typedef typename std::conditional<(OPK == 1 || OPK == 2 || OPK == 3), double, float>::type T;
  T a0, a1, a2, a3, a4, a5, a6, a7, b, c;
  float seed = (float)threadIdx.x * 1e-3f;
  if constexpr (sizeof(T) == 8) {
    a0 = a1 = a2 = a3 = a4 = a5 = a6 = a7 = (double)seed;
    b = 0.999; c = 1e-3;
  } else {
    a0 = a1 = a2 = a3 = a4 = a5 = a6 = a7 = seed;
    b = 0.999f; c = 1e-3f;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    if constexpr (OPK == 0) CHAIN8("v_fma_f32");
    else if constexpr (OPK == 1) CHAIN8("v_pk_fma_f32");
    else if constexpr (OPK == 2) CHAIN8_2("v_pk_mul_f32");
    else if constexpr (OPK == 3) CHAIN8_2("v_pk_add_f32");
    else if constexpr (OPK == 4) CHAIN8("v_pk_fma_f16");
    else if constexpr (OPK == 5) CHAIN8_1("v_exp_f32");
    else if constexpr (OPK == 6) CHAIN8_1("v_exp_f16");
    else if constexpr (OPK == 7) CHAIN8_1("v_rcp_f32");
    else if constexpr (OPK == 8) CHAIN8_2("v_mul_f32");
    else if constexpr (OPK == 9) CHAIN8("v_med3_f32");
    else if constexpr (OPK == 10) CHAIN8_2("v_pk_mul_f16");
    else if constexpr (OPK == 11) CHAIN8_1("v_rcp_f16");
    else if constexpr (OPK == 12) CHAIN8_2("v_cvt_pk_bf16_f32");
    else if constexpr (OPK == 13) CHAIN8_2("v_add_f32");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
  T s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  if ((float)s == 12345.678f) out[0] = 0;  // keep the chains live
}

extern "C" int valu_run(int opk, int waves_per_simd, int iters, unsigned long long* d_out, float* ms) {
  const int threads = 256 * waves_per_simd;  // 4 SIMDs per CU, one block per CU
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
#define L(K) hipLaunchKernelGGL((valu_kernel<K>), dim3(256), dim3(threads), 0, 0, d_out, iters)
  switch (opk) {
    case 0: L(0); break; case 1: L(1); break; case 2: L(2); break; case 3: L(3); break;
    case 4: L(4); break; case 5: L(5); break; case 6: L(6); break; case 7: L(7); break;
    case 8: L(8); break; case 9: L(9); break; case 10: L(10); break; case 11: L(11); break;
    case 12: L(12); break; case 13: L(13); break;
    default: return -1;
  }
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  hipEventElapsedTime(ms, e0, e1);
  return (int)hipGetLastError();
}
