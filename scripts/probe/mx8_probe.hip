// One v_mfma_scale_f32_16x16x128_f8f6f4 on raw per-lane operands (hardware layout probe).
#include <hip/hip_runtime.h>
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
__global__ void probe(const int* a, const int* b, const int* sa, const int* sb, float* d) {
  const int l = threadIdx.x;
  i32x8 av, bv;
  for (int i = 0; i < 8; ++i) { av[i] = a[l * 8 + i]; bv[i] = b[l * 8 + i]; }
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, sa[l], 0, sb[l]);
  for (int i = 0; i < 4; ++i) d[l * 4 + i] = c[i];
}
extern "C" int run_probe(const int* a, const int* b, const int* sa, const int* sb, float* d) {
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, a, b, sa, sb, d);
  return (int)hipDeviceSynchronize();
}
