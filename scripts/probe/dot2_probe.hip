// Probe: semantics of v_dot2c_f32_bf16 (__builtin_amdgcn_fdot2_f32_bf16) on gfx950.
#include <hip/hip_runtime.h>
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
__global__ void dot2_kernel(const unsigned* a, const unsigned* b, const float* c, float* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, a[i]), __builtin_bit_cast(bf16x2, b[i]), c[i], false);
}
extern "C" int dot2_probe(const unsigned* a, const unsigned* b, const float* c, float* out, int n) {
  hipLaunchKernelGGL(dot2_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, a, b, c, out, n);
  return hipDeviceSynchronize();
}
