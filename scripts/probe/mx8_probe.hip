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

// Throughput of back-to-back independent MX / bf16 MFMAs (8 accumulators per wave).
__global__ __launch_bounds__(256) void mfma_rate_mx(int iters, float* out) {
  i32x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = 0x38383838 + threadIdx.x; b[i] = 0x30303030 + i; }
  f32x4 c[8];
  for (int k = 0; k < 8; ++k) c[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int k = 0; k < 8; ++k)
      c[k] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c[k], 0, 0, 0, 127, 0, 127);
  float s = 0.f;
  for (int k = 0; k < 8; ++k) s += c[k][0] + c[k][1] + c[k][2] + c[k][3];
  if (s == 1.2345f) out[threadIdx.x] = s;
}
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
__global__ __launch_bounds__(256) void mfma_rate_bf16(int iters, float* out) {
  bf16x8_t a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(0.001f * threadIdx.x); b[i] = (__bf16)(0.002f * i); }
  f32x4 c[8];
  for (int k = 0; k < 8; ++k) c[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int k = 0; k < 8; ++k)
      c[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c[k], 0, 0, 0);
  float s = 0.f;
  for (int k = 0; k < 8; ++k) s += c[k][0] + c[k][1] + c[k][2] + c[k][3];
  if (s == 1.2345f) out[threadIdx.x] = s;
}
extern "C" float run_rate(int which, int blocks, int iters, float* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0, 0);
    if (which == 0) hipLaunchKernelGGL(mfma_rate_mx, dim3(blocks), dim3(256), 0, 0, iters, out);
    else hipLaunchKernelGGL(mfma_rate_bf16, dim3(blocks), dim3(256), 0, 0, iters, out);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
  }
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}
