// Memory-bound kernels of the ViT forward on gfx950: patchify (+CLS row) and a standalone LayerNorm.
//
// In the model forward the encoder LayerNorms are folded into the GEMMs (gemm.hip header); the
// standalone LayerNorm below is the op-level evt_layernorm (Keras LayerNormalization(epsilon),
// reference `modeling/layers/norm.py:6`): population variance over the last axis, fp32
// statistics, one wave64 per row, 16-B loads, the row held in registers (D <= 1024), two-pass
// mean / variance with butterfly wave reductions, output in the activation dtype.
//
// patchify replaces the einops Rearrange 'b c (h p1) (w p2) -> b (h w) (p1 p2 c)' of reference
// `modeling/models/vit.py:31-32,45`: one workgroup per (image, patch-row) stages the
// [C][ps][W] strip of the NCHW image in LDS with coalesced 16-B loads, then writes the 14 patch
// vectors of that row coalesced in (p1 p2 c) order. The first strip of each image also writes the
// CLS token row x[b, 0] = cls + pos[0] (reference vit.py:48-51) into the token stream, with the
// row statistics the folded LayerNorm of layer 0 needs.
#include <type_traits>

#include "common.h"
#include "evt_internal.h"

namespace evt {

namespace {

template <typename TO, int NV>  // NV = float4 groups per lane (D <= 256*NV)
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, int64_t ldx,
                                                        TO* __restrict__ y, int64_t ldy,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, int rows,
                                                        int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + (int64_t)row * ldx;
  f32x4 v[NV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    v[i] = c < D ? load4(xr + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  }
  const float inv_d = 1.0f / (float)D;
  const float mean = wave_sum(s) * inv_d;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < D) {
      const f32x4 d = v[i] - mean;
      q += d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3];
    }
  }
  const float rstd = rsqrtf(wave_sum(q) * inv_d + eps);
  TO* yr = y + (int64_t)row * ldy;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < D) store4(yr + c, (v[i] - mean) * rstd * load4(gamma + c) + load4(beta + c));
  }
}

// grid (HW/ps, B); block 256. LDS strip [C][ps][HW] fp32.
template <typename TO>
__global__ __launch_bounds__(256) void patchify_kernel(const float* __restrict__ img, int C, int HW,
                                                       int ps, TO* __restrict__ out,
                                                       TO* __restrict__ x,
                                                       const float* __restrict__ cls,
                                                       const float* __restrict__ pos, int D,
                                                       float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* strip = (float*)smem;
  const int hh = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int np = HW / ps;
  // stage rows hh*ps .. hh*ps+ps-1 of every channel (contiguous ps*HW floats per channel)
  const int per_c = ps * HW;  // multiple of 4 (HW % 4 == 0 checked on host)
  for (int c = 0; c < C; ++c) {
    const float* src = img + (((int64_t)b * C + c) * HW + (int64_t)hh * ps) * HW;
    for (int i = tid * 4; i < per_c; i += 256 * 4) *(f32x4*)(strip + c * per_c + i) = load4(src + i);  // LDS
  }
  __syncthreads();
  const int pd = ps * ps * C;  // patch vector length
  TO* orow = out + ((int64_t)b * np * np + (int64_t)hh * np) * pd;
  if (pd % 8 == 0) {
    // 8 consecutive (p1 p2 c) elements per thread -> one 16-B (bf16) / 2 x 16-B (f32) store; the
    // strip offsets of a chunk depend only on its position in the patch vector (no per-element
    // division by the patch index)
    const int cpp = pd / 8;  // chunks per patch
    for (int e = tid; e < np * cpp; e += 256) {
      const int ww = e / cpp, f0 = (e - ww * cpp) * 8;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int f = f0 + j, c = f % C, p12 = f / C, p1 = p12 / ps, p2 = p12 - p1 * ps;
        v[j] = strip[c * per_c + p1 * HW + ww * ps + p2];
      }
      TO* op = orow + (int64_t)ww * pd + f0;
      store4(op, f32x4{v[0], v[1], v[2], v[3]});
      store4(op + 4, f32x4{v[4], v[5], v[6], v[7]});
    }
  } else {
    for (int e = tid; e < np * pd; e += 256) {
      const int ww = e / pd, f = e - ww * pd;
      const int c = f % C, p12 = f / C, p1 = p12 / ps, p2 = p12 - p1 * ps;
      orow[(int64_t)ww * pd + f] = from_f32<TO>(strip[c * per_c + p1 * HW + ww * ps + p2]);
    }
  }
  if (hh == 0 && tid < 64) {  // one wave writes the CLS row and its LayerNorm statistics
    const int64_t row = (int64_t)b * (np * np + 1);
    TO* xr = x + row * D;
    float s1 = 0.f, s2 = 0.f;
    for (int n = tid; n < D; n += 64) {
      const TO v = from_f32<TO>(cls[n] + pos[n]);
      xr[n] = v;
      const float q = to_f32(v);
      s1 += q;
      s2 += q * q;
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (stats && tid < stats_slots(D)) {
      float* st = stats + 2 * (stats_slots(D) * row + tid);
      st[0] = tid == 0 ? s1 : 0.f;
      st[1] = tid == 0 ? s2 : 0.f;
    }
  }
}

// Channel-major patch vectors (the model's layout): out[patch][c ps ps + p1 ps + p2], i.e. the
// reference vector (p1 p2 c) with its K axis permuted; the patch-embedding weight is packed with
// the same row permutation (patch_weight_cm), so the product is the reference Dense. Each patch
// vector is then C * ps runs of ps contiguous image pixels: every thread reads 8 consecutive
// pixels of one run from the LDS strip (two 16-B reads) and writes one 16-B (bf16) chunk, and a
// wave's stores cover 1 KB of consecutive output. grid (HW/ps, B); requires ps % 8 == 0.
template <typename TO>
__global__ __launch_bounds__(256) void patchify_cm_kernel(const float* __restrict__ img, int C,
                                                          int HW, int ps, TO* __restrict__ out,
                                                          TO* __restrict__ x,
                                                          const float* __restrict__ cls,
                                                          const float* __restrict__ pos, int D,
                                                          float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* strip = (float*)smem;
  const int hh = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int np = HW / ps;
  const int per_c = ps * HW;
  if (per_c % 256 == 0) {  // every strip load straight to LDS (global_load_lds), one wait
    const int wave = tid >> 6, lane = tid & 63;
    for (int c = 0; c < C; ++c) {
      const float* src = img + (((int64_t)b * C + c) * HW + (int64_t)hh * ps) * HW;
      for (int i0 = wave * 256; i0 < per_c; i0 += 1024)
        glds16(src + i0 + lane * 4, (EVT_LDS char*)smem + (c * per_c + i0) * 4);
    }
    wait_vmcnt0();
  } else {
    for (int c = 0; c < C; ++c) {
      const float* src = img + (((int64_t)b * C + c) * HW + (int64_t)hh * ps) * HW;
      for (int i = tid * 4; i < per_c; i += 256 * 4) *(f32x4*)(strip + c * per_c + i) = load4(src + i);  // LDS
    }
  }
  __syncthreads();
  const int pd = ps * ps * C;
  const int cpr = ps / 8;        // 8-pixel chunks per run
  const int cpp = pd / 8;        // chunks per patch vector
  TO* orow = out + ((int64_t)b * np * np + (int64_t)hh * np) * pd;
  for (int e = tid; e < np * cpp; e += 256) {
    const int ww = e / cpp, q = e - ww * cpp;
    const int run = q / cpr, c = run / ps, p1 = run - c * ps, p2 = (q - run * cpr) * 8;
    const float* sp = strip + c * per_c + p1 * HW + ww * ps + p2;
    const f32x4 v0 = *(const f32x4*)sp, v1 = *(const f32x4*)(sp + 4);
    TO* op = orow + (int64_t)ww * pd + q * 8;
    if constexpr (std::is_same<TO, bf16>::value) {  // one 16-B store per 8 pixels
      const bf16x8 o = {(bf16)v0[0], (bf16)v0[1], (bf16)v0[2], (bf16)v0[3],
                        (bf16)v1[0], (bf16)v1[1], (bf16)v1[2], (bf16)v1[3]};
      store_bf16x8(op, o);
    } else {
      store4(op, v0);
      store4(op + 4, v1);
    }
  }
  if (hh == 0 && tid < 64) {  // one wave writes the CLS row and its LayerNorm statistics
    const int64_t row = (int64_t)b * (np * np + 1);
    TO* xr = x + row * D;
    float s1 = 0.f, s2 = 0.f;
    for (int n = tid; n < D; n += 64) {
      const TO v = from_f32<TO>(cls[n] + pos[n]);
      xr[n] = v;
      const float q = to_f32(v);
      s1 += q;
      s2 += q * q;
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (stats && tid < stats_slots(D)) {
      float* st = stats + 2 * (stats_slots(D) * row + tid);
      st[0] = tid == 0 ? s1 : 0.f;
      st[1] = tid == 0 ? s2 : 0.f;
    }
  }
}

// Keras patch_to_embedding kernel [(p1 p2 c), N] -> rows in the channel-major order above.
__global__ void patch_weight_cm_kernel(const float* __restrict__ W, float* __restrict__ Wcm, int C,
                                       int ps, int N) {
  const int kcm = blockIdx.x;  // c ps ps + p1 ps + p2
  const int c = kcm / (ps * ps), p12 = kcm - c * ps * ps;
  const int k = p12 * C + c;   // (p1 ps + p2) C + c
  for (int n = threadIdx.x; n < N; n += blockDim.x) Wcm[(int64_t)kcm * N + n] = W[(int64_t)k * N + n];
}

template <typename TO, int NV>
hipError_t ln_nv(const float* x, int64_t ldx, void* y, int64_t ldy, const float* g,
                 const float* bb, int rows, int D, float eps, hipStream_t s) {
  hipLaunchKernelGGL((layernorm_kernel<TO, NV>), dim3((rows + 3) / 4), dim3(256), 0, s, x, ldx,
                     (TO*)y, ldy, g, bb, rows, D, eps);
  return hipGetLastError();
}

template <typename TO>
hipError_t ln_t(const float* x, int64_t ldx, void* y, int64_t ldy, const float* g, const float* bb,
                int rows, int D, float eps, hipStream_t s) {
  if (D <= 256) return ln_nv<TO, 1>(x, ldx, y, ldy, g, bb, rows, D, eps, s);
  if (D <= 512) return ln_nv<TO, 2>(x, ldx, y, ldy, g, bb, rows, D, eps, s);
  if (D <= 768) return ln_nv<TO, 3>(x, ldx, y, ldy, g, bb, rows, D, eps, s);
  return ln_nv<TO, 4>(x, ldx, y, ldy, g, bb, rows, D, eps, s);
}

}  // namespace

hipError_t layernorm_launch(int dtype, const float* x, int64_t ldx, void* y, int64_t ldy,
                            const float* gamma, const float* beta, int rows, int D, float eps,
                            hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  if (D <= 0 || D > 1024 || (D & 3) || (ldx & 3) || (ldy & 3)) return hipErrorInvalidValue;
  return dtype == DT_BF16 ? ln_t<bf16>(x, ldx, y, ldy, gamma, beta, rows, D, eps, s)
                          : ln_t<float>(x, ldx, y, ldy, gamma, beta, rows, D, eps, s);
}

hipError_t patch_weight_cm(const float* W, float* Wcm, int C, int ps, int N, hipStream_t s) {
  hipLaunchKernelGGL(patch_weight_cm_kernel, dim3(C * ps * ps), dim3(256), 0, s, W, Wcm, C, ps, N);
  return hipGetLastError();
}

hipError_t patchify_launch(int dtype, const float* img, int B, int C, int HW, int ps, void* out,
                           void* x, const float* cls, const float* pos, int D, float* stats,
                           hipStream_t s, bool channel_major) {
  if (B <= 0) return hipSuccess;
  if (HW % ps || (ps * HW) % 4) return hipErrorInvalidValue;
  const size_t lds = (size_t)C * ps * HW * sizeof(float);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  dim3 grid(HW / ps, B);
  if (channel_major) {
    if (ps % 8) return hipErrorInvalidValue;
    if (dtype == DT_BF16) {
      hipFuncSetAttribute((const void*)patchify_cm_kernel<bf16>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(patchify_cm_kernel<bf16>, grid, dim3(256), lds, s, img, C, HW, ps,
                         (bf16*)out, (bf16*)x, cls, pos, D, stats);
    } else {
      hipFuncSetAttribute((const void*)patchify_cm_kernel<float>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(patchify_cm_kernel<float>, grid, dim3(256), lds, s, img, C, HW, ps,
                         (float*)out, (float*)x, cls, pos, D, stats);
    }
    return hipGetLastError();
  }
  if (dtype == DT_BF16) {
    hipFuncSetAttribute((const void*)patchify_kernel<bf16>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(patchify_kernel<bf16>, grid, dim3(256), lds, s, img, C, HW, ps, (bf16*)out,
                       (bf16*)x, cls, pos, D, stats);
  } else {
    hipFuncSetAttribute((const void*)patchify_kernel<float>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(patchify_kernel<float>, grid, dim3(256), lds, s, img, C, HW, ps,
                       (float*)out, (float*)x, cls, pos, D, stats);
  }
  return hipGetLastError();
}

}  // namespace evt
