// Shared device-side helpers for the gfx950 (MI355X / CDNA4) ViT kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace evt {

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(4))) short i16x4;
typedef __attribute__((ext_vector_type(8))) short i16x8;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;

#define EVT_LDS __attribute__((address_space(3)))

// ---- conversions -------------------------------------------------------------------
__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
// plain cast: hipcc -O3 emits v_cvt_pk_bf16_f32 (round-to-nearest-even, NaN preserved)
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

// Load 4 consecutive elements as fp32 (16 B for f32, 8 B for bf16).
__device__ __forceinline__ f32x4 load4(const float* p) { return *(const f32x4*)p; }
__device__ __forceinline__ f32x4 load4(const bf16* p) {
  bf16x4 v = *(const bf16x4*)p;
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
// ---- wide (> 64-bit) vector-memory stores -------------------------------------------------
// A store of more than 64 bits reads its data VGPRs after issue: a VALU write to them fewer than
// 2 wait states later (gfx940 family, gfx950 included) can land first. hipcc 7.2 inserts those
// wait states for global / flat stores but not for buffer stores with an SGPR soffset, and in the
// persistent GEMM epilogue a v_and_b32 v3 right after buffer_store_dwordx4 v[2:5] stored zeros into
// dword 1 of 8 lanes in about 1 launch in 12. EVERY store of more than 64 bits in this library goes
// through the helpers below, each followed by wide_store_fence(): a scheduling barrier and s_nop 1
// (2 wait states) between the store and whatever the scheduler would put next.
// tests/test_isa_hazards.py checks the built code objects (every wide vector-memory store is
// fenced, no VALU write of its data VGPRs inside 2 wait states) and that no kernel source issues
// such a store except through these helpers.
__device__ __forceinline__ void wide_store_fence() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 1");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void store_b128(void* p, u32x4 v) {
  *(u32x4*)p = v;
  wide_store_fence();
}
// non-temporal (streaming past L2)
__device__ __forceinline__ void store_b128_nt(void* p, u32x4 v) {
  __builtin_nontemporal_store(v, (u32x4*)p);
  wide_store_fence();
}
// AUX: the cache-policy bits (2 = nt)
template <int AUX>
__device__ __forceinline__ void buffer_store_b128(u32x4 v, __amdgpu_buffer_rsrc_t rs, int voff,
                                                  int soff) {
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff, soff, AUX);
  wide_store_fence();
}
// 64-bit buffer store: outside the hazard class above (data of at most 64 bits), no fence; a
// helper so that the source check of tests/test_isa_hazards.py still sees every raw buffer store
template <int AUX>
__device__ __forceinline__ void buffer_store_b64(u32x2 v, __amdgpu_buffer_rsrc_t rs, int voff,
                                                 int soff) {
  __builtin_amdgcn_raw_buffer_store_b64(v, rs, voff, soff, AUX);
}
__device__ __forceinline__ void store_f32x4(float* p, f32x4 v) {
  store_b128(p, __builtin_bit_cast(u32x4, v));
}
__device__ __forceinline__ void store_bf16x8(bf16* p, bf16x8 v) {
  store_b128(p, __builtin_bit_cast(u32x4, v));
}

__device__ __forceinline__ void store4(float* p, f32x4 v) { store_f32x4(p, v); }
__device__ __forceinline__ void store4(bf16* p, f32x4 v) {
  bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  *(bf16x4*)p = o;
}

// v_permlane16_swap_b32 on two dwords: odd 16-lane rows of x <-> even rows of y (lanes 16-31 of x
// with lanes 0-15 of y, 48-63 of x with 32-47 of y). Scalars only: applied to vector elements in a
// loop, hipcc 7.2 miscompiles the builtin (it reuses element 0 for every j).
__device__ __forceinline__ void permlane16_swap(unsigned& x, unsigned& y) {
  const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  x = (unsigned)r[0];
  y = (unsigned)r[1];
}

// Non-temporal (streaming) stores for GEMM outputs: they go to HBM without displacing the operand
// panels the other CUs of the XCD still read from L2 (measured: -15% on the K = 768 GEMMs).
__device__ __forceinline__ void store4_nt(float* p, f32x4 v) {
  store_b128_nt(p, __builtin_bit_cast(u32x4, v));
}
__device__ __forceinline__ void store4_nt(bf16* p, f32x4 v) {
  const bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  __builtin_nontemporal_store(o, (bf16x4*)p);
}

// tanh-approximate GELU in fp32 (reference modeling/layers/activation.py:13-15), evaluated as
// x * 0.5 * (1 + tanh(u)) == x * sigmoid(2u) = x / (1 + 2^(-2u*log2 e)): one v_exp_f32 and one
// v_rcp_f32. Tails saturate cleanly (2^+inf -> inf -> x * 0; 2^-inf -> 0 -> x).
__device__ __forceinline__ float gelu_tanh(float x) {
  const float c1 = -2.0f * 0.7978845608028654f * 1.4426950408889634f;  // -2*sqrt(2/pi)*log2(e)
  const float c3 = c1 * 0.044715f;
  const float e = __builtin_amdgcn_exp2f(x * (c1 + c3 * x * x));
  return x * __builtin_amdgcn_rcpf(1.0f + e);
}

// Packed-pair forms of the two GELUs (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 for everything but
// the transcendentals, which have no packed form): the GEMM epilogues are VALU-bound on these.
__device__ __forceinline__ f32x2 gelu_tanh2(f32x2 x) {
  const float c1 = -2.0f * 0.7978845608028654f * 1.4426950408889634f;
  const float c3 = c1 * 0.044715f;
  const f32x2 u = x * (f32x2{c1, c1} + f32x2{c3, c3} * (x * x));
  const f32x2 d = f32x2{1.f, 1.f} + f32x2{__builtin_amdgcn_exp2f(u[0]), __builtin_amdgcn_exp2f(u[1])};
  return x * f32x2{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
}
// Exact-form GELU (torch nn.GELU(), the Swin MLP) for the fp32 parity path: x * Phi(x) with erf from
// Abramowitz & Stegun 7.1.26 (|error| <= 2.1e-7, branch-free; libm erff is a ranged polynomial with
// divergent branches: measured 3x slower FC1 epilogues), rescaled so that z' = |x| sqrt(log2 e / 2): exp(-x^2/2) = 2^(-z'^2),
// t = 1 / (1 + p' z') with p' = 0.3275911 / sqrt(log2 e), polynomial coefficients pre-halved (the
// 0.5 of 0.5 erfc), Phi = 0.5 + copysign(0.5 - q, x).
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) {
  const float cz = 0.7071067811865476f * 1.2011224087864498f;  // sqrt(1/2) * sqrt(log2 e)
  const float pp = 0.3275911f / 1.2011224087864498f;
  const f32x2 z = f32x2{fabsf(x[0]), fabsf(x[1])} * f32x2{cz, cz};
  const f32x2 d = f32x2{1.f, 1.f} + f32x2{pp, pp} * z;
  const f32x2 t = f32x2{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  const f32x2 a5 = {0.5f * 1.061405429f, 0.5f * 1.061405429f}, a4 = {0.5f * -1.453152027f, 0.5f * -1.453152027f};
  const f32x2 a3 = {0.5f * 1.421413741f, 0.5f * 1.421413741f}, a2 = {0.5f * -0.284496736f, 0.5f * -0.284496736f};
  const f32x2 a1 = {0.5f * 0.254829592f, 0.5f * 0.254829592f};
  const f32x2 p = t * (a1 + t * (a2 + t * (a3 + t * (a4 + t * a5))));
  const f32x2 zz = z * z;
  const f32x2 q = p * f32x2{__builtin_amdgcn_exp2f(-zz[0]), __builtin_amdgcn_exp2f(-zz[1])};
  const f32x2 h = f32x2{0.5f, 0.5f} - q;
  const f32x2 phi = f32x2{0.5f, 0.5f} + f32x2{copysignf(h[0], x[0]), copysignf(h[1], x[1])};
  return x * phi;
}
// Exact-form GELU for the bf16 paths: x * sigmoid(g(x)) with g(x) = x (b1 + b3 x^2 + b5 x^4) on x
// clamped to [-8, 8] (a minimax fit of logit(Phi); |error| <= 8.0e-5 against 0.5 x (1 + erf(x/sqrt 2))
// over all x, checked on the host in fp32 emulation), far below the bf16 rounding of the result
// (>= 2^-9 relative). 6 packed ops + 4 transcendentals per pair versus 10 + 4 (+4 bit ops) for the
// A&S form: the erf-GELU epilogues are VALU-bound. The fp32 (parity) path keeps gelu_erf2.
__device__ __forceinline__ f32x2 gelu_erf_fast2(f32x2 x) {
  const float L = 1.4426950408889634f;  // coefficients carry -log2(e): u = -g(x) log2(e)
  const f32x2 k1 = {-1.5956037891885726f * L, -1.5956037891885726f * L};
  const f32x2 k3 = {-0.07321892474744947f * L, -0.07321892474744947f * L};
  const f32x2 k5 = {0.0005657298523499585f * L, 0.0005657298523499585f * L};
  const f32x2 xc = {__builtin_amdgcn_fmed3f(x[0], -8.f, 8.f), __builtin_amdgcn_fmed3f(x[1], -8.f, 8.f)};
  const f32x2 x2 = xc * xc;
  const f32x2 u = xc * (k1 + x2 * (k3 + x2 * k5));
  const f32x2 d = f32x2{1.f, 1.f} + f32x2{__builtin_amdgcn_exp2f(u[0]), __builtin_amdgcn_exp2f(u[1])};
  return x * f32x2{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
}
// mode: 0 tanh form (reference activation.py), 1 erf form (A&S, parity path), 2 erf form (fast)
__device__ __forceinline__ f32x4 gelu4(f32x4 v, int mode) {
  f32x2 lo = {v[0], v[1]}, hi = {v[2], v[3]};
  if (mode == 0) {
    lo = gelu_tanh2(lo);
    hi = gelu_tanh2(hi);
  } else if (mode == 1) {
    lo = gelu_erf2(lo);
    hi = gelu_erf2(hi);
  } else {
    lo = gelu_erf_fast2(lo);
    hi = gelu_erf_fast2(hi);
  }
  return f32x4{lo[0], lo[1], hi[0], hi[1]};
}

// Wave64 reductions (butterfly over all 64 lanes).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Async global -> LDS copy of 16 B per lane; LDS destination = wave-uniform base + lane*16.
__device__ __forceinline__ void glds16(const void* gsrc, EVT_LDS void* lds_base) {
  __builtin_amdgcn_global_load_lds(gsrc, lds_base, 16, 0, 0);
}

// glds16 through the SGPR-base form (global_load_lds_dwordx4 v_off, s[base]): a wave-uniform
// 64-bit base plus a per-lane 32-bit offset, so a K-loop advances the base in SALU and keeps
// loop-invariant 32-bit lane offsets instead of one 64-bit VALU address add per piece (hipcc only
// emits the 64-bit vaddr form for the builtin). The wait state between the M0 write and the LDS
// DMA (as hipcc emits it) is the s_nop. hipcc does not count these loads: every consumer retires
// them with explicit s_waitcnt vmcnt (big8_* counted waits).
__device__ __forceinline__ void glds16s(const void* sbase, uint32_t voff, EVT_LDS void* lds_base) {
  const uint32_t m = (uint32_t)(uintptr_t)lds_base;
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(voff), "s"(sbase), "s"(m) : "memory", "m0");
}

// Two glds16s pieces whose LDS destinations are 1 KiB apart under one M0 write: the second uses
// instruction offset 1024, which global_load_lds applies to the LDS and the global address alike
// (its lane offset voff1 is the global offset minus 1024). Issue order: voff0's piece first.
__device__ __forceinline__ void glds16s_pair(const void* sbase, uint32_t voff0, uint32_t voff1,
                                             EVT_LDS void* lds_base) {
  const uint32_t m = (uint32_t)(uintptr_t)lds_base;
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %2\n\t"
               "global_load_lds_dwordx4 %1, %2 offset:1024"
               :: "v"(voff0), "v"(voff1), "s"(sbase), "s"(m) : "memory", "m0");
}

__device__ __forceinline__ void wait_vmcnt0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

}  // namespace evt
