// Fused multi-head self-attention for the ViT encoder on gfx950.
//
// Replaces reference `modeling/layers/attention.py:20-34`: the (qkv h d) split, q.k^T * h_k^-0.5,
// tf.nn.softmax, attn.v and the 'b h n d -> b n (h d)' rearrange, without materialising the
// [B, h, N, N] score tensor (954 MB per layer at DeiT-base bs512 in fp32).
//
// One workgroup per (image, head); 4 waves. K and V of the head (N <= 256 rows x 64) are staged
// once into LDS with global_load_lds straight from the QKV GEMM output (token rows, columns
// (qkv h d), so no re-layout kernel exists), rows past N clamped (their scores are masked to -inf
// and their P is exactly 0). Each wave then walks 16-query tiles:
//
//   S^T = K . Q^T      (MFMA A = K rows from LDS, B = Q rows straight from global)
//   exact softmax      (the key axis lives in registers + 4 lane groups: 2 shuffles per reduction)
//   O^T = V^T . P^T    (A = V^T via ds_read_b64_tr_b16 transposed LDS reads; B = P^T is the S^T
//                       accumulator itself, converted to bf16 in place: no LDS round trip)
//
// Computing the transposed products puts one query per lane column, so the row max / row sum and
// the final 1/l scaling are lane-local, and each lane stores 4 consecutive head features.
// LDS images use the swizzle chunk ^ (row & 7) (bf16, 128-B rows) / chunk ^ (row & 15) (fp32,
// 256-B rows), applied on the glds source address and on every read: conflict-free for both the
// row reads and the transposed reads (checked with the bank model of the CDNA4 guide).
//
// The fp32 variant (exact v_mfma_f32_16x16x4_f32, for the 1e-3 parity path) uses the same
// structure; its V^T operand is a plain ds_read_b32 per MFMA.
#include "common.h"
#include "evt_internal.h"

namespace evt {

namespace {

// One 16-query tile of one (image, head): S^T = K Q^T, softmax, O^T = V^T P^T, stores.
// Ks / Vs: the head's K and V rows staged in LDS (NKT*16 rows of 128 B, swizzle chunk ^ (row & 7)).

template <int NKT, bool PLAIN_STORE>
__device__ __forceinline__ void attn_tile_bf16(const AttnParams& p, const EVT_LDS char* Ks,
                                               const EVT_LDS char* Vs, u32x4 qf0, u32x4 qf1,
                                               int qt, int b, int h, int lane) {
  constexpr int ROWB = 128;
  const int g = lane >> 4, c16 = lane & 15, sw = lane & 7;
  f32x4 s[NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    const EVT_LDS char* kr = Ks + (kt * 16 + c16) * ROWB;
    const u32x4 k0 = *(const EVT_LDS u32x4*)(kr + ((g ^ sw) * 16));
    const u32x4 k1 = *(const EVT_LDS u32x4*)(kr + (((g + 4) ^ sw) * 16));
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, k0),
                                                  __builtin_bit_cast(bf16x8, qf0), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, k1),
                                                  __builtin_bit_cast(bf16x8, qf1), acc, 0, 0, 0);
    s[kt] = acc;
  }
  // s[kt][j] = S^T[key = kt*16 + 4g + j][query = qt*16 + c16]. Keys past N exist only in the
  // tiles that reach past N (a wave-uniform test): the rest skip the masking VALU work.
  // (NFULL: tiles that are full for every N this NKT is launched for, attention_launch)
  constexpr int NFULL = NKT == 13 ? 12 : NKT == 12 ? 8 : NKT == 14 ? 13 : NKT == 16 ? 14 : NKT == 8 ? 4 : 0;
#pragma unroll
  for (int kt = NFULL; kt < NKT; ++kt)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (kt * 16 + 4 * g + j >= p.N) s[kt][j] = -INFINITY;
  // max of the raw scores in two v_max3 chains (one new pair per op; -fno-honor-nans: no
  // canonicalising v_max per MFMA result), then exp2(s c - m c) as one packed FMA per pair
  // (scale_log2 > 0, so the max commutes with the scale). Round 3: 521 -> 458 VALU instructions
  // per tile, attention 131.5 -> 129.3 us per layer (DeiT-base bs512, alternating same-box runs)
  float m0 = fmaxf(fmaxf(s[0][0], s[0][1]), s[0][2]), m1 = fmaxf(fmaxf(s[0][3], s[1][0]), s[1][1]);
#pragma unroll
  for (int i = 6; i + 3 < 4 * NKT; i += 4) {
    m0 = fmaxf(fmaxf(m0, s[i >> 2][i & 3]), s[(i + 1) >> 2][(i + 1) & 3]);
    m1 = fmaxf(fmaxf(m1, s[(i + 2) >> 2][(i + 2) & 3]), s[(i + 3) >> 2][(i + 3) & 3]);
  }
  float mx = fmaxf(m0, m1);
  if constexpr ((4 * NKT - 6) % 4 != 0) mx = fmaxf(fmaxf(mx, s[NKT - 1][2]), s[NKT - 1][3]);
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  const f32x2 sc2 = {p.scale_log2, p.scale_log2};
  const f32x2 mo2 = {-mx * p.scale_log2, -mx * p.scale_log2};
  f32x2 sum2 = {0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      f32x2 v = {s[kt][2 * hh], s[kt][2 * hh + 1]};
      v = v * sc2 + mo2;
      v[0] = __builtin_amdgcn_exp2f(v[0]);
      v[1] = __builtin_amdgcn_exp2f(v[1]);
      s[kt][2 * hh] = v[0];
      s[kt][2 * hh + 1] = v[1];
      sum2 += v;
    }
  float sum = sum2[0] + sum2[1];
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);

  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  // transposed-read addressing: lane 16g + 4q + pp reads row 4g+q, cols dt*16 + 4pp .. +3
  const int tq = (lane >> 2) & 3, tp = lane & 3;
#pragma unroll
  for (int ks = 0; ks < NKT / 2; ++ks) {
    bf16x8 pf;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pf[j] = (bf16)s[2 * ks][j];
      pf[4 + j] = (bf16)s[2 * ks + 1][j];
    }
    __builtin_amdgcn_sched_barrier(0);  // keep each step's tr-reads next to their MFMAs
    const int key0 = ks * 32 + 4 * g + tq;  // key0 & 7 == key1 & 7
    const int ksw = key0 & 7;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int chunk = 2 * dt + (tp >> 1);
      const int off = ((chunk ^ ksw) * 16) + (tp & 1) * 8;
      const i16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((EVT_LDS i16x4*)(Vs + key0 * ROWB + off));
      const i16x4 v1 =
          __builtin_amdgcn_ds_read_tr16_b64_v4i16((EVT_LDS i16x4*)(Vs + (key0 + 16) * ROWB + off));
      const i16x8 vv = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vv), pf, o[dt],
                                                      0, 0, 0);
    }
  }
  if constexpr (NKT % 2) {  // last 16 keys: the upper k half of the MFMA is zero
    bf16x8 pf;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pf[j] = (bf16)s[NKT - 1][j];
      pf[4 + j] = (bf16)0.f;
    }
    __builtin_amdgcn_sched_barrier(0);
    const int key0 = (NKT - 1) * 16 + 4 * g + tq;
    const int ksw = key0 & 7;
    const i16x4 z = {0, 0, 0, 0};
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int chunk = 2 * dt + (tp >> 1);
      const int off = ((chunk ^ ksw) * 16) + (tp & 1) * 8;
      const i16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((EVT_LDS i16x4*)(Vs + key0 * ROWB + off));
      const i16x8 vv = __builtin_shufflevector(v0, z, 0, 1, 2, 3, 4, 5, 6, 7);
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vv), pf, o[dt],
                                                      0, 0, 0);
    }
  }
  // o[dt][j] = O^T[d = dt*16 + 4g + j][query]
  const int q = qt * 16 + c16;
  if (p.q8) {  // MX8 output: 32-feature block blk = dt pair (2 blk, 2 blk + 1), 4 lanes per query
    const float inv = 1.0f / sum;
    const int64_t row = (int64_t)b * p.N + q;
#pragma unroll
    for (int blk = 0; blk < 2; ++blk) {
      const f32x4 lo = o[2 * blk] * inv, hi = o[2 * blk + 1] * inv;
      float am = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) am = fmaxf(am, fmaxf(fabsf(lo[j]), fabsf(hi[j])));
      am = fmaxf(am, __shfl_xor(am, 16, 64));
      am = fmaxf(am, __shfl_xor(am, 32, 64));
      const int E = (int)((__float_as_uint(am) >> 23) & 0xff);
      const unsigned sb = (unsigned)max(E - 8, 0);  // OCP MX shared exponent (mx8.hip)
      const float is = __uint_as_float((254u - sb) << 23);
      float c[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c[j] = __builtin_amdgcn_fmed3f(lo[j] * is, -448.f, 448.f);
        c[4 + j] = __builtin_amdgcn_fmed3f(hi[j] * is, -448.f, 448.f);
      }
      int w0 = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
      w0 = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], w0, true);
      int w1 = __builtin_amdgcn_cvt_pk_fp8_f32(c[4], c[5], 0, false);
      w1 = __builtin_amdgcn_cvt_pk_fp8_f32(c[6], c[7], w1, true);
      if (q < p.N) {
        uint8_t* dst = p.q8 + row * p.ldq8 + h * 64 + 32 * blk + 4 * g;
        *(int*)dst = w0;
        *(int*)(dst + 16) = w1;
        if (g == 0) {
          const int bi = 2 * h + blk;
          ((uint8_t*)p.s8)[((int64_t)(bi >> 2) * p.rows8 + row) * 4 + (bi & 3)] = (uint8_t)sb;
        }
      }
    }
    return;
  }
  // bf16 pairs, then one permlane16 swap per dword of each (dt, dt + 1) pair: lane group g ends
  // up with features 32 pr + 16 (g & 1) + 8 (g >> 1) .. + 7 of its query in {x[0..1], y[0..1]},
  // so O leaves as two 16-B stores per lane instead of four 8-B ones (store-issue bound)
  const float inv = 1.0f / sum;
  u32x2 ob[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const f32x4 v = o[dt] * inv;
    const bf16x4 w = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    ob[dt] = __builtin_bit_cast(u32x2, w);
  }
  unsigned x0[2], x1[2], y0[2], y1[2];
#pragma unroll
  for (int pr = 0; pr < 2; ++pr) {
    unsigned a0 = ob[2 * pr][0], a1 = ob[2 * pr][1], c0 = ob[2 * pr + 1][0], c1 = ob[2 * pr + 1][1];
    permlane16_swap(a0, c0);
    permlane16_swap(a1, c1);
    x0[pr] = a0; x1[pr] = a1; y0[pr] = c0; y1[pr] = c1;
  }
  if (q < p.N) {
    bf16* op = (bf16*)p.out + ((int64_t)b * p.N + q) * p.ldo + h * 64 + 16 * (g & 1) + 8 * (g >> 1);
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const u32x4 v = {x0[pr], x1[pr], y0[pr], y1[pr]};
      if (PLAIN_STORE) store_b128(op + 32 * pr, v);
      else store_b128_nt(op + 32 * pr, v);
    }
  }
}

// Stage one (image, head)'s K and V rows (NP rows, clamped past N) into LDS with glds, WAVES
// waves sharing the rows, and load the Q fragments of query tiles wave, wave + WAVES, ...
template <int NKT, int WAVES, int NQW, bool NT = false, bool NTQ = NT>
__device__ __forceinline__ void attn_stage_bf16(const AttnParams& p, EVT_LDS char* Ks,
                                                EVT_LDS char* Vs, u32x4 (&qf)[NQW][2], int b,
                                                int h, int wave, int lane) {
  constexpr int NP = NKT * 16, ROWB = 128;
  const bf16* qkv = (const bf16*)p.qkv + b * p.sb + h * p.sh;  // the (image, head) slice
  const int g = lane >> 4, c16 = lane & 15;
#pragma unroll
  for (int i = 0; i < NQW; ++i) {
    const int qi = min((wave + WAVES * i) * 16 + c16, p.N - 1);
    const bf16* qrow = qkv + (int64_t)qi * p.ldq;
    if (NTQ) {
      qf[i][0] = __builtin_nontemporal_load((const u32x4*)(qrow + 8 * g));
      qf[i][1] = __builtin_nontemporal_load((const u32x4*)(qrow + 8 * (g + 4)));
    } else {
      qf[i][0] = *(const u32x4*)(qrow + 8 * g);
      qf[i][1] = *(const u32x4*)(qrow + 8 * (g + 4));
    }
  }
  const int srow = lane >> 3, sslot = lane & 7;  // 8 rows of 128 B per wave-instruction
  for (int i = wave; i < NP / 8; i += WAVES) {
    const int row = i * 8 + srow;
    const int gr = min(row, p.N - 1);
    const bf16* rp = qkv + (int64_t)gr * p.ldq + ((sslot ^ srow) * 8);
    if (NT) {
      __builtin_amdgcn_global_load_lds(rp + p.ko, Ks + i * 8 * ROWB, 16, 0, 2);
      __builtin_amdgcn_global_load_lds(rp + p.vo, Vs + i * 8 * ROWB, 16, 0, 2);
    } else {
      glds16(rp + p.ko, Ks + i * 8 * ROWB);
      glds16(rp + p.vo, Vs + i * 8 * ROWB);
    }
  }
}

// One workgroup (4 waves) per (image, head); 3 per CU (53 KiB of LDS each).
template <int NKT, int NTM = 0>  // 16-key tiles (keys padded to NKT*16; odd NKT: a half last PV step)
__global__ __launch_bounds__(256, (NKT == 13 || NKT == 12) ? 3 : 1) void attn_bf16_kernel(AttnParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NP = NKT * 16, ROWB = 128;
  constexpr int NQW = (NP / 16 + 3) / 4;
  EVT_LDS char* Ks = (EVT_LDS char*)smem;
  EVT_LDS char* Vs = Ks + NP * ROWB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x / p.H, h = blockIdx.x - b * p.H;
  const int nqt = (p.N + 15) >> 4;
  u32x4 qf[NQW][2];
  // NTM: cache policy of the qkv loads / O stores, non-temporal for 1 all, 2 K/V loads only, 3 O
  // stores only, 4 K/V + Q loads only, 5 K/V loads + O stores (the launched form)
  attn_stage_bf16<NKT, 4, NQW, (NTM == 1 || NTM == 2 || NTM == 4 || NTM == 5), (NTM == 1 || NTM == 4)>(
      p, Ks, Vs, qf, b, h, wave, lane);
  wait_vmcnt0();
  __syncthreads();
#pragma unroll
  for (int it = 0; it < NQW; ++it) {
    const int qt = wave + 4 * it;
    if (qt >= nqt) break;
    attn_tile_bf16<NKT, !(NTM == 1 || NTM == 3 || NTM == 5)>(p, Ks, Vs, qf[it][0], qf[it][1], qt, b, h, lane);
  }
}

#ifndef ATTN_F32_WAVES
#define ATTN_F32_WAVES 8
#endif

template <int NKT>
__global__ __launch_bounds__(64 * ATTN_F32_WAVES) void attn_f32_kernel(AttnParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NP = NKT * 16;
  constexpr int ROWB = 256;  // 64 fp32
  EVT_LDS char* Ks = (EVT_LDS char*)smem;
  EVT_LDS char* Vs = Ks + NP * ROWB;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x / p.H, h = blockIdx.x - b * p.H;
  const float* qkv = (const float*)p.qkv + (int64_t)b * p.N * p.ldq;

  {
    const int srow = lane >> 4, sslot = lane & 15;  // 4 rows of 256 B per wave-instruction
    for (int i = wave; i < NP / 4; i += ATTN_F32_WAVES) {
      const int row = i * 4 + srow;
      const int gr = min(row, p.N - 1);
      const float* rp = qkv + (int64_t)gr * p.ldq + ((sslot ^ (row & 15)) * 4);
      glds16(rp + (p.H + h) * 64, Ks + i * 4 * ROWB);
      glds16(rp + (2 * p.H + h) * 64, Vs + i * 4 * ROWB);
    }
    wait_vmcnt0();
    __syncthreads();
  }

  const int g = lane >> 4, c16 = lane & 15;
  const int nqt = (p.N + 15) >> 4;
  for (int qt = wave; qt < nqt; qt += ATTN_F32_WAVES) {
    const int qi = min(qt * 16 + c16, p.N - 1);
    const float* qrow = qkv + (int64_t)qi * p.ldq + h * 64;
    f32x4 qf[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) qf[kk] = *(const f32x4*)(qrow + 4 * (g + 4 * kk));

    f32x4 s[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      const int row = kt * 16 + c16;
      const EVT_LDS char* kr = Ks + row * ROWB;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const f32x4 kf = *(const EVT_LDS f32x4*)(kr + (((g + 4 * kk) ^ (row & 15)) * 16));
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[e], qf[kk][e], acc, 0, 0, 0);
      }
      s[kt] = acc;
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int key = kt * 16 + 4 * g + j;
        if (key >= p.N) s[kt][j] = -INFINITY;
        mx = fmaxf(mx, s[kt][j]);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float moff = mx * p.scale_log2;
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float e = exp2f(s[kt][j] * p.scale_log2 - moff);
        s[kt][j] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);

    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        __builtin_amdgcn_sched_barrier(0);
        const int key = kt * 16 + 4 * g + e;
        // MFMA row m of o[dt] is head dim d = 4 m + dt: the lane's four V values are one 16-byte
        // LDS chunk (d = 4 c16 .. 4 c16 + 3)
        const f32x4 v = *(const EVT_LDS f32x4*)(Vs + key * ROWB + ((c16 ^ (key & 15)) * 16));
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[dt], s[kt][e], o[dt], 0, 0, 0);
      }
    const int q = qt * 16 + c16;
    if (q < p.N) {
      const float inv = 1.0f / sum;
      // lane holds O[d = 16 g + 4 j + dt][q] in o[dt][j]
      float* op = (float*)p.out + ((int64_t)b * p.N + q) * p.ldo + h * 64 + 16 * g;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        store4(op + 4 * j, f32x4{o[0][j], o[1][j], o[2][j], o[3][j]} * inv);
    }
  }
}

// ---- any head size (attention.py:6-12: h_k = dim // heads; attention_launch routes h_k != 64
// here). Same transposed-product structure as the head-size-64 kernels above.
//
// bf16: one workgroup (4 waves) per (image, head). K and V rows are staged to LDS with the head
// feature axis zero-padded to DP (h_k rounded up to 32, one k-step of v_mfma_f32_16x16x32_bf16),
// rows of DP * 2 bytes, 16-B chunk c of row r at chunk c ^ (r & SWM) (SWM: 7 / 3 when the chunk
// count is a power of two >= 8 / = 4, else unswizzled). S^T = K Q^T takes DP / 32 MFMA steps per
// 16-key tile, O^T = V^T P^T DP / 16 output tiles with V^T from ds_read_b64_tr_b16.
template <int DP>
constexpr int gen_swm() {
  constexpr int nch = DP / 8;
  return nch == 4 ? 3 : ((nch >= 8 && (nch & (nch - 1)) == 0) ? 7 : 0);
}

// 8 consecutive head features [d0, d0 + 8) of row `row` (bf16), zero past h_k
__device__ __forceinline__ u32x4 gen_chunk(const bf16* row, int d0, int hd) {
  if ((hd & 7) == 0) {
    if (d0 < hd) return *(const u32x4*)(row + d0);
    return u32x4{0u, 0u, 0u, 0u};
  }
  bf16x8 v;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = d0 + e < hd ? row[d0 + e] : (bf16)0.f;
  return __builtin_bit_cast(u32x4, v);
}

template <int NKT, int DP>
__global__ __launch_bounds__(256) void attn_gen_bf16_kernel(AttnParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NP = NKT * 16, NCH = DP / 8, RB = DP * 2, SWM = gen_swm<DP>(), KS = DP / 32;
  EVT_LDS char* Ks = (EVT_LDS char*)smem;
  EVT_LDS char* Vs = Ks + NP * RB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x / p.H, h = blockIdx.x - b * p.H, hd = p.hd;
  const bf16* qkv = (const bf16*)p.qkv + (int64_t)b * p.N * p.ldq;
  for (int i = tid; i < NP * NCH; i += 256) {
    const int row = i / NCH, ch = i - row * NCH;
    const bf16* rp = qkv + (int64_t)min(row, p.N - 1) * p.ldq;
    const int so = row * RB + ((ch ^ (row & SWM)) << 4);
    *(EVT_LDS u32x4*)(Ks + so) = gen_chunk(rp + (p.H + h) * hd, ch * 8, hd);
    *(EVT_LDS u32x4*)(Vs + so) = gen_chunk(rp + (2 * p.H + h) * hd, ch * 8, hd);
  }
  __syncthreads();
  const int g = lane >> 4, c16 = lane & 15;
  const int tq = (lane >> 2) & 3, tp = lane & 3;
  const int nqt = (p.N + 15) >> 4;
  for (int qt = wave; qt < nqt; qt += 4) {
    const bf16* qrow = qkv + (int64_t)min(qt * 16 + c16, p.N - 1) * p.ldq + h * hd;
    u32x4 qf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = gen_chunk(qrow, 32 * ks + 8 * g, hd);
    f32x4 s[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      const int row = kt * 16 + c16;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const u32x4 kf = *(const EVT_LDS u32x4*)(Ks + row * RB + (((4 * ks + g) ^ (row & SWM)) << 4));
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kf),
                                                      __builtin_bit_cast(bf16x8, qf[ks]), acc, 0, 0, 0);
      }
      s[kt] = acc;  // S^T[key = kt*16 + 4g + j][query = qt*16 + c16]
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (kt * 16 + 4 * g + j >= p.N) s[kt][j] = -INFINITY;
        mx = fmaxf(mx, s[kt][j]);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float moff = mx * p.scale_log2;
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float e = __builtin_amdgcn_exp2f(s[kt][j] * p.scale_log2 - moff);
        s[kt][j] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    f32x4 o[DP / 16];
#pragma unroll
    for (int dt = 0; dt < DP / 16; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < (NKT + 1) / 2; ++ks) {
      const bool half = 2 * ks + 1 >= NKT;  // odd NKT: the last 16 keys, upper k half zero
      bf16x8 pf;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pf[j] = (bf16)s[2 * ks][j];
        pf[4 + j] = half ? (bf16)0.f : (bf16)s[min(2 * ks + 1, NKT - 1)][j];
      }
      const int key0 = ks * 32 + 4 * g + tq;
      const int ksw = key0 & SWM;
#pragma unroll
      for (int dt = 0; dt < DP / 16; ++dt) {
        const int off = (((2 * dt + (tp >> 1)) ^ ksw) << 4) + (tp & 1) * 8;
        const i16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((EVT_LDS i16x4*)(Vs + key0 * RB + off));
        const i16x4 v1 = half ? i16x4{0, 0, 0, 0}
                              : __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                    (EVT_LDS i16x4*)(Vs + (key0 + 16) * RB + off));
        const i16x8 vv = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vv), pf, o[dt],
                                                        0, 0, 0);
      }
    }
    // o[dt][j] = O^T[d = dt*16 + 4g + j][query]
    const int q = qt * 16 + c16;
    if (q < p.N) {
      const float inv = 1.0f / sum;
      bf16* op = (bf16*)p.out + ((int64_t)b * p.N + q) * p.ldo + h * hd;
#pragma unroll
      for (int dt = 0; dt < DP / 16; ++dt) {
        const int d0 = dt * 16 + 4 * g;
        if ((hd & 3) == 0) {
          if (d0 < hd) store4(op + d0, o[dt] * inv);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (d0 + j < hd) op[d0 + j] = (bf16)(o[dt][j] * inv);
        }
      }
    }
  }
}

// fp32 (the exact parity path): one workgroup (4 waves) per (image, head), every operand read
// straight from the qkv rows (L2-resident per head): S^T = K Q^T on v_mfma_f32_16x16x4_f32 over
// 16-feature chunks, O^T = V^T P^T with MFMA row m of output tile (grp, dt) = head feature
// 64 grp + 4 m + dt; NG = ceil(h_k / 64) feature groups.
__device__ __forceinline__ f32x4 gen_load4(const float* row, int d0, int hd) {
  if ((hd & 3) == 0) return d0 < hd ? *(const f32x4*)(row + d0) : f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 v;
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = d0 + e < hd ? row[d0 + e] : 0.f;
  return v;
}

template <int NKT, int NG>
__global__ __launch_bounds__(256) void attn_gen_f32_kernel(AttnParams p) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x / p.H, h = blockIdx.x - b * p.H, hd = p.hd;
  const float* qkv = (const float*)p.qkv + (int64_t)b * p.N * p.ldq;
  const int g = lane >> 4, c16 = lane & 15;
  const int nqt = (p.N + 15) >> 4;
  for (int qt = wave; qt < nqt; qt += 4) {
    const float* qrow = qkv + (int64_t)min(qt * 16 + c16, p.N - 1) * p.ldq + h * hd;
    f32x4 s[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kk = 0; kk < 4 * NG; ++kk) {
      const int d0 = 16 * kk + 4 * g;
      const f32x4 qf = gen_load4(qrow, d0, hd);
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        const float* krow = qkv + (int64_t)min(kt * 16 + c16, p.N - 1) * p.ldq + (p.H + h) * hd;
        const f32x4 kf = gen_load4(krow, d0, hd);
#pragma unroll
        for (int e = 0; e < 4; ++e) s[kt] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[e], qf[e], s[kt], 0, 0, 0);
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (kt * 16 + 4 * g + j >= p.N) s[kt][j] = -INFINITY;
        mx = fmaxf(mx, s[kt][j]);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float moff = mx * p.scale_log2;
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float e = exp2f(s[kt][j] * p.scale_log2 - moff);
        s[kt][j] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    f32x4 o[NG][4];
#pragma unroll
    for (int gr = 0; gr < NG; ++gr)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[gr][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int key = min(kt * 16 + 4 * g + e, p.N - 1);  // P is 0 for keys past N
        const float* vrow = qkv + (int64_t)key * p.ldq + (2 * p.H + h) * hd;
#pragma unroll
        for (int gr = 0; gr < NG; ++gr) {
          const f32x4 v = gen_load4(vrow, 64 * gr + 4 * c16, hd);
#pragma unroll
          for (int dt = 0; dt < 4; ++dt)
            o[gr][dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[dt], s[kt][e], o[gr][dt], 0, 0, 0);
        }
      }
    const int q = qt * 16 + c16;
    if (q < p.N) {
      const float inv = 1.0f / sum;
      float* op = (float*)p.out + ((int64_t)b * p.N + q) * p.ldo + h * hd;
      // lane holds O[d = 64 grp + 16 g + 4 j + dt][q] in o[grp][dt][j]
#pragma unroll
      for (int gr = 0; gr < NG; ++gr)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int d0 = 64 * gr + 16 * g + 4 * j;
          const f32x4 v = f32x4{o[gr][0][j], o[gr][1][j], o[gr][2][j], o[gr][3][j]} * inv;
          if ((hd & 3) == 0) {
            if (d0 < hd) store4(op + d0, v);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (d0 + e < hd) op[d0 + e] = v[e];
          }
        }
    }
  }
}

template <int NKT, int DP>
hipError_t launch_gen_bf16(const AttnParams& p, hipStream_t s) {
  const size_t lds = 2 * (size_t)NKT * 16 * DP * 2;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)attn_gen_bf16_kernel<NKT, DP>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((attn_gen_bf16_kernel<NKT, DP>), dim3(p.B * p.H), dim3(256), lds, s, p);
  return hipGetLastError();
}

template <int NKT>
hipError_t launch_gen(int dtype, const AttnParams& p, hipStream_t s) {
  if (dtype == DT_BF16) {
    if (p.hd <= 32) return launch_gen_bf16<NKT, 32>(p, s);
    if (p.hd <= 64) return launch_gen_bf16<NKT, 64>(p, s);
    if (p.hd <= 96) return launch_gen_bf16<NKT, 96>(p, s);
    return launch_gen_bf16<NKT, 128>(p, s);
  }
  if (p.hd <= 64)
    hipLaunchKernelGGL((attn_gen_f32_kernel<NKT, 1>), dim3(p.B * p.H), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((attn_gen_f32_kernel<NKT, 2>), dim3(p.B * p.H), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t attention_gen_launch(int dtype, const AttnParams& p, hipStream_t s) {
  if (p.N <= 64) return launch_gen<4>(dtype, p, s);
  if (p.N <= 128) return launch_gen<8>(dtype, p, s);
  if (p.N <= 208) return launch_gen<13>(dtype, p, s);
  return launch_gen<16>(dtype, p, s);
}

template <int NKT>
hipError_t launch_nkt(int dtype, const AttnParams& p, hipStream_t s) {
  const int rowb = dtype == DT_BF16 ? 128 : 256;
  const size_t lds = 2 * (size_t)NKT * 16 * rowb;
  // K / V loads and O stores non-temporal (NTM 5): measured in the model, out-proj (whose A is O
  // and whose residual x was read by the QKV GEMM just before) 161 -> 157 us and attention equal
  // or 2 us faster; all-NT (Q too) made attention 4 us slower (scripts/gpu_attnnt.sh)
  if (dtype == DT_BF16)
    hipLaunchKernelGGL((attn_bf16_kernel<NKT, 5>), dim3(p.B * p.H), dim3(256), lds, s, p);
  else if constexpr (NKT % 2 == 0)
    hipLaunchKernelGGL(attn_f32_kernel<NKT>, dim3(p.B * p.H), dim3(64 * ATTN_F32_WAVES), lds, s, p);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

bool g_attr_set = false;

void set_lds_attrs() {
  if (g_attr_set) return;
  g_attr_set = true;
  (void)hipFuncSetAttribute((const void*)attn_f32_kernel<14>, hipFuncAttributeMaxDynamicSharedMemorySize,
                      2 * 14 * 16 * 256);
  (void)hipFuncSetAttribute((const void*)attn_f32_kernel<16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                      2 * 16 * 16 * 256);
}

}  // namespace

hipError_t attention_launch(int dtype, const AttnParams& p_in, hipStream_t s) {
  if (p_in.B <= 0) return hipSuccess;
  if (p_in.N <= 0 || p_in.N > 256 || p_in.H <= 0 || p_in.hd <= 0 || p_in.hd > 128)
    return hipErrorInvalidValue;
  AttnParams p = p_in;
  const bool strided = p.sb || p.sh || p.ko || p.vo;
  if (strided) {  // an explicit slice layout: the bf16 h_k = 64 kernels only, 16-B aligned pieces
    if (dtype != DT_BF16 || p.hd != 64 || p.q8 || p.sb % 8 || p.sh % 8 || p.ldq % 8 || p.ko % 8 ||
        p.vo % 8 || p.ldq < 64 || p.ko < 0 || p.vo < 0 || p.sb < 0 || p.sh < 0)
      return hipErrorInvalidValue;
  } else {
    p.sb = (int64_t)p.N * p.ldq;
    p.sh = 64;
    p.ko = p.H * 64;
    p.vo = 2 * p.H * 64;
  }
  if (p.hd != 64) {  // any other head size: the generic kernels (MX8 output: head size 64 only)
    if (p.q8) return hipErrorInvalidValue;
    return attention_gen_launch(dtype, p, s);
  }
  set_lds_attrs();
  if (p.N <= 64) return launch_nkt<4>(dtype, p, s);
  if (p.N <= 128) return launch_nkt<8>(dtype, p, s);
  if (dtype == DT_BF16 && p.N <= 192) return launch_nkt<12>(dtype, p, s);
  if (dtype == DT_BF16 && p.N <= 208) return launch_nkt<13>(dtype, p, s);  // 3 blocks per CU (LDS)
  if (p.N <= 224) return launch_nkt<14>(dtype, p, s);  // (f32: N in (128, 224])
  return launch_nkt<16>(dtype, p, s);
}

}  // namespace evt
