// MXFP8 (OCP Microscaling) GEMM, activation quantizer and weight packer for gfx950.
//
// The MI355X counterpart of the reference's reduced-precision axis (TFLite float16 / dynamic-range
// / int8 post-training quantization, `utils.py:242-294`, driven by `tools.py:458-498,826-844`):
// instead of TFLite's per-tensor int8, the matrix cores' native block-scaled format. A tensor is
// e4m3fn elements (OCP FP8, max 448) with one e8m0 scale per 32 consecutive K elements:
//
//   value(r, k) = e4m3(q[r][k]) * 2^(sbyte(r, k / 32) - 127)
//
// Scales are stored k-step-major as dwords S[K / 128][ld_s] (byte j of S[ks][r] = block 4 ks + j of
// row r), so one GEMM k-step of a 128-row tile reads 512 contiguous bytes of each operand's scales.
// Quantization follows the OCP MX v1.0 rule: shared exponent = floor(log2(amax)) - 8 (8 = emax of
// e4m3), elements = RNE(v / 2^e) saturated to +-448; an all-zero block gets scale byte 0.
//
// GEMM: v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3, hardware-applied block scales), 2x the
// bf16 MFMA rate (operand K order and scale lanes measured on the device: scripts/probe/).
// Persistent 128 x 256 tiles, 8 waves (2 x 4) of 64 x 64, K step 128 bytes, operands and
// scales staged into LDS with global_load_lds in a 3-stage pipeline (148.5 KiB, one workgroup
// per CU, two stages in flight under every k-step; 128 x 128 tiles with 2 stages and 2
// workgroups per CU measured 755 TF/s on the DeiT QKV shape: load-latency bound). The product is computed transposed
// (D^T = W . X^T) with the W rows of each 32-column pair interleaved, so every lane ends with 8
// consecutive output columns of one row: 16-B bf16 stores, and a 32-column MX block of the output
// spans exactly the 4 lane groups of one row (2 shuffles for its amax).
#include <mutex>

#include "common.h"
#include "evt_internal.h"

namespace evt {

namespace {

constexpr int MX_BM = 128, MX_BN = 256, MX_BK = 128;  // K step in elements (= bytes)
constexpr int MX_STAGE = MX_BM * MX_BK + MX_BN * MX_BK + 4 * MX_BM + 4 * MX_BN;  // 50688 B
constexpr int MX_NSTAGE = 3;                                                    // 148.5 KiB

typedef __attribute__((ext_vector_type(8))) int i32x8;

// Shared MX scale of a block with absolute maximum amax: the e8m0 byte, and 2^-(e) as fp32.
__device__ __forceinline__ unsigned mx8_scale_byte(float amax) {
  const int E = (int)((__float_as_uint(amax) >> 23) & 0xff);  // biased exponent (0: zero/denormal)
  return (unsigned)max(E - 8, 0);
}
__device__ __forceinline__ float mx8_inv_scale(unsigned sb) {  // 2^(127 - sb), sb <= 246
  return __uint_as_float((254u - sb) << 23);
}
// 8 fp32 values (already multiplied by the inverse scale) -> 8 e4m3fn bytes, RNE, saturated.
__device__ __forceinline__ u32x2 mx8_pack8(const float (&v)[8]) {
  float c[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = __builtin_amdgcn_fmed3f(v[i], -448.f, 448.f);
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[4], c[5], 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[6], c[7], hi, true);
  return u32x2{(unsigned)lo, (unsigned)hi};
}

// ---- activation quantizer: rows of K (bf16 / fp32) -> MX8 rows of Kpad ------------------------
// One lane per 8 elements, 4 lanes per 32-element block (amax over xor-1/2 shuffles).
template <typename T>
__global__ __launch_bounds__(256) void mx8_quantize_kernel(const T* __restrict__ x, int64_t ldx,
                                                           int rows, int K, int Kpad,
                                                           uint8_t* __restrict__ q, int64_t ldq,
                                                           uint32_t* __restrict__ s, int64_t lds) {
  const int chunks = Kpad >> 3;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int r = (int)(t / chunks), c = (int)(t - (int64_t)r * chunks);
  const bool live = r < rows;
  float v[8];
  const int k0 = c * 8;
  if (live && k0 < K) {
    const T* p = x + (int64_t)r * ldx + k0;
    const f32x4 a = load4(p), b = load4(p + 4);
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
    v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0.f;
  }
  float am = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) am = fmaxf(am, fabsf(v[i]));
  am = fmaxf(am, __shfl_xor(am, 1, 64));
  am = fmaxf(am, __shfl_xor(am, 2, 64));
  const unsigned sb = mx8_scale_byte(am);
  const float inv = mx8_inv_scale(sb);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] *= inv;
  const u32x2 o = mx8_pack8(v);
  if (!live) return;
  *(u32x2*)(q + (int64_t)r * ldq + k0) = o;
  if ((c & 3) == 0) {
    const int blk = c >> 2;  // 32-element block
    ((uint8_t*)s)[((int64_t)(blk >> 2) * lds + r) * 4 + (blk & 3)] = (uint8_t)sb;
  }
}

// ---- LayerNorm + MX8 quantization of a bf16 token stream (the MX8 model's LN1 / LN2) --------
// One wave per row: y = (x - mu) * rsqrt(var + eps) * gamma + beta (population variance, Keras
// LayerNormalization, reference norm.py:6) written as MX8 [Kpad] (columns past D quantized as
// zeros), and (mu, rstd) per row when stats != null: the consumer GEMM re-forms the reference
// block's residual LN(x) (norm.py:11-12) in its epilogue (EPI_RESLN) instead of a bf16 copy.
// Lane l owns 8-element chunks l, l + 64 (D <= 1024); 4 consecutive chunks = one MX block.
__global__ __launch_bounds__(256) void ln_mx8_kernel(const bf16* __restrict__ x, int rows, int D,
                                                     int Kpad, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps,
                                                     f32x2* __restrict__ stats,
                                                     uint8_t* __restrict__ q,
                                                     uint32_t* __restrict__ s) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;  // wave-uniform
  const int nch = D >> 3, nq = Kpad >> 3;
  const bf16* xr = x + (int64_t)r * D;
  float v[2][8];
  float sum = 0.f;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int c = lane + 64 * it;
    if (c < nch) {
      const bf16x8 b = *(const bf16x8*)(xr + 8 * c);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[it][e] = (float)b[e];
        sum += v[it][e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[it][e] = 0.f;
    }
  }
  const float mu = wave_sum(sum) / (float)D;
  float sq = 0.f;
#pragma unroll
  for (int it = 0; it < 2; ++it)
    if (lane + 64 * it < nch)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[it][e] - mu;
        sq += d * d;
      }
  const float rstd = rsqrtf(wave_sum(sq) / (float)D + eps);
  if (stats && lane == 0) stats[r] = f32x2{mu, rstd};
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int c = lane + 64 * it;
    if (64 * it >= nq) break;  // wave-uniform: no chunk of this pass is in the padded row
    const bool live = c < nch;
    if (live) {
      const f32x4 g0 = *(const f32x4*)(gamma + 8 * c), g1 = *(const f32x4*)(gamma + 8 * c + 4);
      const f32x4 b0 = *(const f32x4*)(beta + 8 * c), b1 = *(const f32x4*)(beta + 8 * c + 4);
      const float gg[8] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3]};
      const float bb[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[it][e] = (v[it][e] - mu) * rstd * gg[e] + bb[e];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[it][e] = 0.f;
    }
    float am = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(v[it][e]));
    am = fmaxf(am, __shfl_xor(am, 1, 64));
    am = fmaxf(am, __shfl_xor(am, 2, 64));
    const unsigned sb = mx8_scale_byte(am);
    const float inv = mx8_inv_scale(sb);
    float t[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) t[e] = v[it][e] * inv;
    const u32x2 o8 = mx8_pack8(t);
    // the 4 scale bytes of a 128-column k-step come from lanes c, c+4, c+8, c+12 (c % 16 == 0):
    // gather them into one dword store instead of 4 byte stores
    const unsigned s1 = __shfl_down(sb, 4, 64), s2 = __shfl_down(sb, 8, 64),
                   s3 = __shfl_down(sb, 12, 64);
    if (c < nq) {
      *(u32x2*)(q + (int64_t)r * Kpad + 8 * c) = o8;
      if ((c & 15) == 0) s[(int64_t)(c >> 4) * rows + r] = sb | (s1 << 8) | (s2 << 16) | (s3 << 24);
    }
  }
}

// ---- weight packer: Keras W[K][N] fp32 (optionally row-scaled) -> Wq[Npad][Kpad], S[Kpad/128][Npad]
// One thread per (column n, 32-row block of K); consecutive threads take consecutive n (coalesced
// reads of the W rows). Padding rows / columns are written as zeros with scale byte 0.
__global__ __launch_bounds__(256) void mx8_pack_kernel(const float* __restrict__ W,
                                                       const float* __restrict__ row_scale, int K,
                                                       int N, uint8_t* __restrict__ Wq, int Kpad,
                                                       int Npad, uint32_t* __restrict__ s) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int nblk = Kpad >> 5;
  if (t >= (int64_t)nblk * Npad) return;
  const int blk = (int)(t / Npad), n = (int)(t - (int64_t)blk * Npad);
  float v[32];
  float am = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int k = blk * 32 + i;
    float w = 0.f;
    if (n < N && k < K) {
      w = W[(int64_t)k * N + n];
      if (row_scale) w *= row_scale[k];
    }
    v[i] = w;
    am = fmaxf(am, fabsf(w));
  }
  const unsigned sb = mx8_scale_byte(am);
  const float inv = mx8_inv_scale(sb);
  uint8_t* dst = Wq + (int64_t)n * Kpad + blk * 32;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float c[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = v[8 * j + i] * inv;
    *(u32x2*)(dst + 8 * j) = mx8_pack8(c);
  }
  ((uint8_t*)s)[((int64_t)(blk >> 2) * Npad + n) * 4 + (blk & 3)] = (uint8_t)sb;
}

// ---- GEMM -----------------------------------------------------------------------------------
// LDS images are 128-B rows of 16-B chunks, physical chunk = chunk ^ key(row), applied on the glds
// source address and on every read. ds_read_b128 is serviced in 16-lane groups whose 16 reads must
// hit distinct (row parity, chunk) slots of the 256-B bank row: X fragments read 16 consecutive
// rows -> key (row >> 1) & 7; W fragments read rows 8q + s (+ 4h) for l16 = 4q + s -> key
// 2 ((row >> 3) & 3) + ((row >> 1) & 1). Both conflict-free for the lane groups of the table in
// MI355X_MICROARCH.md (checked by hand for both 16-B halves of every fragment).
__device__ __forceinline__ int xkey(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int wkey(int row) { return (((row >> 3) & 3) << 1) | ((row >> 1) & 1); }

// Epilogue of one tile: lane (l16, g) of wave (wm, wn) holds row m = m0 + wm*64 + mt*16 + l16,
// columns n .. n+7 with n = n0 + wn*64 + pp*32 + 8g, from acc[2pp][mt] (n..n+3) and
// acc[2pp+1][mt] (n+4..n+7).
template <int FL>
__device__ __forceinline__ void mx8_epilogue(const Mx8GemmParams& p, const f32x4 (&acc)[4][4],
                                             int m0, int n0, int wm, int wn, int g, int l16) {
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
    const int n = n0 + wn * 64 + pp * 32 + 8 * g;
    const bool nok = n < p.N;
    f32x4 b0 = {0.f, 0.f, 0.f, 0.f}, b1 = b0, g0 = b0, g1 = b0, e0 = b0, e1 = b0;
    if ((FL & EPI_BIAS) && nok) {
      b0 = *(const f32x4*)(p.bias + n);
      b1 = *(const f32x4*)(p.bias + n + 4);
    }
    if ((FL & EPI_RESLN) && nok) {  // LayerNorm gamma / beta of the residual
      g0 = *(const f32x4*)(p.rgamma + n);
      g1 = *(const f32x4*)(p.rgamma + n + 4);
      e0 = *(const f32x4*)(p.rbeta + n);
      e1 = *(const f32x4*)(p.rbeta + n + 4);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int m = m0 + wm * 64 + mt * 16 + l16;
      const bool ok = nok && m < p.M;
      f32x4 lo = acc[2 * pp][mt], hi = acc[2 * pp + 1][mt];
      if (FL & EPI_BIAS) {
        lo += b0;
        hi += b1;
      }
      if (FL & (EPI_GELU | EPI_GELU_ERF)) {
        const int mode = (FL & EPI_GELU_ERF) ? 2 : 0;
        lo = gelu4(lo, mode);
        hi = gelu4(hi, mode);
      }
      if ((FL & EPI_RESID) && ok) {
        const bf16x8 r8 = *(const bf16x8*)((const bf16*)p.resid + (int64_t)m * p.ldr + n);
        f32x4 rlo = {(float)r8[0], (float)r8[1], (float)r8[2], (float)r8[3]};
        f32x4 rhi = {(float)r8[4], (float)r8[5], (float)r8[6], (float)r8[7]};
        if (FL & EPI_RESLN) {  // residual LN(resid) from the row's (mu, rstd)
          const f32x2 st = ((const f32x2*)p.rstats)[m];
          rlo = (rlo - st[0]) * st[1] * g0 + e0;
          rhi = (rhi - st[0]) * st[1] * g1 + e1;
        }
        lo += rlo;
        hi += rhi;
      }
      if constexpr ((FL & EPI_OUT_MX8) != 0) {
        float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        float am = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) am = fmaxf(am, fabsf(v[i]));
        am = fmaxf(am, __shfl_xor(am, 16, 64));
        am = fmaxf(am, __shfl_xor(am, 32, 64));
        const unsigned sb = mx8_scale_byte(am);
        const float inv = mx8_inv_scale(sb);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] *= inv;
        const u32x2 o = mx8_pack8(v);
        if (ok) {
          *(u32x2*)((uint8_t*)p.C + (int64_t)m * p.ldc + n) = o;
          if (g == 0) {
            const int blk = n >> 5;
            ((uint8_t*)p.Cs)[((int64_t)(blk >> 2) * p.ldcs + m) * 4 + (blk & 3)] = (uint8_t)sb;
          }
        }
      } else if constexpr ((FL & EPI_OUT_F32) != 0) {
        if (ok) {
          float* c = (float*)p.C + (int64_t)m * p.ldc + n;
          store_f32x4(c, lo);
          store_f32x4(c + 4, hi);
        }
      } else {
        if (ok) {
          const bf16x8 o = {(bf16)lo[0], (bf16)lo[1], (bf16)lo[2], (bf16)lo[3],
                            (bf16)hi[0], (bf16)hi[1], (bf16)hi[2], (bf16)hi[3]};
          store_bf16x8((bf16*)p.C + (int64_t)m * p.ldc + n, o);
        }
      }
    }
  }
}

// Persistent: one 8-wave workgroup per CU walks the tiles u = blockIdx + j * gridDim
// (XCD-remapped); the (tile, k-step) sequence is one flat 3-stage glds pipeline (two stages in
// flight during every k-step's MFMAs, the next tile's first stage during the epilogue).
template <int FL>
__global__ __launch_bounds__(512, 1) void gemm_mx8_kernel(Mx8GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int g = lane >> 4, l16 = lane & 15;
  const int ntn = (p.N + MX_BN - 1) / MX_BN, ntm = (p.M + MX_BM - 1) / MX_BM;
  const int nb = ntm * ntn, nk = p.K / MX_BK;
  const int b = blockIdx.x, grid = gridDim.x;
  const int mine = b < nb ? (nb - 1 - b) / grid + 1 : 0;
  const int total = mine * nk;
  // XCD-aware tile order: workgroup b runs on XCD b % 8 (grid is a multiple of 8), so give XCD x
  // a contiguous run of tiles (row panels n-fastest: the A panel stays in its L2)
  // (the first nb & ~7 tiles are dealt out; a tail of < 8 tiles keeps its index)
  const int nb8 = nb & ~7;
  auto tile_of = [&](int j) {
    int u = b + j * grid;
    if ((grid & 7) == 0 && u < nb8) u = (u & 7) * (nb8 >> 3) + (u >> 3);
    return u;
  };

  // glds: per stage 16 A and 32 W wave-instructions of 8 rows x 128 B (2 + 4 per wave), the
  // swizzle on the per-lane source chunk; scale dwords by waves 0 (A, 2 x 64) and 1-2 (W, 4 x 64)
  const int srow = lane >> 3, spc = lane & 7;
  int arow[2], ach[2], wrow[4], wch[4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    arow[i] = (wave * 2 + i) * 8 + srow;
    ach[i] = (spc ^ xkey(arow[i])) * 16;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    wrow[i] = (wave * 4 + i) * 8 + srow;
    wch[i] = (spc ^ wkey(wrow[i])) * 16;
  }
  auto issue = [&](int s) {
    const int j = s / nk, ks = s - j * nk;
    const int t = tile_of(j);
    const int tm = t / ntn, m0 = tm * MX_BM, n0 = (t - tm * ntn) * MX_BN;
    EVT_LDS char* st = (EVT_LDS char*)smem + (s % MX_NSTAGE) * MX_STAGE;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      glds16(p.A + (int64_t)min(m0 + arow[i], p.M - 1) * p.lda + ks * MX_BK + ach[i],
             st + (wave * 2 + i) * 8 * MX_BK);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      glds16(p.W + (int64_t)min(n0 + wrow[i], (int)p.ldws - 1) * p.ldw + ks * MX_BK + wch[i],
             st + MX_BM * MX_BK + (wave * 4 + i) * 8 * MX_BK);
    EVT_LDS char* sd = st + (MX_BM + MX_BN) * MX_BK;
    if (wave == 0) {
      const uint32_t* src = p.As + (int64_t)ks * p.ldas;
      __builtin_amdgcn_global_load_lds(src + min(m0 + lane, p.M - 1), sd, 4, 0, 0);
      __builtin_amdgcn_global_load_lds(src + min(m0 + 64 + lane, p.M - 1), sd + 256, 4, 0, 0);
    } else if (wave <= 2) {
      // (tiles past the packed width, Npad = ldws a multiple of 128 only: rows clamped)
      const uint32_t* src = p.Ws + (int64_t)ks * p.ldws;
      const int c0 = n0 + (wave - 1) * 128 + lane, last = (int)p.ldws - 1;
      EVT_LDS char* wd = sd + 4 * MX_BM + (wave - 1) * 512;
      __builtin_amdgcn_global_load_lds(src + min(c0, last), wd, 4, 0, 0);
      __builtin_amdgcn_global_load_lds(src + min(c0 + 64, last), wd + 256, 4, 0, 0);
    }
  };

  // Lane group g holds k-step bytes [16g, 16g+16) and [64+16g, 64+16g+16) (the hardware K order
  // of the 16x16x128 operands: block b = bytes [32b, 32b+32) is scaled by lane group b's scale).
  // X rows (MFMA B operand): wm*64 + mt*16 + l16. W rows (MFMA A operand) of tile nt = 2 pp + h:
  // wn*64 + pp*32 + 8 (l16 >> 2) + 4 h + (l16 & 3), so that accumulator register r of lane
  // (l16, g) in tiles 2pp / 2pp+1 is output column pp*32 + 8g + r / + 4 + r.
  int xoa[4], xob[4], woa[4], wob[4], xso[4], wso[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int xr = wm * 64 + i * 16 + l16;
    const int wr = wn * 64 + (i >> 1) * 32 + 8 * (l16 >> 2) + 4 * (i & 1) + (l16 & 3);
    xoa[i] = xr * MX_BK + ((g ^ xkey(xr)) << 4);
    xob[i] = xr * MX_BK + (((g + 4) ^ xkey(xr)) << 4);
    woa[i] = MX_BM * MX_BK + wr * MX_BK + ((g ^ wkey(wr)) << 4);
    wob[i] = MX_BM * MX_BK + wr * MX_BK + (((g + 4) ^ wkey(wr)) << 4);
    xso[i] = (MX_BM + MX_BN) * MX_BK + xr * 4;
    wso[i] = (MX_BM + MX_BN) * MX_BK + 4 * MX_BM + wr * 4;
  }

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (total == 0) return;
  issue(0);
  if (total > 1) issue(1);
  int ks = 0, j = 0;
  for (int s = 0; s < total; ++s) {
    // stage s complete; stage s+1 may stay in flight. The vector memory counter retires in order
    // and stage s+1 is always the youngest group issued (a tile's epilogue runs BEFORE the next
    // prefetch is issued), so vmcnt(#loads of one stage) also covers the epilogue's loads and
    // stores, whatever their data-dependent count.
    if (s + 1 >= total) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (wave <= 2) {
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    }
    // a bare s_barrier (__syncthreads' fence would drain the prefetch stage with vmcnt(0))
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const bool tile_end = ks + 1 == nk;
    if (!tile_end && s + 2 < total) issue(s + 2);
    const EVT_LDS char* st = (const EVT_LDS char*)smem + (s % MX_NSTAGE) * MX_STAGE;
    i32x8 xf[4], wf[4];
    int xs[4], ws[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const u32x4 x0 = *(const EVT_LDS u32x4*)(st + xoa[i]);
      const u32x4 x1 = *(const EVT_LDS u32x4*)(st + xob[i]);
      const u32x4 w0 = *(const EVT_LDS u32x4*)(st + woa[i]);
      const u32x4 w1 = *(const EVT_LDS u32x4*)(st + wob[i]);
      xf[i] = i32x8{(int)x0[0], (int)x0[1], (int)x0[2], (int)x0[3],
                    (int)x1[0], (int)x1[1], (int)x1[2], (int)x1[3]};
      wf[i] = i32x8{(int)w0[0], (int)w0[1], (int)w0[2], (int)w0[3],
                    (int)w1[0], (int)w1[1], (int)w1[2], (int)w1[3]};
      xs[i] = (int)(*(const EVT_LDS uint32_t*)(st + xso[i]) >> (8 * g));
      ws[i] = (int)(*(const EVT_LDS uint32_t*)(st + wso[i]) >> (8 * g));
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        acc[nt][mt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
            wf[nt], xf[mt], acc[nt][mt], 0, 0, 0, ws[nt], 0, xs[mt]);
    if (tile_end) {
      const int t = tile_of(j);
      const int tm = t / ntn;
      mx8_epilogue<FL>(p, acc, tm * MX_BM, (t - tm * ntn) * MX_BN, wm, wn, g, l16);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (s + 2 < total) issue(s + 2);
      ks = 0;
      ++j;
    } else {
      ++ks;
    }
  }
}

// Per-device launch state: the dynamic-LDS attribute of each kernel instantiation (set once per
// device, return code checked) and the device's CU count. Guarded by a mutex: the first calls
// from two threads, or on two devices, must not race on the caches.
constexpr int MX_MAX_DEV = 64;
std::mutex g_mx8_mu;
int g_mx8_cus[MX_MAX_DEV];

template <int FL>
hipError_t launch_mx8(const Mx8GemmParams& p, hipStream_t s) {
  static bool attr[MX_MAX_DEV];
  int dev = 0, cus = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= MX_MAX_DEV) return hipErrorInvalidDevice;
  {
    std::lock_guard<std::mutex> lk(g_mx8_mu);
    if (!attr[dev]) {
      e = hipFuncSetAttribute((const void*)gemm_mx8_kernel<FL>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, MX_NSTAGE * MX_STAGE);
      if (e != hipSuccess) return e;
      attr[dev] = true;
    }
    if (!g_mx8_cus[dev]) {
      e = hipDeviceGetAttribute(&g_mx8_cus[dev], hipDeviceAttributeMultiprocessorCount, dev);
      if (e != hipSuccess || g_mx8_cus[dev] <= 0) g_mx8_cus[dev] = 256;
    }
    cus = g_mx8_cus[dev];
  }
  const int nb = ((p.M + MX_BM - 1) / MX_BM) * ((p.N + MX_BN - 1) / MX_BN);
  const int grid = min(nb, cus);  // one resident 8-wave workgroup per CU (148.5 KiB of LDS)
  hipLaunchKernelGGL(gemm_mx8_kernel<FL>, dim3(grid), dim3(512), MX_NSTAGE * MX_STAGE, s, p);
  return hipGetLastError();
}

}  // namespace

hipError_t mx8_quantize_launch(int in_dtype, const void* x, int64_t ldx, int rows, int K, int Kpad,
                               void* q, int64_t ldq, uint32_t* s, int64_t lds, hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  const int64_t threads = (int64_t)rows * (Kpad >> 3);
  const dim3 grid((unsigned)((threads + 255) / 256));
  if (in_dtype == DT_BF16)
    hipLaunchKernelGGL(mx8_quantize_kernel<bf16>, grid, dim3(256), 0, st, (const bf16*)x, ldx,
                       rows, K, Kpad, (uint8_t*)q, ldq, s, lds);
  else
    hipLaunchKernelGGL(mx8_quantize_kernel<float>, grid, dim3(256), 0, st, (const float*)x, ldx,
                       rows, K, Kpad, (uint8_t*)q, ldq, s, lds);
  return hipGetLastError();
}

hipError_t ln_mx8_launch(const void* x, int rows, int D, int Kpad, const float* gamma,
                         const float* beta, float eps, float* stats, void* q, uint32_t* s,
                         hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  if (D % 8 || D > 1024 || Kpad % 128 || Kpad < D || Kpad > 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ln_mx8_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, (const bf16*)x, rows,
                     D, Kpad, gamma, beta, eps, (f32x2*)stats, (uint8_t*)q, s);
  return hipGetLastError();
}

hipError_t mx8_pack_launch(const float* W, const float* row_scale, int K, int N, void* Wq, int Kpad,
                           int Npad, uint32_t* s, hipStream_t st) {
  const int64_t threads = (int64_t)(Kpad >> 5) * Npad;
  hipLaunchKernelGGL(mx8_pack_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st,
                     W, row_scale, K, N, (uint8_t*)Wq, Kpad, Npad, s);
  return hipGetLastError();
}

hipError_t gemm_mx8_launch(int flags, const Mx8GemmParams& p, hipStream_t s) {
  if (p.M <= 0) return hipSuccess;
  switch (flags) {
    case 0: return launch_mx8<0>(p, s);
    case EPI_BIAS: return launch_mx8<EPI_BIAS>(p, s);
    case EPI_BIAS | EPI_GELU: return launch_mx8<EPI_BIAS | EPI_GELU>(p, s);
    case EPI_BIAS | EPI_GELU_ERF: return launch_mx8<EPI_BIAS | EPI_GELU_ERF>(p, s);
    case EPI_BIAS | EPI_RESID: return launch_mx8<EPI_BIAS | EPI_RESID>(p, s);
    case EPI_BIAS | EPI_RESID | EPI_RESLN:  // the MX8 model's out-proj / FC2 (capi.cpp)
      return launch_mx8<EPI_BIAS | EPI_RESID | EPI_RESLN>(p, s);
    case EPI_OUT_F32: return launch_mx8<EPI_OUT_F32>(p, s);
    case EPI_BIAS | EPI_OUT_F32: return launch_mx8<EPI_BIAS | EPI_OUT_F32>(p, s);
    case EPI_BIAS | EPI_GELU | EPI_OUT_F32: return launch_mx8<EPI_BIAS | EPI_GELU | EPI_OUT_F32>(p, s);
    case EPI_BIAS | EPI_GELU_ERF | EPI_OUT_F32:
      return launch_mx8<EPI_BIAS | EPI_GELU_ERF | EPI_OUT_F32>(p, s);
    case EPI_OUT_MX8: return launch_mx8<EPI_OUT_MX8>(p, s);
    case EPI_BIAS | EPI_OUT_MX8: return launch_mx8<EPI_BIAS | EPI_OUT_MX8>(p, s);
    case EPI_BIAS | EPI_GELU | EPI_OUT_MX8: return launch_mx8<EPI_BIAS | EPI_GELU | EPI_OUT_MX8>(p, s);
    case EPI_BIAS | EPI_GELU_ERF | EPI_OUT_MX8:
      return launch_mx8<EPI_BIAS | EPI_GELU_ERF | EPI_OUT_MX8>(p, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace evt
