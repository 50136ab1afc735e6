// Token-matrix GEMM for the ViT encoder on gfx950 (MI355X, CDNA4).
//
// Replaces every tf.keras.layers.Dense on the hot path (reference `modeling/layers/attention.py:17-18`
// to_qkv / to_out, `modeling/layers/ffn.py:8-9` FC1+gelu / FC2, `modeling/models/vit.py:23,38-39`
// patch_to_embedding / mlp_head) with fused epilogues, including the two LayerNorms of every
// encoder layer (reference `modeling/layers/norm.py:6,12`), which never run as kernels of their
// own (see "LayerNorm folding" below).
//
// Layout. A (activations) is row-major [M][lda]; weights are packed once at model creation to
// Wp[Npad][Kpad] (K-contiguous, zero padded), so both MFMA operands are 16-byte K-contiguous
// reads. Tiles of A and W are staged into LDS with global_load_lds (async, 16 B/lane); the LDS
// image is row-linear and the bank-conflict swizzle (chunk ^ (row & 7)) is applied to the
// per-lane SOURCE address and to the ds_read address (glds writes lane-linear).
//
// MFMA. The product is computed transposed, C^T = W . A^T (16x16 C layout: col = lane&15 ->
// token row m, row = 4*(lane>>4)+j -> feature n).
//   bf16: v_mfma_f32_16x16x32_bf16, one 16-B chunk (8 k) per MFMA.
//   f32 : v_mfma_f32_16x16x4_f32 (exact fp32, the parity path), one 16-B chunk = 4 MFMAs with a
//         k-permutation shared by both operands.
//
// Kernels.
//   gemm_nt_kernel   128x128 tile, 4 waves (64x64 each), 2 blocks/CU; bf16 and f32.
//   gemm_big_kernel  256x256 tile, 8 waves (128x64 each), 128 KiB LDS, 1 block/CU; bf16, used
//                    when the problem has >= 256 such tiles (every encoder GEMM at bs >= 64).
// Both stage the finished accumulator tile through LDS (fp32, XOR-swizzled 512-B rows) and run
// the epilogue row-major ("epi_rows"): every lane owns 4 consecutive columns of one row and a
// wave streams 2 full 128-column row segments per instruction, so bias / residual / position
// loads, output stores and LayerNorm row statistics are all coalesced.
//
// LayerNorm folding. The reference sublayer is y = LN(x); out = f(y) + y (norm.py:11-12 +
// residual.py:9; the residual is the NORMALISED input). With per-row mean mu, rstd r of x and
// LN(x) = (x - mu) r gamma + beta, the first Dense of the sublayer is
//     y . W = r (x . W') - r mu s + c,   W' = diag(gamma) W,  s = 1^T W',  c = beta . W (+ bias)
// so QKV / FC1 consume the raw stream x and apply (mu, r) per row in the epilogue (EPI_LNIN);
// the residual y is rebuilt element-wise from x in the out-proj / FC2 epilogue (EPI_RESLN), and
// those epilogues accumulate the row sums (sum x, sum x^2) of the new stream for the next
// LayerNorm with one atomic pair per row segment (EPI_STATS). No LayerNorm kernel, no fp32
// stream: the token stream x is kept in the activation dtype.
//
// Grid. 1-D, XCD-aware bijective remap so that consecutive logical tiles (same A rows, all N
// tiles) run on one XCD and share its L2.
#include <type_traits>

#include "common.h"
#include "evt_internal.h"

namespace evt {

namespace {

constexpr int ROWB = 128;                       // bytes of K per row per stage
constexpr int TILE_BYTES = GEMM_BM * ROWB;      // 16 KiB per operand tile
constexpr int STAGE_BYTES = 2 * TILE_BYTES;     // A + W

template <typename T> struct Mma;
template <> struct Mma<bf16> {
  static __device__ __forceinline__ void run(const u32x4& a, const u32x4& b, f32x4& c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};
template <> struct Mma<float> {
  static __device__ __forceinline__ void run(const u32x4& a, const u32x4& b, f32x4& c) {
    const f32x4 af = __builtin_bit_cast(f32x4, a), bf = __builtin_bit_cast(f32x4, b);
#pragma unroll
    for (int e = 0; e < 4; ++e) c = __builtin_amdgcn_mfma_f32_16x16x4f32(af[e], bf[e], c, 0, 0, 0);
  }
};

// Bijective XCD-aware remap: blocks b and b+8 share an XCD (round-robin dispatch), so give each
// XCD a contiguous range of logical tiles (tile order: all N tiles of one M block consecutively,
// so an XCD's L2 keeps the A panel while it sweeps N).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, local = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
}

// Load 4 per-column fp32 values (zero past N).
__device__ __forceinline__ f32x4 col4(const float* v, int n, int N, bool full) {
  if (full) return load4(v + n);
  f32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = (n + j < N) ? v[n + j] : 0.f;
  return r;
}

// LayerNorm coefficients of one row from its per-slab partial statistics
// stats[row][slot][2] = (sum, sumsq), summed over the slots in a fixed order (deterministic).
__device__ __forceinline__ void ln_coef(const float* stats, int nslots, int64_t row, float inv_d,
                                        float eps, float& mu, float& r) {
  const float2* st = (const float2*)(stats + 2 * nslots * row);
  float s1 = 0.f, s2 = 0.f;
  for (int j = 0; j < nslots; ++j) {
    const float2 v = st[j];
    s1 += v.x;
    s2 += v.y;
  }
  mu = s1 * inv_d;
  r = rsqrtf(fmaxf(s2 * inv_d - mu * mu, 0.f) + eps);
}

// Staged-tile addressing: fp32 rows of 512 B (128 columns), 16-B chunk c of row r at
// c ^ (r & 7): conflict-free for the 16-B fragment writes and the row reads.
__device__ __forceinline__ int stg_off(int row, int chunk) { return row * 512 + ((chunk ^ (row & 7)) << 4); }

// Broadcast the value held by lane `l0` (lanes 0-31) or `l0 + 1` (lanes 32-63): per-row
// coefficients of the two rows an iteration covers, with two v_readlane (no LDS traffic).
__device__ __forceinline__ float row_bcast(float v, int l0, int sub) {
  const int a = __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l0);
  const int b = __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l0 + 1);
  return __builtin_bit_cast(float, sub ? b : a);
}

// Row-major epilogue over the 32 staged rows [row_lo, row_lo+32) of one wave (2 rows per
// iteration: lane>>5) of a staged 128-column slab; lane chunk c = lane & 31 holds global columns
// n .. n+3 (n supplied by the caller: the slab need not be contiguous). Per-row LayerNorm
// coefficients are computed once per lane (lane c: row row_lo + c) and broadcast with readlane.
// EPI_STATS: each lane parks its 4-column partial (sum, sumsq) of the stored values in the LDS
// row it has just consumed; at the end every row's 32 partials are summed in a fixed order and
// written to stats slot `slot` of that row (no atomics: bitwise reproducible).
template <typename T, int FL, bool INTERIOR>
__device__ __forceinline__ void epi_rows_t(const GemmParams& p, EVT_LDS char* stg, int m0, int n,
                                           int row_lo, int lane, int slot) {
  typedef typename std::conditional<(FL & EPI_OUT_F32) != 0, float, T>::type TO;
  constexpr bool interior = INTERIOR;  // interior tiles: no per-row / per-column range checks
  const int sub = lane >> 5, c = lane & 31;
  const bool col_ok = interior || n < p.N;
  const bool full = interior || (p.vec_ok && n + 4 <= p.N);
  f32x4 bias4 = f32x4{0.f, 0.f, 0.f, 0.f}, cs4 = bias4, g4 = bias4, b4 = bias4;
  if (col_ok) {
    if (FL & EPI_BIAS) bias4 = col4(p.bias, n, p.N, full);
    if (FL & EPI_LNIN) cs4 = col4(p.colsum, n, p.N, full);
    if (FL & EPI_RESLN) {
      g4 = col4(p.rgamma, n, p.N, full);
      b4 = col4(p.rbeta, n, p.N, full);
    }
  }
  // per-row LayerNorm coefficients: lane c (both halves) owns row row_lo + c
  float in_mu = 0.f, in_r = 0.f, rs_mu = 0.f, rs_r = 0.f;
  if (FL & (EPI_LNIN | EPI_RESLN)) {
    const int mr = m0 + row_lo + c;
    if (interior || mr < p.M) {
      if (FL & EPI_LNIN)
        ln_coef(p.stats_in, p.nslots, (int64_t)mr * (p.stats_step > 1 ? p.stats_step : 1), p.inv_d,
                p.eps, in_mu, in_r);
      if (FL & EPI_RESLN) ln_coef(p.rstats, p.nslots, mr, p.inv_d, p.eps, rs_mu, rs_r);
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    // two groups of 8 iterations: bounds how many loads the scheduler hoists (VGPR pressure)
    if (i == 8) __builtin_amdgcn_sched_barrier(0);
    const int row = row_lo + 2 * i + sub;
    const int m = m0 + row;
    const bool ok = col_ok && (interior || m < p.M);
    f32x4 v = *(const EVT_LDS f32x4*)(stg + stg_off(row, c));
    int64_t orow = m;
    if (FL & EPI_LNIN) {
      const float mu = row_bcast(in_mu, 2 * i, sub), r = row_bcast(in_r, 2 * i, sub);
      v = v * r - cs4 * (r * mu) + bias4;
    } else if (FL & EPI_BIAS) {
      v += bias4;
    }
    if (FL & (EPI_GELU | EPI_GELU_ERF))
      v = gelu4(v, (FL & EPI_GELU) ? 0 : std::is_same<T, bf16>::value ? 2 : 1);
    if (FL & EPI_POS) {
      const int img = m / p.P, t = m - img * p.P;
      orow = (int64_t)img * (p.P + 1) + 1 + t;
      if (ok) v += col4(p.pos + (int64_t)(t + 1) * p.ldp, n, p.N, full);
    }
    if (FL & EPI_RESID) {
      f32x4 rv = f32x4{0.f, 0.f, 0.f, 0.f};
      if (ok) {
        const T* rp = (const T*)p.resid + (int64_t)m * p.ldr + n;
        if (full) rv = load4(rp);
        else
          for (int j = 0; j < 4; ++j) rv[j] = (n + j < p.N) ? to_f32(rp[j]) : 0.f;
      }
      if (FL & EPI_RESLN) {
        const float mu = row_bcast(rs_mu, 2 * i, sub), r = row_bcast(rs_r, 2 * i, sub);
        rv = (rv - mu) * r * g4 + b4;
      }
      v += rv;
    }
    if (ok) {
      TO* cp = (TO*)p.C + orow * p.ldc + n;
      if (full) store4_nt(cp, v);
      else
        for (int j = 0; j < 4; ++j)
          if (n + j < p.N) cp[j] = from_f32<TO>(v[j]);
    }
    if (FL & EPI_STATS) {
      // partial statistics of the values as stored (what the next LayerNorm reads), parked in
      // the first 512 B of row row_lo + 2i, which both half-waves have already read
      float s1 = 0.f, s2 = 0.f;
      if (ok) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float q = (full || n + j < p.N) ? to_f32(from_f32<TO>(v[j])) : 0.f;
          s1 += q;
          s2 += q * q;
        }
      }
      *(EVT_LDS f32x2*)(stg + (row_lo + 2 * i) * 512 + sub * 256 + c * 8) = f32x2{s1, s2};
    }
  }
  if (FL & EPI_STATS) {
    // lane (q = lane & 31, hf = lane >> 5): row row_lo + q, partials [16 hf, 16 hf + 16)
    const int q = lane & 31, hf = lane >> 5;
    const EVT_LDS char* src = stg + (row_lo + (q & ~1)) * 512 + (q & 1) * 256 + hf * 128;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4 v = *(const EVT_LDS f32x4*)(src + j * 16);
      s1 += v[0] + v[2];
      s2 += v[1] + v[3];
    }
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 32, 64);
    const int m = m0 + row_lo + q;
    if (hf == 0 && (interior || m < p.M)) {
      int64_t orow = m;
      if (FL & EPI_POS) {
        const int img = m / p.P, t = m - img * p.P;
        orow = (int64_t)img * (p.P + 1) + 1 + t;
      }
      *(f32x2*)(p.stats_out + 2 * (p.nslots * orow + slot)) = f32x2{s1, s2};
    }
  }
}

// bf16-output form of epi_rows: every lane owns 8 consecutive columns (two staged chunks) of one
// row, 4 rows per iteration, so each output store is 16 B per lane (dwordx4). Measured: the
// 8-B-store epilogue is store-issue bound (writing fp32 with 16-B stores was faster than bf16
// with 8-B stores). Per-row coefficients come from lane (4i + q) via ds_bpermute; statistics
// partials (16 per row) are parked in the row just consumed and summed in a fixed order.
// Requires p.vec_ok >= 2 (ldc, ldr, ldp multiples of 8); n = first of the lane's 8 columns.
template <int FL, bool INTERIOR>
__device__ __forceinline__ void epi_rows8_t(const GemmParams& p, EVT_LDS char* stg, int m0, int n,
                                            int row_lo, int lane, int slot) {
  constexpr bool interior = INTERIOR;
  const int q = lane >> 4, c8 = lane & 15;
  const bool col_ok = interior || n < p.N;
  const bool full = interior || n + 8 <= p.N;
  f32x4 bias4[2], cs4[2], g4[2], b4[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    bias4[h] = cs4[h] = g4[h] = b4[h] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool fh = interior || n + 4 * h + 4 <= p.N;
    if (col_ok) {
      if (FL & EPI_BIAS) bias4[h] = col4(p.bias, n + 4 * h, p.N, fh);
      if (FL & EPI_LNIN) cs4[h] = col4(p.colsum, n + 4 * h, p.N, fh);
      if (FL & EPI_RESLN) {
        g4[h] = col4(p.rgamma, n + 4 * h, p.N, fh);
        b4[h] = col4(p.rbeta, n + 4 * h, p.N, fh);
      }
    }
  }
  float in_mu = 0.f, in_r = 0.f, rs_mu = 0.f, rs_r = 0.f;  // lane c: row row_lo + (c & 31)
  if (FL & (EPI_LNIN | EPI_RESLN)) {
    const int mr = m0 + row_lo + (lane & 31);
    if (interior || mr < p.M) {
      if (FL & EPI_LNIN)
        ln_coef(p.stats_in, p.nslots, (int64_t)mr * (p.stats_step > 1 ? p.stats_step : 1), p.inv_d,
                p.eps, in_mu, in_r);
      if (FL & EPI_RESLN) ln_coef(p.rstats, p.nslots, mr, p.inv_d, p.eps, rs_mu, rs_r);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    // bound how many iterations' loads the scheduler hoists (VGPR pressure: the other half of
    // the accumulators is still live in pass 0)
    if ((FL & EPI_RESID) ? (i & 1) == 0 && i > 0 : i == 4) __builtin_amdgcn_sched_barrier(0);
    const int row = row_lo + 4 * i + q;
    const int m = m0 + row;
    const bool ok = col_ok && (interior || m < p.M);
    const int src = (4 * i + q) * 4;  // ds_bpermute byte index of the lane holding this row
    f32x4 v[2];
    v[0] = *(const EVT_LDS f32x4*)(stg + stg_off(row, 2 * c8));
    v[1] = *(const EVT_LDS f32x4*)(stg + stg_off(row, 2 * c8 + 1));
    int64_t orow = m;
    if (FL & EPI_LNIN) {
      const float mu = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, in_mu)));
      const float r = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, in_r)));
#pragma unroll
      for (int h = 0; h < 2; ++h) v[h] = v[h] * r - cs4[h] * (r * mu) + bias4[h];
    } else if (FL & EPI_BIAS) {
      v[0] += bias4[0];
      v[1] += bias4[1];
    }
    if (FL & (EPI_GELU | EPI_GELU_ERF)) {
#pragma unroll
      for (int h = 0; h < 2; ++h) v[h] = gelu4(v[h], (FL & EPI_GELU) ? 0 : 2);  // bf16 only
    }
    if (FL & EPI_POS) {
      const int img = m / p.P, t = m - img * p.P;
      orow = (int64_t)img * (p.P + 1) + 1 + t;
      if (ok) {
        const float* pr = p.pos + (int64_t)(t + 1) * p.ldp;
        v[0] += col4(pr, n, p.N, interior || n + 4 <= p.N);
        v[1] += col4(pr, n + 4, p.N, full);
      }
    }
    if (FL & EPI_RESID) {
      f32x4 rv[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      if (ok) {
        const bf16* rp = (const bf16*)p.resid + (int64_t)m * p.ldr + n;
        if (full) {
          const bf16x8 r8 = __builtin_bit_cast(bf16x8, *(const u32x4*)rp);
          rv[0] = f32x4{(float)r8[0], (float)r8[1], (float)r8[2], (float)r8[3]};
          rv[1] = f32x4{(float)r8[4], (float)r8[5], (float)r8[6], (float)r8[7]};
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (n + j < p.N) rv[j >> 2][j & 3] = to_f32(rp[j]);
        }
      }
      if (FL & EPI_RESLN) {
        const float mu = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, rs_mu)));
        const float r = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, rs_r)));
#pragma unroll
        for (int h = 0; h < 2; ++h) rv[h] = (rv[h] - mu) * r * g4[h] + b4[h];
      }
      v[0] += rv[0];
      v[1] += rv[1];
    }
    const bf16x8 o = {(bf16)v[0][0], (bf16)v[0][1], (bf16)v[0][2], (bf16)v[0][3],
                      (bf16)v[1][0], (bf16)v[1][1], (bf16)v[1][2], (bf16)v[1][3]};
    if (ok) {
      bf16* cp = (bf16*)p.C + orow * p.ldc + n;
      if (full) store_b128_nt(cp, __builtin_bit_cast(u32x4, o));
      else
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (n + j < p.N) cp[j] = o[j];
    }
    if (FL & EPI_STATS) {
      float s1 = 0.f, s2 = 0.f;
      if (ok) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x = (full || n + j < p.N) ? (float)o[j] : 0.f;
          s1 += x;
          s2 += x * x;
        }
      }
      // park in row `row` (read above by these same lanes): partial c8 at byte c8 * 8
      *(EVT_LDS f32x2*)(stg + row * 512 + c8 * 8) = f32x2{s1, s2};
    }
  }
  if (FL & EPI_STATS) {
    // lane (r = lane & 31, hf = lane >> 5): row row_lo + r, partials [8 hf, 8 hf + 8)
    const int r = lane & 31, hf = lane >> 5;
    const EVT_LDS char* src = stg + (row_lo + r) * 512 + hf * 64;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 v = *(const EVT_LDS f32x4*)(src + j * 16);
      s1 += v[0] + v[2];
      s2 += v[1] + v[3];
    }
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 32, 64);
    const int m = m0 + row_lo + r;
    if (hf == 0 && (interior || m < p.M)) {
      int64_t orow = m;
      if (FL & EPI_POS) {
        const int img = m / p.P, t = m - img * p.P;
        orow = (int64_t)img * (p.P + 1) + 1 + t;
      }
      *(f32x2*)(p.stats_out + 2 * (p.nslots * orow + slot)) = f32x2{s1, s2};
    }
  }
}

// n4: first column of the lane in the 4-column layout (lane chunk c = lane & 31);
// n8: first column in the 8-column layout (lane chunks 2 (lane & 15), +1).
// ONLY8: the caller guarantees p.vec_ok >= 2 (the 256x256 kernel), so only the 8-column form is
// compiled in (the dead 4-column form otherwise costs registers: hoisted addresses spill).
template <typename T, int FL, bool ONLY8 = false>
__device__ __forceinline__ void epi_rows(const GemmParams& p, EVT_LDS char* stg, int m0, int n4,
                                         int n8, int row_lo, int lane, int slot, bool interior) {
  constexpr bool out16 = std::is_same<T, bf16>::value && !(FL & EPI_OUT_F32);
  if (out16 && (ONLY8 || p.vec_ok >= 2)) {
    if (interior) epi_rows8_t<FL, true>(p, stg, m0, n8, row_lo, lane, slot);
    else epi_rows8_t<FL, false>(p, stg, m0, n8, row_lo, lane, slot);
    return;
  }
  if constexpr (!(out16 && ONLY8)) {
    if (interior) epi_rows_t<T, FL, true>(p, stg, m0, n4, row_lo, lane, slot);
    else epi_rows_t<T, FL, false>(p, stg, m0, n4, row_lo, lane, slot);
  }
}

// ---------------------------------------------------------------------------------------------
// 128x128 tile kernel (bf16 and f32): 256 threads = 4 waves in 2 (m) x 2 (n), 64x64 per wave,
// 2-stage glds double buffer (64 KiB), two blocks per CU.
// ---------------------------------------------------------------------------------------------
template <typename T, int FL>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];
  if (gridDim.y > 1) {  // split-K (gemm_splitk_launch): this block's K range and partial C
    const int z = blockIdx.y;
    p.A = (const T*)p.A + (int64_t)z * p.ks_chunk;
    p.W = (const T*)p.W + (int64_t)z * p.ks_chunk;
    p.K = p.ks_chunk;
    p.C = (float*)p.C + (int64_t)z * p.ks_stride;
  }

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably uniform -> SGPR math
  const int wm = wave & 1, wn = wave >> 1;
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = wgid / p.ntiles, tn = wgid - tm * p.ntiles;
  const int m0 = tm * GEMM_BM, n0 = tn * GEMM_BN;

  // ---- staging: wave stages rows [wave*32, wave*32+32) of both tiles ----
  const int srow = lane >> 3, sslot = lane & 7;
  const int64_t lda_b = p.lda * (int64_t)sizeof(T), ldw_b = p.ldw * (int64_t)sizeof(T);
  const int arow0 = m0 + wave * 32 + srow;
  const char* a_base = (const char*)p.A + ((sslot ^ srow) * 16);
  const char* w_base = (const char*)p.W + (int64_t)(n0 + wave * 32 + srow) * ldw_b + ((sslot ^ srow) * 16);
  auto stage = [&](int kt, int buf) {
    EVT_LDS char* base = (EVT_LDS char*)smem + buf * STAGE_BYTES;
    const int64_t koff = (int64_t)kt * ROWB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gm = min(arow0 + i * 8, p.M - 1);
      glds16(a_base + gm * lda_b + koff, base + (wave * 32 + i * 8) * ROWB);
      glds16(w_base + (i * 8) * ldw_b + koff, base + TILE_BYTES + (wave * 32 + i * 8) * ROWB);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K * (int)sizeof(T) / ROWB;
  stage(0, 0);
  const int frow = lane & 15, fsw = lane & 7, fg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    wait_vmcnt0();
    __syncthreads();
    if (kt + 1 < nk) stage(kt + 1, (kt + 1) & 1);
    const EVT_LDS char* As = (const EVT_LDS char*)smem + (kt & 1) * STAGE_BYTES;
    const EVT_LDS char* Ws = As + TILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int coff = ((fg + 4 * kk) ^ fsw) * 16;
      u32x4 a[4], w[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        a[mt] = *(const EVT_LDS u32x4*)(As + (wm * 64 + mt * 16 + frow) * ROWB + coff);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        w[nt] = *(const EVT_LDS u32x4*)(Ws + (wn * 64 + nt * 16 + frow) * ROWB + coff);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) Mma<T>::run(w[nt], a[mt], acc[nt][mt]);
    }
  }

  // ---- stage the 128x128 fp32 tile (exactly the 64 KiB of LDS), then row-major epilogue ----
  __syncthreads();
  EVT_LDS char* stg = (EVT_LDS char*)smem;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int row = wm * 64 + mt * 16 + frow;
      *(EVT_LDS f32x4*)(stg + stg_off(row, wn * 16 + nt * 4 + fg)) = acc[nt][mt];
    }
  __syncthreads();
  const bool interior = p.vec_ok && (n0 + GEMM_BN <= p.N) && (m0 + GEMM_BM <= p.M);
  epi_rows<T, FL>(p, stg, m0, n0 + (lane & 31) * 4, n0 + (lane & 15) * 8, wave * 32, lane,
                  n0 / 128, interior);
}

// ---------------------------------------------------------------------------------------------
// Large-tile bf16 kernel: 256x256 output tile, BK = 64, 512 threads = 8 waves in 2 (m) x 4 (n),
// each wave a 128 (m) x 64 (n) sub-tile = 8 x 4 MFMA tiles (128 fp32 accumulators per lane).
// 128 KiB LDS (2 buffers x {A 32 KiB, W 32 KiB}), one block per CU; one barrier per K-tile.
// VAR 6 (default): after the barrier, k-step-0 fragments are read, the 8 DMA pieces of the next
// K-tile are spread between the first 16 MFMAs and the k-step-1 reads between the next 12
// (sched_group_barrier), so the DMA issue and LDS latency hide under MFMA issue.
// VAR 0: the same without the explicit issue order (kept for A/B measurements).
// ---------------------------------------------------------------------------------------------
constexpr int BIG_BM = 256, BIG_BN = 256;
constexpr int BIG_TILE = BIG_BM * ROWB;       // 32 KiB per operand
constexpr int BIG_STAGE = 2 * BIG_TILE;       // 64 KiB per K-tile

// evt_set_gemm_variant, per calling thread (launch decisions are made on the launching thread):
// 0 auto, 1 force 128x128, 2 / 6 / 8 non-persistent 256x256 main loops, 9 tile-persistent,
// 16 stream-K, 30 128 x 384 persistent wherever it applies, 31 automatic without it. Lab builds
// (-DEVT_GEMM_LAB) add the ablation / timeline / A-B variants 10, 11, 13, 15, 17-25, 106, 108 used
// by scripts/gemm_bench.py and scripts/probe/pers_timeline.py. (Round-4 main-loop experiments
// measured slower - B-fragment prefetch, buffer-descriptor loader, residual in the main loop,
// residual L2 prefetch, phase-level lgkmcnt waits, DMA-first phases, MFMA priority - were removed
// in round 5; DESIGN.md records them and git history holds the code.)
thread_local int g_gemm_variant = 0;

int num_cus();

// The big kernels address inside a tile with 32-bit offsets: the LDS-DMA lane offsets (glds16s,
// unsigned, up to 384 rows of lda / ldw) and the epilogue's buffer-descriptor ranges (signed, up
// to 256 rows of ldc / ldr). Leading dimensions past that take the 128 x 128 kernel.
constexpr int64_t BIG_MAX_LD = ((int64_t)1 << 31) / (2 * 384) - 64;

bool use_big(const GemmParams& p, int flags) {
  if ((p.ntiles * GEMM_BN) % BIG_BN) return false;
  if (std::max(std::max(p.lda, p.ldw), std::max(p.ldc, p.resid ? p.ldr : (int64_t)0)) > BIG_MAX_LD)
    return false;
  if (!(flags & EPI_OUT_F32) && p.vec_ok < 2) return false;  // big epilogue: 16-B bf16 stores only
  // 31: automatic without 128 x 384, 36: automatic without grid balancing (launch_pers)
  const int v = (g_gemm_variant == 31 || g_gemm_variant == 36) ? 0 : g_gemm_variant;
  if (v == 1) return false;
  if (v >= 2) return true;
  // 256x256 tiles unless their rounds cost more: time in 256-tile units, the 128x128 kernel at a
  // quarter of the work per tile and about half the FLOP rate (measured at 64 images: FC2 107 us
  // on 594 128x128 tiles against ~80 us for one round of 150 256x256 tiles); tiny problems (the
  // bs1 forward) keep the small tiles
  const int64_t G = num_cus();
  const int64_t t256 = (int64_t)((p.M + 255) / 256) * (p.ntiles * GEMM_BN / 256);
  const int64_t t128 = (int64_t)((p.M + 127) / 128) * p.ntiles;
  return (t256 + G - 1) / G <= 0.5 * (double)((t128 + G - 1) / G);
}

// Epilogue of the 256x256 kernels: two passes staged through the (idle) 128 KiB of LDS; in
// pass h every wave hands over its column tiles nt = 2h, 2h+1 (half of its accumulators die per
// pass) and all 8 waves then stream 32 rows each of the staged 256 x 128 slab. Stats slot of
// pass h: 2*tn + h. The wave's 128 x 64 sub-tile is rows wm*128.., columns wn*64...
template <int FL>
__device__ __forceinline__ void big_epilogue(const GemmParams& p, char* smem, f32x4 (&acc)[4][8],
                                             int wm, int wn, int m0, int n0, int tn, int wave,
                                             int lane) {
  EVT_LDS char* stg = (EVT_LDS char*)smem;
  const bool interior = p.vec_ok && (n0 + BIG_BN <= p.N) && (m0 + BIG_BM <= p.M);
  const int c = lane & 31, frow = lane & 15, fg = lane >> 4;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __builtin_amdgcn_s_barrier();  // previous readers of the staging area are done
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        const int row = wm * 128 + mt * 16 + frow;
        *(EVT_LDS f32x4*)(stg + stg_off(row, wn * 8 + t * 4 + fg)) = acc[2 * h + t][mt];
      }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    // staged chunk c holds global columns n0 + (c>>3)*64 + h*32 + (c&7)*4 .. +3
    // (8-column layout: lane chunks 2 c8, 2 c8 + 1 -> n0 + (c8>>2)*64 + h*32 + (c8&3)*8 .. +7)
    const int c8 = lane & 15;
    epi_rows<bf16, FL, true>(p, stg, m0, n0 + (c >> 3) * 64 + h * 32 + (c & 7) * 4,
                       n0 + (c8 >> 2) * 64 + h * 32 + (c8 & 3) * 8, wave * 32, lane, 2 * tn + h,
                       interior);
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
}


// ---------------------------------------------------------------------------------------------
// 8-phase ping-pong main loop (VAR 8 of gemm_big_kernel, and gemm_pers_kernel).
// Four phases per K-tile. Each K-tile buffer is split into four 16 KiB regions: j = 0 A rows of
// m-half 0 (of both wm), 1 W rows of n-half 0 (of all wn), 2 W n-half 1, 3 A m-half 1, read in
// phases 1 / 1 / 2 / 3 of the tile (the wave's 128 x 64 sub-tile is done as four 64 x 32
// quadrants, B n-half 0 stays in registers for the 4th). Region s = 4 T + j is DMA'd (2 glds
// per lane) in global phase s - 6, i.e. into the buffer still being read, two or more phases
// after the region's last read (WAR), and retired by a counted vmcnt before the first barrier
// of the phase preceding its first read (RAW): every DMA gets about one K-tile of flight time
// and 8 glds per lane stay in flight. Wave group wm = 1 runs one barrier behind group 0, so
// while one group issues MFMAs (at raised priority) the other issues ds_reads and DMAs on the
// same SIMD (waves w and w + 4 share a SIMD).
// ---------------------------------------------------------------------------------------------
struct NoOp {
  __device__ void operator()() const {}
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void big8_bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}

// Params types of the EPI_GATHER / EPI_SPLIT instantiations: the A loader gathers (the type
// selects the loader at compile time; every other GEMM keeps the plain one): Swin PatchMerging
// (gmode 1) / the T2T soft split (gmode 2).
struct MergeParams : GemmParams {};
struct UnfoldParams : GemmParams {};
// 128 x 384 tiles (gemm_p384_kernel): the params type selects the tile geometry at compile time
struct P384Params : GemmParams {};

// Tile geometry of the 8-phase main loop by params type: BM x BN block tile, 8 waves as 2 (wm) x 4
// (wn), each wave (BM / 2) x (BN / 4) = MF x NF fragments of 16 x 16. The K-tile's LDS stage is
// A (BM rows) then W (BN rows) of 128 B, 64 KiB for both geometries; its four DMA regions are the
// A m-halves (AI instructions per wave) and the W n-halves (WI per wave), AI + WI = 4.
template <typename P>
struct GeoOf {
  static constexpr int BM = 256, BN = 256, MF = 8, NF = 4;
};
template <>
struct GeoOf<P384Params> {
  static constexpr int BM = 128, BN = 384, MF = 4, NF = 6;
};
template <typename P>
struct Geo : GeoOf<P> {
  using G = GeoOf<P>;
  static constexpr int WR = G::BM / 2, WC = G::BN / 4;  // wave tile rows / columns
  static constexpr int MH = G::MF / 2, NH = G::NF / 2;  // fragments per m-half / n-half
  static constexpr int A_TILE = G::BM * ROWB;
  static constexpr int AI = G::BM / 128, WI = G::BN / 128;  // DMA instructions per wave per region
  static_assert(A_TILE + G::BN * ROWB == BIG_STAGE && AI + WI == 4, "64 KiB K-tile stages");
};

// EPI_GATHER A address (Swin PatchMerging, reference SwinTransformer PatchMerging.forward:
// x0 | x1 | x2 | x3 = x[0::2, 0::2] | x[1::2, 0::2] | x[0::2, 1::2] | x[1::2, 1::2]): GEMM row gm
// is token (b, y, x) of the R/2 grid, element k = q C + c is channel c of source token
// (2y + (q & 1), 2x + (q >> 1)) of the R-grid stream. Divisions by float reciprocals (exact for
// gm < 2^22 with the half-unit offset, as pos_img).
// gmode 2 (T2T soft_split1, tf_Unfold k 3 s 2 p 1 of the 64-channel token map, t2t_vit.py:72):
// element k = (3 kh + kw) 64 + c is channel c of source token (2y - 1 + kh, 2x - 1 + kw), or of a
// zero row outside the map.
template <int MODE>
__device__ __forceinline__ const char* gather_addr(const GemmParams& p, int gm, int k) {
  const int OW = p.gOW;
  const int b = (int)(((float)gm + 0.5f) * p.g_inv_rr);
  const int r = gm - b * OW * OW;
  const int y = (int)(((float)r + 0.5f) * p.g_inv_r);
  const int x = r - y * OW;
  if constexpr (MODE == 2) {
    const int win = k >> 6, c = k & 63;
    const int kh = (win * 11) >> 5, kw = win - 3 * kh;  // win / 3 for win < 9
    const int iy = 2 * y - 1 + kh, ix = 2 * x - 1 + kw;
    if (iy < 0 || iy >= p.gR || ix < 0 || ix >= p.gR) return (const char*)p.gzero + c * 2;
    const int64_t src = ((int64_t)b * p.gR + iy) * p.gR + ix;
    return (const char*)p.A + (src * p.lda + c) * 2;
  }
  const int q = (k >= p.gC) + (k >= 2 * p.gC) + (k >= 3 * p.gC);
  const int c = k - q * p.gC;
  const int64_t src = ((int64_t)b * p.gR + 2 * y + (q & 1)) * p.gR + 2 * x + (q >> 1);
  return (const char*)p.A + (src * p.lda + c) * 2;
}

// DMA region j of K-tile T into buffer (T ^ par) & 1 (par: the buffer parity of the tile's
// K-tile 0; persistent kernel with an odd K-tile count: alternates from tile to tile).
template <typename P>
__device__ __forceinline__ void big8_stage(const P& p, char* smem, int wave, int lane,
                                           int m0, int n0, int T, int j, int par = 0) {
  typedef Geo<P> Gm;
  const int srow = lane >> 3, sslot = lane & 7;
  EVT_LDS char* base = (EVT_LDS char*)smem + ((T ^ par) & 1) * BIG_STAGE;
#ifdef EVT_ABL_KT0  // lab ablation: every K-tile DMAs K-tile 0's bytes (cache-resident; wrong results)
  const int Tg = 0;
#else
  const int Tg = T;
#endif
  const int64_t koff = (int64_t)T * ROWB + ((sslot ^ srow) << 4);
  if constexpr (Gm::BM != 256) {
    // general geometry: a K-tile's 8 DMA instructions per wave in the region order of the 256 x 256
    // one (A m-half 0, W n-half 0, W n-half 1, A m-half 1: AI, WI, WI, AI instructions), issued
    // two per phase: "j" is the pair (0, 1: the first half of that order, 2, 3: the second), so
    // unequal regions (1 + 3 + 3 + 1 for 128 x 384) still spread evenly over the phases
    auto a_ins = [&](int h, int i) {  // A m-half h, instruction i of AI: rows wm*WR + h*WR/2 + ..
      const int g = wave * Gm::AI + i, gpw = Gm::WR / 16;
      const int row = (g / gpw) * Gm::WR + h * (Gm::WR / 2) + (g % gpw) * 8;
      const int gm = min(m0 + row + srow, p.M - 1);
      glds16s((const char*)p.A + (int64_t)m0 * (p.lda * 2) + Tg * ROWB,
              (uint32_t)((gm - m0) * (p.lda * 2)) + ((sslot ^ srow) << 4), base + row * ROWB);
    };
    auto w_ins = [&](int h, int i) {  // W n-half h, instruction i of WI: rows wn*WC + h*WC/2 + ..
      const int g = wave * Gm::WI + i, gpw = Gm::WC / 16;
      const int row = (g / gpw) * Gm::WC + h * (Gm::WC / 2) + (g % gpw) * 8;
      glds16s((const char*)p.W + (int64_t)n0 * (p.ldw * 2) + Tg * ROWB,
              (uint32_t)((row + srow) * (p.ldw * 2)) + ((sslot ^ srow) << 4),
              base + Gm::A_TILE + row * ROWB);
    };
    auto ins = [&](int q) {  // instruction q (0..7) of the K-tile's sequence
      if (q < Gm::AI) a_ins(0, q);
      else if (q < Gm::AI + Gm::WI) w_ins(0, q - Gm::AI);
      else if (q < Gm::AI + 2 * Gm::WI) w_ins(1, q - Gm::AI - Gm::WI);
      else a_ins(1, q - Gm::AI - 2 * Gm::WI);
    };
    ins(2 * j);
    ins(2 * j + 1);
    return;
  }
#ifndef EVT_GLDS_UNPAIRED
  if constexpr (!std::is_same<P, MergeParams>::value && !std::is_same<P, UnfoldParams>::value) {
    // the wave's two pieces of the region are 8 rows = 1 KiB apart in LDS: one M0 for both, the
    // second at instruction offset 1024 (applied to the LDS and the global address alike; the
    // SGPR base moves down 1 KiB so that no lane offset goes negative)
    const int r = wave * 16;
    const uint32_t swz = (uint32_t)((sslot ^ srow) << 4);
    if (j == 0 || j == 3) {
      const int row = (r & 63) + ((r >> 6) << 7) + (j == 3 ? 64 : 0);
      const int gm0 = min(m0 + row + srow, p.M - 1), gm1 = min(m0 + row + 8 + srow, p.M - 1);
      glds16s_pair(((const char*)p.A - 1024 + (int64_t)m0 * (p.lda * 2)) + Tg * ROWB,
                   (uint32_t)((gm0 - m0) * (p.lda * 2)) + swz + 1024,
                   (uint32_t)((gm1 - m0) * (p.lda * 2)) + swz, base + row * ROWB);
    } else {
      const int row = ((r >> 5) << 6) + (r & 31) + (j == 2 ? 32 : 0);
      glds16s_pair(((const char*)p.W - 1024 + (int64_t)n0 * (p.ldw * 2)) + Tg * ROWB,
                   (uint32_t)((row + srow) * (p.ldw * 2)) + swz + 1024,
                   (uint32_t)((row + 8 + srow) * (p.ldw * 2)) + swz,
                   base + BIG_TILE + row * ROWB);
    }
    return;
  }
#endif
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (wave * 2 + i) * 8;  // region row of this wave-instruction (8 rows)
    if (j == 0 || j == 3) {
      const int row = (r & 63) + ((r >> 6) << 7) + (j == 3 ? 64 : 0);
      const int gm = min(m0 + row + srow, p.M - 1);
      if constexpr (std::is_same<P, MergeParams>::value)
        glds16(gather_addr<1>(p, gm, T * 64 + ((sslot ^ srow) << 3)), base + row * ROWB);
      else if constexpr (std::is_same<P, UnfoldParams>::value)
        glds16(gather_addr<2>(p, gm, T * 64 + ((sslot ^ srow) << 3)), base + row * ROWB);
      else  // SGPR base = the tile's first row at K-tile T, 32-bit lane offsets (glds16s)
        glds16s((const char*)p.A + (int64_t)m0 * (p.lda * 2) + Tg * ROWB,
                (uint32_t)((gm - m0) * (p.lda * 2)) + ((sslot ^ srow) << 4), base + row * ROWB);
    } else {
      const int row = ((r >> 5) << 6) + (r & 31) + (j == 2 ? 32 : 0);
      glds16s((const char*)p.W + (int64_t)n0 * (p.ldw * 2) + Tg * ROWB,
              (uint32_t)((row + srow) * (p.ldw * 2)) + ((sslot ^ srow) << 4),
              base + BIG_TILE + row * ROWB);
    }
  }
}

__device__ __forceinline__ int big8_npro(int nk) { return min(6, 4 * nk); }

template <typename P>
__device__ __forceinline__ void big8_prologue(const P& p, char* smem, int wave, int lane,
                                              int m0, int n0, int nk, int par = 0) {
  // regions s = 0..5 (tile 0, then regions 0 / 1 of tile 1); only 0..3 when nk == 1
#pragma unroll
  for (int s = 0; s < 4; ++s) big8_stage(p, smem, wave, lane, m0, n0, 0, s, par);
  if (nk >= 2) {
    big8_stage(p, smem, wave, lane, m0, n0, 1, 0, par);
    big8_stage(p, smem, wave, lane, m0, n0, 1, 1, par);
  }
}

// One K-tile. MODE 0 steady (all DMAs, waits 8), 1 second-to-last tile, 2 last tile. X is
// added to every wait of the tile: the number of VMEM instructions each wave is known to have
// issued after the prologue DMAs (gemm_pers_kernel's epilogue stores; first K-tile only).
// cont (persistent kernel, even nk): the last 1.5 K-tiles' DMA slots, idle otherwise, carry the
// NEXT tile's prologue (its K-tiles 0 and 1 are this tile's K-tiles nk and nk + 1 of one continuous
// stream: same buffers, same WAR distances, the steady-state waits), at (nm0, nn0).
// OPEN (last K-tile of a persistent-kernel tile): wave group 1 skips the barrier that closes its
// final MFMA phase and group 0 the resync barrier after the loop, so group 0 starts its epilogue
// while group 1 still issues its last 16 MFMAs (the two barriers cancel in every wave's count).
// ph3: issues X3 further VMEM loads at the start of phase 3 (added to that phase's wait).
template <int MODE, int X, bool OPEN = false, int X3 = 0, typename Ph3 = NoOp,
          typename P = GemmParams>
__device__ __forceinline__ void big8_ktile(const P& p, char* smem,
                                           f32x4 (&acc)[GeoOf<P>::NF][GeoOf<P>::MF],
                                           int wave, int lane, int wm, int wn, int m0, int n0,
                                           int t, bool cont = false, int nm0 = 0, int nn0 = 0,
                                           Ph3 ph3 = {}, int par = 0, int npar = 0) {
  typedef Geo<P> Gm;
  constexpr int MH = Gm::MH, NH = Gm::NH;
  const int frow = lane & 15, fsw = lane & 7, fg = lane >> 4;
  const EVT_LDS char* As = (const EVT_LDS char*)smem + ((t ^ par) & 1) * BIG_STAGE;
  const EVT_LDS char* Ws = As + Gm::A_TILE;
  auto rd = [&](const EVT_LDS char* S, int row, int ks) {
    return *(const EVT_LDS u32x4*)(S + row * ROWB + (((fg + 4 * ks) ^ fsw) << 4));
  };
  u32x4 af[MH][2], bf0[NH][2], bf1[NH][2];
#pragma unroll
  for (int ph = 0; ph < 4; ++ph) {
    // the phase's fragment reads, then its DMA issue (the DMA regions are >= 2 phases from any
    // read here; issuing the DMA first measured 0.7 % slower, round 3)
    if (ph == 0) {
#pragma unroll
      for (int nt = 0; nt < NH; ++nt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) bf0[nt][ks] = rd(Ws, wn * Gm::WC + nt * 16 + frow, ks);
#pragma unroll
      for (int mt = 0; mt < MH; ++mt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) af[mt][ks] = rd(As, wm * Gm::WR + mt * 16 + frow, ks);
    } else if (ph == 1) {
#pragma unroll
      for (int nt = 0; nt < NH; ++nt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          bf1[nt][ks] = rd(Ws, wn * Gm::WC + Gm::WC / 2 + nt * 16 + frow, ks);
    } else if (ph == 2) {
#pragma unroll
      for (int mt = 0; mt < MH; ++mt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          af[mt][ks] = rd(As, wm * Gm::WR + Gm::WR / 2 + mt * 16 + frow, ks);
    }
    if (ph == 3) ph3();
    // DMA of region s = 4 t + ph + 6
    if (MODE == 0 || (MODE == 1 && ph < 2)) {
      if (ph < 2) big8_stage(p, smem, wave, lane, m0, n0, t + 1, ph + 2, par);
      else big8_stage(p, smem, wave, lane, m0, n0, t + 2, ph - 2, par);
    } else if (cont) {  // MODE 1 phases 2, 3 and MODE 2: the next tile's regions, in order
      const int s6 = (MODE == 1 ? ph - 2 : ph + 2);  // 0..5: (K-tile 0, regions 0-3), (1, 0-1)
      big8_stage(p, smem, wave, lane, nm0, nn0, s6 >> 2, s6 & 3, npar);
    }
    // retire what the next phase reads (phases 4, 1, 2 precede reading phases). W0: after phase 0
    // the W n-half-1 region must have landed; its last instruction is followed by 8 younger ones
    // in the 256 x 256 order, by 7 in the paired order of the 128 x 384 geometry (big8_stage)
    constexpr int W0 = Gm::WI == 3 ? 7 : 8;
    if (ph != 2) {
      if (MODE == 0 || cont) {  // (cont: the steady-state DMA pattern continues)
        if (ph == 3) wait_vm<8 + X + X3>();
        else if (ph == 0) wait_vm<W0 + X>();
        else wait_vm<8 + X>();
      } else if (MODE == 1) {
        if (ph == 3) wait_vm<4 + X>();
        else if (ph == 0) wait_vm<W0 + X>();
        else wait_vm<8 + X>();
      } else if (ph == 0) {
        wait_vm<Gm::AI + X>();  // the last K-tile's A m-half-1 region (j3) follows
      } else if (ph == 1) {
        wait_vm<0 + X>();
      }
    }
    big8_bar();
    __builtin_amdgcn_sched_barrier(0);
    const int mb = (ph >= 2) ? MH : 0, nb = (ph == 1 || ph == 2) ? NH : 0;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int nt = 0; nt < NH; ++nt)
#pragma unroll
        for (int mt = 0; mt < MH; ++mt)
          Mma<bf16>::run(nb ? bf1[nt][ks] : bf0[nt][ks], af[mt][ks], acc[nb + nt][mb + mt]);
    if (!(OPEN && MODE == 2 && ph == 3 && wm == 1)) big8_bar();
  }
}

// Two-phase schedule (big8_loop<..., KT2 = true>: the LN-folded FC1 + GELU kernels only): per
// K-tile and wave group two MFMA bursts of 32 (n-halves 0 and 1 of m-half 0, then of m-half 1)
// instead of four of 16 (FC1 -1.5 %; the instances with residual or head-major epilogues spill
// with it, profiles/r05_gemm_two_phase_ab.txt). The region stream keeps the order of
// big8_prologue; regions 0..2 of K-tile T are issued in phase 1 of K-tile T - 2, region 3 in phase
// 0 of K-tile T - 1 (one K-tile of flight each), 8 glds per lane younger at every wait; K-tile 1's
// region 2 waits for K-tile 0's phase 0 (the epilogue's scratch is in it: with cont, the previous
// tile's last K-tile issues the next tile's (0, 0..3), (1, 0..1) like big8_prologue). WAR: a
// region is overwritten one barrier after its last read, so every wave retires its fragment reads
// (lgkmcnt 0) before its opening barrier.
template <int MODE, int X, bool OPEN = false, int X3 = 0, typename Ph3 = NoOp,
          typename P = GemmParams>
__device__ __forceinline__ void big8_ktile2(const P& p, char* smem,
                                            f32x4 (&acc)[GeoOf<P>::NF][GeoOf<P>::MF],
                                            int wave, int lane, int wm, int wn, int m0, int n0,
                                            int t, bool cont = false, int nm0 = 0, int nn0 = 0,
                                            Ph3 ph3 = {}, int par = 0, int npar = 0) {
  typedef Geo<P> Gm;
  constexpr int MH = Gm::MH, NH = Gm::NH;
  // phase 0 reads regions 0..2 (and, 128 x 384, the first instruction of region 3): 8 younger
  // glds after region 2, 7 after that instruction (big8_stage's paired order)
  constexpr int W0 = Gm::WI == 3 ? 7 : 8;
  const int frow = lane & 15, fsw = lane & 7, fg = lane >> 4;
  const EVT_LDS char* As = (const EVT_LDS char*)smem + ((t ^ par) & 1) * BIG_STAGE;
  const EVT_LDS char* Ws = As + Gm::A_TILE;
  auto rd = [&](const EVT_LDS char* S, int row, int ks) {
    return *(const EVT_LDS u32x4*)(S + row * ROWB + (((fg + 4 * ks) ^ fsw) << 4));
  };
  u32x4 af[MH][2], bf0[NH][2], bf1[NH][2];
#pragma unroll
  for (int ph = 0; ph < 2; ++ph) {
    // the DMA first: its address arithmetic then overlaps dead fragment registers (issued after
    // the reads it spilled in the out-proj / QKV instantiations)
    if (MODE == 0 || (MODE == 1 && ph == 0)) {
      if (ph == 0) {
        if (t == 0) big8_stage(p, smem, wave, lane, m0, n0, 1, 2, par);
        big8_stage(p, smem, wave, lane, m0, n0, t + 1, 3, par);
      } else {
#pragma unroll
        for (int j = 0; j < 3; ++j) big8_stage(p, smem, wave, lane, m0, n0, t + 2, j, par);
      }
    } else if (cont) {  // the next tile's regions: (0, 0..2) | (0, 3), (1, 0..1)
      if (ph == 0) {
        big8_stage(p, smem, wave, lane, nm0, nn0, 0, 3, npar);
      } else {
#pragma unroll
        for (int j = 0; j < (MODE == 1 ? 3 : 2); ++j)
          big8_stage(p, smem, wave, lane, nm0, nn0, MODE == 1 ? 0 : 1, j, npar);
      }
    }
    if (ph == 0) {
#pragma unroll
      for (int nt = 0; nt < NH; ++nt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) bf0[nt][ks] = rd(Ws, wn * Gm::WC + nt * 16 + frow, ks);
#pragma unroll
      for (int mt = 0; mt < MH; ++mt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) af[mt][ks] = rd(As, wm * Gm::WR + mt * 16 + frow, ks);
#pragma unroll
      for (int nt = 0; nt < NH; ++nt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          bf1[nt][ks] = rd(Ws, wn * Gm::WC + Gm::WC / 2 + nt * 16 + frow, ks);
    } else {
#pragma unroll
      for (int mt = 0; mt < MH; ++mt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          af[mt][ks] = rd(As, wm * Gm::WR + Gm::WR / 2 + mt * 16 + frow, ks);
    }
    // retire what the next phase reads: region 3 after phase 0 (X: younger, issued before the
    // K-tile), the next K-tile's regions 0..2 after phase 1 (X older than those)
    if (ph == 0) {
      if (MODE != 2 || cont) wait_vm<8 + X>();
      else wait_vm<0 + X>();
    } else if (MODE == 0 || (MODE == 1 && cont)) {
      wait_vm<W0>();
    } else if (MODE == 1) {
      wait_vm<W0 - 6>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    big8_bar();
    __builtin_amdgcn_sched_barrier(0);
    const int mb = ph ? MH : 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int nb = (ph ^ h) ? NH : 0;  // phase 0: n-half 0 then 1; phase 1: 1 then 0
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int nt = 0; nt < NH; ++nt)
#pragma unroll
          for (int mt = 0; mt < MH; ++mt)
            Mma<bf16>::run(nb ? bf1[nt][ks] : bf0[nt][ks], af[mt][ks], acc[nb + nt][mb + mt]);
      // the X3 loads once the n-half-1 fragments are dead (their registers)
      if (ph == 1 && h == 0) ph3();
    }
    if (!(OPEN && MODE == 2 && ph == 1 && wm == 1)) big8_bar();
  }
}

// one K-tile of either schedule
template <bool KT2, int MODE, int X, bool OPEN = false, int X3 = 0, typename Ph3 = NoOp,
          typename P = GemmParams>
__device__ __forceinline__ void big8_kt(const P& p, char* smem,
                                        f32x4 (&acc)[GeoOf<P>::NF][GeoOf<P>::MF], int wave,
                                        int lane, int wm, int wn, int m0, int n0, int t,
                                        bool cont = false, int nm0 = 0, int nn0 = 0, Ph3 ph3 = {},
                                        int par = 0, int npar = 0) {
  if constexpr (KT2)
    big8_ktile2<MODE, X, OPEN, X3>(p, smem, acc, wave, lane, wm, wn, m0, n0, t, cont, nm0, nn0,
                                   ph3, par, npar);
  else
    big8_ktile<MODE, X, OPEN, X3>(p, smem, acc, wave, lane, wm, wn, m0, n0, t, cont, nm0, nn0,
                                  ph3, par, npar);
}

// Main loop over the nk K-tiles after big8_prologue (whose DMAs may be followed by X further
// VMEM instructions per wave, or by a vmcnt(0)). Ends with every wave past a common barrier.
// pre1: run by wave group 1 in the slot where it waits one barrier for group 0 (per-tile LDS
// setup work that is then off the critical path); mid: after K-tile 0 (nk >= 3 only).
// last: issues LX further VMEM loads per wave just before the last K-tile (added to its waits:
// they are younger than every DMA that tile waits for); last3: LX3 more at the start of the last
// K-tile's phase 3.
template <int X, bool OPEN = false, typename Pre1 = NoOp, typename Mid = NoOp, int LX = 0,
          typename Last = NoOp, int LX3 = 0, typename Last3 = NoOp, typename P = GemmParams,
          bool KT2 = false, bool U2 = false>
__device__ __forceinline__ void big8_loop(const P& p, char* smem,
                                          f32x4 (&acc)[GeoOf<P>::NF][GeoOf<P>::MF],
                                          int wave, int lane, int wm, int wn, int m0, int n0,
                                          int nk, bool cont = false, int nm0 = 0, int nn0 = 0,
                                          Pre1 pre1 = {}, Mid mid = {}, Last last = {},
                                          Last3 last3 = {}, int par = 0) {
  // K-tile t of this tile sits in buffer (t ^ par) & 1; the next tile (cont) starts at the parity
  // of stream K-tile nk
  const int npar = par ^ (nk & 1);
  if constexpr (KT2) {
    // phase 0 reads regions 0..2 (big8_ktile2): younger are (0, 3) and (1, 0..1)
    constexpr int W0 = Geo<P>::WI == 3 ? 7 : 8;
    if (nk >= 2) wait_vm<W0 - 2 + X>();
    else wait_vm<W0 - 6 + X>();
  } else {
    if (nk >= 2) wait_vm<8 + X>();
    else wait_vm<4 + X>();
  }
  big8_bar();
  if (wm == 1) {
    pre1();
    big8_bar();
  }
  if (nk >= 3) {
    big8_kt<KT2, 0, X>(p, smem, acc, wave, lane, wm, wn, m0, n0, 0, false, 0, 0, {}, par, 0);
    mid();
    int t = 1;
    // U2: two K-tiles per iteration: t is odd in the first, even in the second, so each one's
    // buffer parity (t ^ par) & 1 and region addresses are loop-invariant (round 6: SALU 42 -> 18.5
    // and VALU 6 -> 2 per K-tile; QKV 315.4 -> 310.9 µs, FC2 386.4 -> 377.7, DeiT-base +0.9 %,
    // profiles/r06_unroll2_ab.txt); not where the doubled body spills (pers_run)
    if constexpr (U2) {
      for (; t + 3 < nk; t += 2) {
        big8_kt<KT2, 0, 0>(p, smem, acc, wave, lane, wm, wn, m0, n0, t, false, 0, 0, {}, par, 0);
        big8_kt<KT2, 0, 0>(p, smem, acc, wave, lane, wm, wn, m0, n0, t + 1, false, 0, 0, {}, par, 0);
      }
    }
    for (; t + 2 < nk; ++t)
      big8_kt<KT2, 0, 0>(p, smem, acc, wave, lane, wm, wn, m0, n0, t, false, 0, 0, {}, par, 0);
    big8_kt<KT2, 1, 0>(p, smem, acc, wave, lane, wm, wn, m0, n0, t, cont, nm0, nn0, {}, par, npar);
    last();
    big8_kt<KT2, 2, LX, OPEN, LX3>(p, smem, acc, wave, lane, wm, wn, m0, n0, t + 1, cont, nm0, nn0,
                                 last3, par, npar);
  } else if (nk == 2) {
    big8_kt<KT2, 1, X>(p, smem, acc, wave, lane, wm, wn, m0, n0, 0, cont, nm0, nn0, {}, par, npar);
    last();
    big8_kt<KT2, 2, LX, OPEN, LX3>(p, smem, acc, wave, lane, wm, wn, m0, n0, 1, cont, nm0, nn0, last3,
                                 par, npar);
  } else {
    last();
    big8_kt<KT2, 2, X + LX, OPEN, LX3>(p, smem, acc, wave, lane, wm, wn, m0, n0, 0, false, 0, 0,
                                     last3, par);
  }
  if (!OPEN && wm == 0) big8_bar();
}

template <int FL, int VAR_, bool NOEPI = false>
__global__ __launch_bounds__(512, 2) void gemm_big_kernel(GemmParams p) {
  constexpr int VAR = VAR_;
  __shared__ __attribute__((aligned(16))) char smem[2 * BIG_STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably uniform -> SGPR math
  // VAR 8 pairs the two waves of a SIMD across the wave groups wm = 0 / 1 (waves w, w + 4)
  const int wm = VAR == 8 ? wave >> 2 : wave & 1, wn = VAR == 8 ? wave & 3 : wave >> 1;
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = wgid / p.ntiles, tn = wgid - tm * p.ntiles;
  const int m0 = tm * BIG_BM, n0 = tn * BIG_BN;

  const int srow = lane >> 3, sslot = lane & 7;
  const int64_t lda_b = p.lda * 2, ldw_b = p.ldw * 2;
  // Addresses are recomputed per stage (a few VALU ops) instead of held in 16 VGPRs.
  const int arow0 = m0 + wave * 32 + srow;
  const char* a_base = (const char*)p.A + ((sslot ^ srow) * 16);
  const char* w_base = (const char*)p.W + (int64_t)(n0 + wave * 32 + srow) * ldw_b + ((sslot ^ srow) * 16);
  auto stage = [&](int kt, int buf) {
    EVT_LDS char* base = (EVT_LDS char*)smem + buf * BIG_STAGE;
    const int64_t koff = (int64_t)kt * ROWB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gm = min(arow0 + i * 8, p.M - 1);
      glds16(a_base + gm * lda_b + koff, base + (wave * 32 + i * 8) * ROWB);
      glds16(w_base + (i * 8) * ldw_b + koff, base + BIG_TILE + (wave * 32 + i * 8) * ROWB);
    }
  };

  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / 64;
  const int frow = lane & 15, fsw = lane & 7, fg = lane >> 4;
  auto read_step = [&](int kt, int ks, u32x4 (&a)[8], u32x4 (&w)[4]) {
    const EVT_LDS char* As = (const EVT_LDS char*)smem + (kt & 1) * BIG_STAGE;
    const EVT_LDS char* Ws = As + BIG_TILE;
    const int coff = ((fg + 4 * ks) ^ fsw) * 16;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
      w[nt] = *(const EVT_LDS u32x4*)(Ws + (wn * 64 + nt * 16 + frow) * ROWB + coff);
#pragma unroll
    for (int mt = 0; mt < 8; ++mt)
      a[mt] = *(const EVT_LDS u32x4*)(As + (wm * 128 + mt * 16 + frow) * ROWB + coff);
  };
  auto mfma_step = [&](const u32x4 (&a)[8], const u32x4 (&w)[4]) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) Mma<bf16>::run(w[nt], a[mt], acc[nt][mt]);
  };
  if constexpr (VAR == 8) {
    big8_prologue(p, smem, wave, lane, m0, n0, nk);
    big8_loop<0>(p, smem, acc, wave, lane, wm, wn, m0, n0, nk);
  } else {
  stage(0, 0);
  if constexpr (VAR == 6) {
    auto tile = [&](int kt, bool dma) {
      wait_vmcnt0();
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      u32x4 a0[8], w0[4], a1[8], w1[4];
      read_step(kt, 0, a0, w0);
      if (dma) stage(kt + 1, (kt + 1) & 1);
      read_step(kt, 1, a1, w1);
      mfma_step(a0, w0);
      mfma_step(a1, w1);
      __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);  // DS read
      if (dma) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // MFMA
          __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);  // VMEM (glds)
        }
      } else {
        __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
      }
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 36, 0);
      __builtin_amdgcn_sched_barrier(0);
    };
    for (int kt = 0; kt + 1 < nk; ++kt) tile(kt, true);
    tile(nk - 1, false);
  } else {
    for (int kt = 0; kt < nk; ++kt) {
      wait_vmcnt0();
      __builtin_amdgcn_s_barrier();
      if (kt + 1 < nk) stage(kt + 1, (kt + 1) & 1);
      u32x4 a[8], w[4];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        read_step(kt, ks, a, w);
        mfma_step(a, w);
      }
    }
  }
  }

  if constexpr (NOEPI) {  // ablation: main loop only, accumulators kept live by a dead store
    float sink = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) sink += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (sink == 1234.5f) ((float*)p.C)[tid] = sink;
  } else {
    big_epilogue<FL>(p, smem, acc, wm, wn, m0, n0, tn, wave, lane);
  }
}


// ---------------------------------------------------------------------------------------------
// Persistent 256x256 kernel with the epilogue in registers (bf16 output; FL without POS /
// OUT_F32). One block per CU walks its tiles (XCD-aware: in every round an XCD takes a
// contiguous range of logical tiles); per tile:
//   main loop (big8_loop) -> LayerNorm coefficients / column vectors into LDS ->
//   DMA of the NEXT tile's prologue (and its statistics / column vectors) ->
//   epilogue of this tile straight from the accumulators, overlapping those DMAs ->
//   the next main loop starts while this tile's output stores drain.
// The accumulators are converted in the MFMA layout (lane: token row mt*16 + (lane & 15),
// features 4 (lane >> 4) + j), then v_permlane16_swap pairs fragments (2k, 2k+1) so that every
// lane holds 8 consecutive features of one row: 16-B residual loads and 16-B output stores,
// no LDS staging of the tile. Row statistics (EPI_STATS): 64-column partials per wave, the two
// waves of a 128-column slab combined in a fixed order (slot 2 tn + slab, as the staged
// epilogue). Every interior tile issues its 16 output stores per wave after the next tile's
// prologue DMAs, which is what the first K-tile's counted waits (X = 16) assume; an edge tile
// drains with vmcnt(0) instead.
// ---------------------------------------------------------------------------------------------
constexpr int PERS_RAW = 2 * BIG_STAGE;         // raw LN statistics of the tile rows [256][<=8] f32x2
constexpr int PERS_COLRAW = PERS_RAW + 16384;   // DMA'd column vectors [3][256] f32
constexpr int PERS_COEF = PERS_COLRAW + 3072;   // LayerNorm (mu, r) per tile row [256] f32x2
constexpr int PERS_COLB = PERS_COEF + 2048;     // column vectors of the tile being finished
constexpr int PERS_PART = PERS_COLB + 3072;     // odd-wn waves' row partials [2][256] f32x2
constexpr int PERS_LDS = PERS_PART + 4096;
constexpr int PERS_LDS_ALL = PERS_LDS + 16;
constexpr int PERS_X = 16;                      // output stores per wave per interior tile

template <int FL>
struct PersFlags {
  static constexpr bool ln = (FL & (EPI_LNIN | EPI_RESLN)) != 0;
  // column vector slots: 0 bias, 1 colsum (LNIN) or rgamma (RESLN), 2 rbeta (RESLN)
  static constexpr bool v0 = (FL & EPI_BIAS) != 0;
  static constexpr bool v1 = (FL & (EPI_LNIN | EPI_RESLN)) != 0;
  static constexpr bool v2 = (FL & EPI_RESLN) != 0;
  static_assert(!((FL & EPI_LNIN) && (FL & EPI_RESLN)), "one LayerNorm source per GEMM");
  static_assert(!(FL & EPI_RESLN) || ((FL & EPI_BIAS) && (FL & EPI_RESID)),
                "RESLN: the residual LayerNorm's beta is folded into the bias add");
  static_assert(!(FL & EPI_OUT_F32), "persistent kernel: bf16 outputs");
  // EPI_POS (patch embedding): + pos[t + 1][n] from a bf16 copy of the table in p.resid (pitch
  // p.ldr), row remap b*P + t -> b*(P+1) + 1 + t of the outputs and their statistics
  static_assert(!(FL & EPI_POS) || !(FL & (EPI_RESID | EPI_LNIN)), "POS: its own residual form");
};

// DMA the tile's LN statistics rows and column vectors into LDS (before its prologue DMAs).
template <int FL>
__device__ __forceinline__ void pers_coop_dma(const GemmParams& p, char* smem, int wave, int lane,
                                              int m0, int n0) {
  typedef PersFlags<FL> F;
  asm volatile("" : "+v"(lane));
  if constexpr (F::ln) {
    const float* st = (FL & EPI_LNIN) ? p.stats_in : p.rstats;
    const int half = p.nslots >> 1;  // 16-B chunks per row
    const int nch = 256 * half;
    const int64_t c0 = (int64_t)m0 * half, clast = (int64_t)p.M * half - 1;
    for (int c = wave * 64; c < nch; c += 512)
      glds16(st + 4 * min(c0 + c + lane, clast), (EVT_LDS char*)smem + PERS_RAW + c * 16);
  }
  const float* v = nullptr;
  if (wave == 0 && F::v0) v = p.bias;
  if (wave == 1 && (FL & EPI_LNIN)) v = p.colsum;
  if (wave == 1 && (FL & EPI_RESLN)) v = p.rgamma;
  if (wave == 2 && F::v2) v = p.rbeta;
  if (v) glds16(v + min(n0 + 4 * lane, p.N - 4), (EVT_LDS char*)smem + PERS_COLRAW + wave * 1024);
}

// Per-row LayerNorm coefficients (as ln_coef) and a copy of the column vectors for the epilogue.
template <int FL>
__device__ __forceinline__ void pers_coef(const GemmParams& p, char* smem, int tid) {
  typedef PersFlags<FL> F;
  asm volatile("" : "+v"(tid));
  if (tid < 256) {
    if constexpr (F::ln) {
      const EVT_LDS f32x2* st = (const EVT_LDS f32x2*)(smem + PERS_RAW) + tid * p.nslots;
      float s1 = 0.f, s2 = 0.f;
      for (int j = 0; j < p.nslots; ++j) {
        const f32x2 v = st[j];
        s1 += v[0];
        s2 += v[1];
      }
      const float mu = s1 * p.inv_d;
      const float r = rsqrtf(fmaxf(s2 * p.inv_d - mu * mu, 0.f) + p.eps);
      ((EVT_LDS f32x2*)(smem + PERS_COEF))[tid] = f32x2{mu, r};
    }
    const EVT_LDS float* src = (const EVT_LDS float*)(smem + PERS_COLRAW);
    EVT_LDS float* dst = (EVT_LDS float*)(smem + PERS_COLB);
    if (F::v0) dst[tid] = src[tid];
    if (F::v1) dst[256 + tid] = src[256 + tid];
    if (F::v2) dst[512 + tid] = src[512 + tid];
  }
}

__device__ __forceinline__ f32x4 lds4(const EVT_LDS float* p) { return *(const EVT_LDS f32x4*)p; }

// v_permlane16_swap_b32 on (x, y): odd 16-lane rows of x <-> even rows of y. Written on scalars:
// applied in place to vector elements (v[j] = swap(...)[0] in a loop) hipcc 7.2 miscompiles the
// builtin (it reuses element 0 for every j).
__device__ __forceinline__ float swp16(float x, float y, float& yo) {
  const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, x),
                                                  __builtin_bit_cast(unsigned, y), false, false);
  yo = __builtin_bit_cast(float, (unsigned)r[1]);
  return __builtin_bit_cast(float, (unsigned)r[0]);
}
__device__ __forceinline__ void swap_rows16(f32x4& a, f32x4& b) {
  float y0, y1, y2, y3;
  const float x0 = swp16(a[0], b[0], y0), x1 = swp16(a[1], b[1], y1);
  const float x2 = swp16(a[2], b[2], y2), x3 = swp16(a[3], b[3], y3);
  a = f32x4{x0, x1, x2, x3};
  b = f32x4{y0, y1, y2, y3};
}

// PADN: the output width N is not a multiple of the tile (Swin / pruned widths): column groups
// entirely past N skip their epilogue VALU work. Compiled out otherwise (the check alone cost
// 2-4 % on the DeiT shapes, measured in one process).
template <int FL, int DBG = 0, bool PADN = true>
__device__ __forceinline__ void pers_epilogue_v1(const GemmParams& p, char* smem, f32x4 (&acc)[4][8],
                                              int wave, int wm, int wn, int m0, int n0, int tn,
                                              int lane, bool interior) {
  asm volatile("" : "+v"(lane));  // keep lane-derived addresses out of the persistent loop (VGPRs)
  if constexpr (DBG == 2) {  // ablation: no epilogue at all, accumulators kept live by a dead store
    float sink = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) sink += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (sink == 1234.5f) ((float*)p.C)[lane] = sink;
    return;
  }
  const int frow = lane & 15, fg = lane >> 4;
  const EVT_LDS f32x2* coef = (const EVT_LDS f32x2*)(smem + PERS_COEF);
  const EVT_LDS float* colb = (const EVT_LDS float*)(smem + PERS_COLB);
  // 1. MFMA layout: row wm*128 + mt*16 + frow, columns wn*64 + nt*16 + 4 fg + j
  if constexpr ((FL & (EPI_LNIN | EPI_BIAS)) != 0) {
    f32x4 b4[4], c4[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int c = wn * 64 + nt * 16 + 4 * fg;
      b4[nt] = (FL & EPI_BIAS) ? lds4(colb + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      if (FL & EPI_LNIN) c4[nt] = lds4(colb + 256 + c);
    }
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      float mu = 0.f, r = 0.f;
      if (FL & EPI_LNIN) {
        const f32x2 cf = coef[wm * 128 + mt * 16 + frow];
        mu = cf[0];
        r = cf[1];
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        if (PADN && !interior && n0 + wn * 64 + nt * 16 >= p.N) continue;  // padding: skip
        if (FL & EPI_LNIN) acc[nt][mt] = acc[nt][mt] * r - c4[nt] * (r * mu) + b4[nt];
        else acc[nt][mt] += b4[nt];
      }
    }
  }
  if constexpr ((FL & (EPI_GELU | EPI_GELU_ERF)) != 0) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      // column group past N (padding of the packed width): wave-uniform skip of the VALU work
      if (PADN && !interior && n0 + wn * 64 + nt * 16 >= p.N) continue;
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) acc[nt][mt] = gelu4(acc[nt][mt], (FL & EPI_GELU) ? 0 : 2);
    }
  }
  // 2. store layout: pair (2k, 2k+1) -> lane row wm*128 + (2k + (fg & 1))*16 + frow, columns
  //    wn*64 + nt*16 + (fg >> 1)*8 + [acc[nt][2k][0..3], acc[nt][2k+1][0..3]]
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int k = 0; k < 4; ++k) swap_rows16(acc[nt][2 * k], acc[nt][2 * k + 1]);
  const int rl = wm * 128 + (fg & 1) * 16 + frow;  // + 32 k
  const int cl = wn * 64 + (fg >> 1) * 8;           // + 16 nt
  bool rok[4], cok[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) rok[k] = interior || m0 + rl + 32 * k < p.M;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) cok[nt] = interior || n0 + cl + 16 * nt < p.N;
  // 3. residual (16-B loads in the store layout, all issued up front), bf16 stores and the row
  //    statistics of the stored values; nt-major so each column-vector slice is read once
  u32x4 rr[4][4];
  if constexpr ((FL & EPI_RESID) != 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        rr[k][nt] = u32x4{0u, 0u, 0u, 0u};
        if (rok[k] && cok[nt])
          rr[k][nt] = *(const u32x4*)((const bf16*)p.resid + (int64_t)(m0 + rl + 32 * k) * p.ldr +
                                      n0 + cl + 16 * nt);
      }
  }
  f32x2 rc[4], st[4];
  u32x4 ov[4][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    rc[k] = (FL & EPI_RESLN) ? coef[rl + 32 * k] : f32x2{0.f, 0.f};
    st[k] = f32x2{0.f, 0.f};
  }
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int c = cl + 16 * nt;
    f32x4 g[2], be[2];
    if (FL & EPI_RESLN) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        g[h] = lds4(colb + 256 + c + 4 * h);
        be[h] = lds4(colb + 512 + c + 4 * h);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f32x4 a = acc[nt][2 * k], b = acc[nt][2 * k + 1];
      if constexpr ((FL & EPI_RESID) != 0) {
        const bf16x8 r8 = __builtin_bit_cast(bf16x8, rr[k][nt]);
        f32x4 rv[2] = {f32x4{(float)r8[0], (float)r8[1], (float)r8[2], (float)r8[3]},
                       f32x4{(float)r8[4], (float)r8[5], (float)r8[6], (float)r8[7]}};
        if (FL & EPI_RESLN) {
#pragma unroll
          for (int h = 0; h < 2; ++h) rv[h] = (rv[h] - rc[k][0]) * rc[k][1] * g[h] + be[h];
        }
        a += rv[0];
        b += rv[1];
      }
      const bf16x8 o = {(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3],
                        (bf16)b[0], (bf16)b[1], (bf16)b[2], (bf16)b[3]};
      ov[k][nt] = __builtin_bit_cast(u32x4, o);
      if (FL & EPI_STATS) {
        if (cok[nt]) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float x = (float)o[e];
            st[k][0] += x;
            st[k][1] += x * x;
          }
        }
      }
    }
  }
  // 4. output: per row pair k, the wave's 32 x 64 block goes through its private 4 KiB of LDS
  //    (free during the epilogue: buffer-1 regions 2 / 3 are only DMA'd in the next tile's
  //    phases 1 / 2) and leaves as whole 128-B row segments, 8 rows per store instruction
  {
    const int w = wave;
    EVT_LDS char* scr = (EVT_LDS char*)smem +
                        (w < 4 ? (96 + 4 + 8 * w) * 1024 : (72 + (w - 4) * 4 + ((w - 4) >> 1) * 8) * 1024);
    const int wrow = (fg & 1) * 16 + frow;               // store-layout row within the pair
    const int rrow = lane >> 3, rch = lane & 7;          // row-layout lane: row i*8 + rrow, chunk
    const bool rcol_ok = interior || n0 + wn * 64 + rch * 8 < p.N;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int ch = 2 * nt + (fg >> 1);
        *(EVT_LDS u32x4*)(scr + wrow * 128 + ((ch ^ (wrow & 7)) << 4)) = ov[k][nt];
      }
      asm volatile("" ::: "memory");  // (a wave's LDS operations execute in order)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = i * 8 + rrow;
        const u32x4 v = *(const EVT_LDS u32x4*)(scr + r * 128 + ((rch ^ (r & 7)) << 4));
        const int m = m0 + wm * 128 + 32 * k + r;
        bool keep = true;
        if (DBG == 1) {  // ablation: no stores, every value stays live
          keep = (v[0] ^ v[1] ^ v[2] ^ v[3]) == 0x12345u;
        }
        if ((interior || m < p.M) && rcol_ok && keep) {
          u32x4* cp = (u32x4*)((bf16*)p.C + (int64_t)m * p.ldc + n0 + wn * 64 + rch * 8);
          store_b128_nt(cp, v);  // whole lines: streamed past L2
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  if constexpr ((FL & EPI_STATS) != 0) {
    // lanes fg and fg ^ 2 hold the two 32-column halves of the same row
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      st[k][0] += __shfl_xor(st[k][0], 32, 64);
      st[k][1] += __shfl_xor(st[k][1], 32, 64);
    }
    EVT_LDS f32x2* part = (EVT_LDS f32x2*)(smem + PERS_PART) + (wn >> 1) * 256;
    if ((wn & 1) && lane < 32) {
#pragma unroll
      for (int k = 0; k < 4; ++k) part[rl + 32 * k] = st[k];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    big8_bar();
    if (!(wn & 1) && lane < 32) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int m = m0 + rl + 32 * k;
        const f32x2 o = part[rl + 32 * k];
        if (interior || m < p.M)
          *(f32x2*)(p.stats_out + 2 * ((int64_t)p.nslots * m + 2 * tn + (wn >> 1))) = st[k] + o;
      }
    }
  }
}

// Buffer resource of one tile's rows of an output / residual matrix [M][ld] (bf16): base = the
// tile's first element (m0, n0), num_records = the bytes to the end of the tile's last valid row,
// so rows past M are dropped (stores) / read as 0 (loads) by the hardware range check instead of
// per-lane branches. m0 / n0 go through readfirstlane and every input stays 32-bit: a 64-bit
// min/max in the byte count is lowered to VALU, and hipcc then no longer proves the descriptor
// wave-uniform and wraps every buffer op in a waterfall loop (guide T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const void* mat, int64_t ld, int M,
                                                           int m0, int n0) {
  m0 = __builtin_amdgcn_readfirstlane(m0);
  n0 = __builtin_amdgcn_readfirstlane(n0);
  const int nr = (min(M - m0, 256) * (int)ld - n0) * 2;  // ld < 2^22: a tile spans < 2 GB
  return __builtin_amdgcn_make_buffer_rsrc((char*)const_cast<void*>(mat) + ((int64_t)m0 * ld + n0) * 2,
                                           0, nr, 0x00020000);
}

// EPI_POS row arithmetic: image of patch row m (m / P, exact in fp32 for m < 2^22 with the
// half-row offset) and its token row in the stream, b*(P+1) + 1 + t = m + m/P + 1.
__device__ __forceinline__ int pos_img(int m, int P) {
  return (int)(((float)m + 0.5f) * (1.0f / (float)P));
}
__device__ __forceinline__ int pos_orow(int m, int P) { return m + pos_img(m, P) + 1; }

// Epilogue of one 256 x 256 tile straight from the accumulators (VALU-bound: every instruction
// here is paid with the MFMA pipe idle, so the arithmetic is in packed form throughout):
//   LNIN   r (acc - mu colsum) + c      2 v_pk_fma per column pair
//   BIAS   acc + bias (+ beta of the residual LayerNorm when RESLN: folded into one add)
//   RESLN  + gamma (r resid - r mu)     2 v_pk_fma per pair on the unpacked bf16 residual
//   STATS  (sum, sumsq) of the stored bf16 values with v_dot2c_f32_bf16 (2 per stored dword)
// Residual loads and output stores go through tile buffer resources (SGPR base per tile, lane
// offsets tile-invariant, row offsets in SGPRs): no per-store 64-bit address arithmetic and no
// exec-mask branches for the M edge.
// Residual of the first ER row pairs (the epilogue's rr[0 .. ER-1]), issued before the tile's last
// K-tile so that part of the residual fetch is in flight under its MFMAs (ER = 1: the most that
// fits in 256 VGPRs without spilling).
template <int K0, int K1>
__device__ __forceinline__ void pers_resid_early(const GemmParams& p, int wm, int wn, int lane,
                                                 int m0, int n0, u32x4 (&rre)[2][4]) {
  const int frow = lane & 15, fg = lane >> 4;
  const int rl = wm * 128 + (fg & 1) * 16 + frow, cl = wn * 64 + (fg >> 1) * 8;
  const __amdgpu_buffer_rsrc_t rs = tile_rsrc(p.resid, p.ldr, p.M, m0, n0);
  const int vo = (rl * (int)p.ldr + cl) * 2;
#pragma unroll
  for (int k = K0; k < K1; ++k) {
    const int so = __builtin_amdgcn_readfirstlane(32 * k * (int)p.ldr * 2);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
      rre[k][nt] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo + 32 * nt, so, 0));
  }
}

template <int FL, int DBG = 0, bool PADN = true, int ER = 0>
__device__ __forceinline__ void pers_epilogue(const GemmParams& p, char* smem, f32x4 (&acc)[4][8],
                                              int wave, int wm, int wn, int m0, int n0, int tn,
                                              int lane, bool interior, int iter = 0,
                                              const u32x4 (*rre)[4] = nullptr, int spar = 0) {
  // DBG 3: sub-stamps 3..5 of the tile's timeline row (wave 0, lane 0)
  auto stamp = [&](int k) {
    if (DBG == 3 && wave == 0 && lane == 0 && iter < 16)
      ((unsigned long long*)p.pos)[((int64_t)blockIdx.x * 16 + iter) * 8 + k] = __builtin_amdgcn_s_memtime();
  };
  asm volatile("" : "+v"(lane));  // keep lane-derived addresses out of the persistent loop (VGPRs)
  if constexpr (DBG == 2) {  // ablation: no epilogue at all, accumulators kept live by a dead store
    float sink = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) sink += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (sink == 1234.5f) ((float*)p.C)[lane] = sink;
    return;
  }
  const int frow = lane & 15, fg = lane >> 4;
  const EVT_LDS f32x2* coef = (const EVT_LDS f32x2*)(smem + PERS_COEF);
  const EVT_LDS float* colb = (const EVT_LDS float*)(smem + PERS_COLB);
  auto padskip = [&](int nt) { return PADN && !interior && n0 + wn * 64 + nt * 16 >= p.N; };
  // 1. MFMA layout: row wm*128 + mt*16 + frow, columns wn*64 + nt*16 + 4 fg + j
  if constexpr ((FL & EPI_LNIN) != 0) {
    f32x4 b4[4], c4[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int c = wn * 64 + nt * 16 + 4 * fg;
      b4[nt] = (FL & EPI_BIAS) ? lds4(colb + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      c4[nt] = lds4(colb + 256 + c);
    }
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      const f32x2 cf = coef[wm * 128 + mt * 16 + frow];
      const f32x2 nmu = {-cf[0], -cf[0]}, rr = {cf[1], cf[1]};
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        if (padskip(nt)) continue;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          f32x2 a = {acc[nt][mt][2 * h], acc[nt][mt][2 * h + 1]};
          const f32x2 cs = {c4[nt][2 * h], c4[nt][2 * h + 1]}, bb = {b4[nt][2 * h], b4[nt][2 * h + 1]};
          a = __builtin_elementwise_fma(cs, nmu, a);
          a = __builtin_elementwise_fma(a, rr, bb);
          acc[nt][mt][2 * h] = a[0];
          acc[nt][mt][2 * h + 1] = a[1];
        }
      }
    }
  } else if constexpr ((FL & EPI_BIAS) != 0) {
    f32x4 b4[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int c = wn * 64 + nt * 16 + 4 * fg;
      b4[nt] = lds4(colb + c);
      if (FL & EPI_RESLN) b4[nt] += lds4(colb + 512 + c);  // + beta of LN(resid)
    }
#pragma unroll
    for (int mt = 0; mt < 8; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        if (padskip(nt)) continue;
        acc[nt][mt] += b4[nt];
      }
  }
  if constexpr ((FL & (EPI_GELU | EPI_GELU_ERF)) != 0) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      // column group past N (padding of the packed width): wave-uniform skip of the VALU work
      if (padskip(nt)) continue;
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) acc[nt][mt] = gelu4(acc[nt][mt], (FL & EPI_GELU) ? 0 : 2);
    }
  }
  stamp(3);
  // 2. store layout: pair (2k, 2k+1) -> lane row wm*128 + (2k + (fg & 1))*16 + frow, columns
  //    wn*64 + nt*16 + (fg >> 1)*8 + [acc[nt][2k][0..3], acc[nt][2k+1][0..3]]
  //    (no residual / position / statistics: the values are packed to bf16 first and the swap
  //    moves 2 dwords per pair instead of 4; the same elements, bitwise the same stores)
  constexpr bool PACK_FIRST = (FL & (EPI_RESID | EPI_POS | EPI_STATS)) == 0;
  if constexpr (!PACK_FIRST) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int k = 0; k < 4; ++k) swap_rows16(acc[nt][2 * k], acc[nt][2 * k + 1]);
  }
  const int rl = wm * 128 + (fg & 1) * 16 + frow;  // + 32 k
  const int cl = wn * 64 + (fg >> 1) * 8;           // + 16 nt
  bool cok[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) cok[nt] = !PADN || interior || n0 + cl + 16 * nt < p.N;
  // 3. residual (16-B buffer loads in the store layout, all issued up front), bf16 stores and the
  //    row statistics of the stored values; nt-major so each column-vector slice is read once
  u32x4 rr[4][4];
  if constexpr (DBG == 7) {  // ablation: no residual loads (zeros)
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) rr[k][nt] = u32x4{0u, 0u, 0u, 0u};
  } else if constexpr ((FL & EPI_RESID) != 0) {
    const __amdgpu_buffer_rsrc_t rs = tile_rsrc(p.resid, p.ldr, p.M, m0, n0);
    const int vo = (rl * (int)p.ldr + cl) * 2;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int so = __builtin_amdgcn_readfirstlane(32 * k * (int)p.ldr * 2);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        rr[k][nt] = k < ER ? rre[k][nt]
                           : __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo + 32 * nt, so, 0));
    }
  } else if constexpr ((FL & EPI_POS) != 0) {  // pos[t + 1][n0 + cl + 16 nt ..] (bf16 table)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(p.resid), 0, (p.P + 1) * (int)p.ldr * 2, 0x00020000);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int m = min(m0 + rl + 32 * k, p.M - 1);
      const int t = m - pos_img(m, p.P) * p.P;
      const int vo = ((t + 1) * (int)p.ldr + n0 + cl) * 2;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        rr[k][nt] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo + 32 * nt, 0, 0));
    }
  }
  f32x2 rc[4], st[4];
  u32x4 ov[4][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    rc[k] = (FL & EPI_RESLN) ? coef[rl + 32 * k] : f32x2{0.f, 0.f};
    st[k] = f32x2{0.f, 0.f};
  }
  const bf16x2 one2 = {(bf16)1.0f, (bf16)1.0f};
  if constexpr (PACK_FIRST) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const f32x4 x = acc[nt][2 * k], y = acc[nt][2 * k + 1];
        const u32x2 xa = __builtin_bit_cast(u32x2, bf16x4{(bf16)x[0], (bf16)x[1], (bf16)x[2], (bf16)x[3]});
        const u32x2 ya = __builtin_bit_cast(u32x2, bf16x4{(bf16)y[0], (bf16)y[1], (bf16)y[2], (bf16)y[3]});
        unsigned x0 = xa[0], x1 = xa[1], y0 = ya[0], y1 = ya[1];
        permlane16_swap(x0, y0);
        permlane16_swap(x1, y1);
        ov[k][nt] = u32x4{x0, x1, y0, y1};
      }
  }
#pragma unroll
  for (int nt = 0; nt < 4 && !PACK_FIRST; ++nt) {
    const int c = cl + 16 * nt;
    f32x4 g[2];
    if (FL & EPI_RESLN) {
#pragma unroll
      for (int h = 0; h < 2; ++h) g[h] = lds4(colb + 256 + c + 4 * h);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f32x4 v[2] = {acc[nt][2 * k], acc[nt][2 * k + 1]};
      if constexpr ((FL & (EPI_RESID | EPI_POS)) != 0) {
        const bf16x8 r8 = __builtin_bit_cast(bf16x8, rr[k][nt]);
        const f32x2 rrow = {rc[k][1], rc[k][1]}, nrm = {-rc[k][1] * rc[k][0], -rc[k][1] * rc[k][0]};
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const f32x2 rv = {(float)r8[4 * h + 2 * q], (float)r8[4 * h + 2 * q + 1]};
            f32x2 a = {v[h][2 * q], v[h][2 * q + 1]};
            if (FL & EPI_RESLN) {  // + gamma (r resid - r mu)   (beta already in the bias)
              const f32x2 t = __builtin_elementwise_fma(rrow, rv, nrm);
              a = __builtin_elementwise_fma(f32x2{g[h][2 * q], g[h][2 * q + 1]}, t, a);
            } else {
              a += rv;
            }
            v[h][2 * q] = a[0];
            v[h][2 * q + 1] = a[1];
          }
      }
      const bf16x8 o = {(bf16)v[0][0], (bf16)v[0][1], (bf16)v[0][2], (bf16)v[0][3],
                        (bf16)v[1][0], (bf16)v[1][1], (bf16)v[1][2], (bf16)v[1][3]};
      ov[k][nt] = __builtin_bit_cast(u32x4, o);
      if (FL & EPI_STATS) {
        if (cok[nt]) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            // (from the bf16x8, not bit_cast(bf16x2, ov[k][nt][e]): hipcc 7.2 then feeds word 0
            // to all four dot2s)
            const bf16x2 w = {o[2 * e], o[2 * e + 1]};
            st[k][0] = __builtin_amdgcn_fdot2_f32_bf16(w, one2, st[k][0], false);
            st[k][1] = __builtin_amdgcn_fdot2_f32_bf16(w, w, st[k][1], false);
          }
        }
      }
    }
  }
  stamp(4);
  // 4. output: per row pair k, the wave's 32 x 64 block goes through its private 4 KiB of LDS
  //    (free during the epilogue: buffer-1 regions 2 / 3 are only DMA'd in the next tile's
  //    phases 1 / 2) and leaves as whole 128-B row segments, 8 rows per store instruction
  {
    const int w = wave;
    // spar: buffer parity of the next tile, whose K-tile 1 (regions 2 / 3 still unloaded) sits in
    // buffer 1 ^ spar
    EVT_LDS char* scr = (EVT_LDS char*)smem - spar * BIG_STAGE +
                        (w < 4 ? (96 + 4 + 8 * w) * 1024 : (72 + (w - 4) * 4 + ((w - 4) >> 1) * 8) * 1024);
    const int wrow = (fg & 1) * 16 + frow;               // store-layout row within the pair
    const int rrow = lane >> 3, rch = lane & 7;          // row-layout lane: row i*8 + rrow, chunk
    const bool rcol_ok = !PADN || interior || n0 + wn * 64 + rch * 8 < p.N;
    __amdgpu_buffer_rsrc_t cs;
    int vo = ((wm * 128 + rrow) * (int)p.ldc + wn * 64 + rch * 8) * 2, orow0 = 0;
    // EPI_HM: this wave's 64 columns are one (part, head) of q | k | v; row m = (b, t) goes to
    // (((b H + h) 3 + part) P + t) 64 + ... of the whole buffer (rows past M land past its end)
    // (lane row base = m0 + wm 128 + rrow as image b0, token t0; the stored rows are base + 8 j,
    // j < 16, at most one image boundary past it for P >= 128, else pos_img per row)
    int hm_b0 = 0, hm_t0 = 0, hm_col = 0, hm_HP = 0, hm_r0 = 0, hm_wrap = 0;
    if constexpr ((FL & EPI_HM) != 0) {
      const int inner = p.N / 3, c0 = n0 + wn * 64;
      const int part = __builtin_amdgcn_readfirstlane(c0 / inner);
      const int h = __builtin_amdgcn_readfirstlane((c0 - part * inner) >> 6);
      hm_HP = 3 * (inner >> 6) * p.P;                      // rows of one image's slices
      hm_col = ((3 * h + part) * p.P * 64 + rch * 8) * 2;  // + ((b 3 H P + t) 64) 2
      const int base = m0 + wm * 128 + rrow;
      hm_b0 = pos_img(base, p.P);
      hm_t0 = base - hm_b0 * p.P;
      hm_r0 = (hm_b0 * hm_HP + hm_t0) * 128 + hm_col;  // the lane's first row; + 8 j rows: + 1 KiB j
      hm_wrap = (hm_HP - p.P) * 128;                   // past the image's last token: the next image
      cs = __builtin_amdgcn_make_buffer_rsrc(p.C, 0, p.M * p.N * 2, 0x00020000);
    } else if constexpr ((FL & EPI_POS) != 0) {  // output rows b*(P+1) + 1 + t, base at tile row 0
      orow0 = __builtin_amdgcn_readfirstlane(pos_orow(m0, p.P));
      const int olast = pos_orow(min(m0 + BIG_BM, p.M) - 1, p.P);
      const int nr = ((olast + 1 - orow0) * (int)p.ldc - n0) * 2;
      cs = __builtin_amdgcn_make_buffer_rsrc((char*)p.C + ((int64_t)orow0 * p.ldc + n0) * 2, 0,
                                             nr, 0x00020000);
    } else {
      cs = tile_rsrc(p.C, p.ldc, p.M, m0, n0);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int ch = 2 * nt + (fg >> 1);
        *(EVT_LDS u32x4*)(scr + wrow * 128 + ((ch ^ (wrow & 7)) << 4)) = ov[k][nt];
      }
      asm volatile("" ::: "memory");  // (a wave's LDS operations execute in order)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = i * 8 + rrow;
        const u32x4 v = *(const EVT_LDS u32x4*)(scr + r * 128 + ((rch ^ (r & 7)) << 4));
        bool keep = rcol_ok;
        if (DBG == 1) {  // ablation: no stores, every value stays live
          keep = (v[0] ^ v[1] ^ v[2] ^ v[3]) == 0x12345u;
        }
        int so = __builtin_amdgcn_readfirstlane((32 * k + 8 * i) * (int)p.ldc * 2), svo = vo;
        if constexpr ((FL & EPI_HM) != 0) {  // per-lane head-major row
          if (p.P >= 128) {  // row offset 8 j (< P): one compare / select per store, j in soffset
            so = __builtin_amdgcn_readfirstlane((32 * k + 8 * i) * 128);
            svo = hm_r0 + (hm_t0 + 32 * k + 8 * i >= p.P ? hm_wrap : 0);
          } else {
            const int m = m0 + wm * 128 + 32 * k + 8 * i + rrow;
            const int b = pos_img(m, p.P), t = m - b * p.P;
            so = 0;
            svo = (b * hm_HP + t) * 128 + hm_col;
          }
        } else if constexpr ((FL & EPI_POS) != 0) {  // per-lane remapped row (rows past M: beyond nr)
          so = 0;
          svo = ((pos_orow(m0 + wm * 128 + 32 * k + 8 * i + rrow, p.P) - orow0) * (int)p.ldc +
                 wn * 64 + rch * 8) * 2;
        }
        if (keep)  // nontemporal (aux nt): whole lines streamed past L2
          buffer_store_b128<2>(v, cs, svo, so);
      }
      asm volatile("" ::: "memory");
    }
  }
  stamp(5);
  if constexpr ((FL & EPI_STATS) != 0) {
    // lanes fg and fg ^ 2 hold the two 32-column halves of the same row
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      st[k][0] += __shfl_xor(st[k][0], 32, 64);
      st[k][1] += __shfl_xor(st[k][1], 32, 64);
    }
    EVT_LDS f32x2* part = (EVT_LDS f32x2*)(smem + PERS_PART) + (wn >> 1) * 256;
    if ((wn & 1) && lane < 32) {
#pragma unroll
      for (int k = 0; k < 4; ++k) part[rl + 32 * k] = st[k];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    big8_bar();
    if (!(wn & 1) && lane < 32) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int m = m0 + rl + 32 * k;
        const f32x2 o = part[rl + 32 * k];
        const int sm = (FL & EPI_POS) ? pos_orow(m, p.P) : m;
        if (interior || m < p.M)
          *(f32x2*)(p.stats_out + 2 * ((int64_t)p.nslots * sm + 2 * tn + (wn >> 1))) = st[k] + o;
      }
    }
  }
}

// Logical walk index -> output tile of the persistent 256 x 256 kernel. Walk index t of round
// r = t / G runs on XCD x of its round slot (blocks b and b + 8 share an XCD; the start index of
// block b is x (G / 8) + (b >> 3), x = b & 7). One group (xgroups <= 1): the rounds sweep the tiles
// m-panel-major, so an XCD's 32 tiles of a round span every weight panel of a wide GEMM (FC1: all
// 12, 4.7 MB, more than its 4 MB L2, fetched again from beyond L2 every round). xgroups = g: the
// XCDs form g groups of 8 / g, group k owns weight panels [k ntiles / g, (k + 1) ntiles / g) for
// the whole launch and walks the m-panels of that slice in the same m-major order, so the slice
// (FC1, g = 2: 2.4 MB) can stay in its XCDs' L2 across rounds while the A panels stream (each A
// panel then read by g XCD groups). Returns whether t names a tile. Which tile a block runs never
// changes a tile's arithmetic (bitwise the same outputs for every xgroups).
__device__ __forceinline__ bool pers_tile(int t, int G, int ntiles, int xgroups, int total, int& tm,
                                          int& tn) {
  if (xgroups <= 1) {
    tm = t / ntiles;
    tn = t - tm * ntiles;
    return t < total;
  }
  const int q = G >> 3, r = t / G, w = t - r * G, x = w / q, l = w - x * q;
  const int xs = 8 / xgroups, k = x / xs, j = (r * xs + (x - k * xs)) * q + l;
  const int ntg = ntiles / xgroups;
  tm = j / ntg;
  tn = k * ntg + (j - tm * ntg);
  return j < total / xgroups;
}

// The persistent tile walk of one GEMM from logical tile `tile` in steps of gridDim.x.
template <int FL, int DBG, bool PADN, typename P = GemmParams>
__device__ __forceinline__ void pers_run(const P& p, int total, int tile, char* smem) {
  // a quarter of the residual before the last K-tile (out-proj 160 -> 153 us); DBG 20: A/B without
  constexpr int ER = ((FL & EPI_RESID) != 0 && DBG != 7 && DBG != 20 && DBG != 18)
                         ? (DBG == 21 ? 1 : 2) : 0;  // DBG 21: A/B with one quarter
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int G = gridDim.x;
  const int nk = p.K / 64;
  const int xg = p.xgroups;
  // the two-phase K-tile for the LN-folded FC1 + GELU kernels (big8_ktile2)
  // (round 6, with the SGPR-base DMA: the two-phase K-tile on every non-residual instance, where
  // it no longer spills, measured equal to this rule: QKV 311.8 vs 311.9 us, r6c A/B)
  constexpr bool KT2 = (FL & EPI_LNIN) && (FL & (EPI_GELU | EPI_GELU_ERF)) &&
                       !(FL & (EPI_RESID | EPI_HM | EPI_STATS | EPI_GATHER | EPI_SPLIT));
  // the two-K-tile steady loop (big8_loop U2) where its doubled body does not spill: not the
  // gathered loaders (Swin PatchMerging, T2T soft splits), the Swin plain-residual epilogue or the
  // column-padded (PADN) instances
  constexpr bool U2 = !PADN && !(FL & (EPI_GATHER | EPI_SPLIT)) &&
                      !((FL & EPI_RESID) && !(FL & EPI_RESLN));
  int tm, tn;
  pers_tile(tile, G, p.ntiles, xg, total, tm, tn);
  if (DBG == 5) {  // experiment: stagger the blocks' start
    const int q = (blockIdx.x >> 3) & 3;
    for (int i = 0; i < q * nk; ++i) __builtin_amdgcn_s_sleep(20);
  }
  pers_coop_dma<FL>(p, smem, wave, lane, tm * BIG_BM, tn * BIG_BN);
  big8_prologue(p, smem, wave, lane, tm * BIG_BM, tn * BIG_BN, nk);
  wait_vmcnt0();  // the first K-tile's waits assume PERS_X younger VMEM ops or a drain
  int par = 0;    // buffer parity of this tile's K-tile 0 (the stream alternates it for odd nk)
  // nk >= 3: per-tile LayerNorm coefficients / next statistics DMA inside the main loop
  const bool early = nk >= 3 && DBG != 16 && DBG != 17;
  int iter = 0;
  auto stamp = [&](int k) {  // DBG 3: timeline of block's tiles (s_memtime, wave 0)
    if ((DBG == 3 || DBG == 5) && tid == 0 && iter < 16)
      ((unsigned long long*)p.pos)[((int64_t)blockIdx.x * 16 + iter) * 8 + k] = __builtin_amdgcn_s_memtime();
  };
  while (true) {
    const int m0 = tm * BIG_BM, n0 = tn * BIG_BN;
    stamp(0);
    f32x4 acc[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int ln = lane;
    asm volatile("" : "+v"(ln));  // per-tile lane addresses: not hoisted out of the tile loop
    u32x4 rre[2][4];  // ER: residual row pair 0 loaded before the last K-tile
    const int next = tile + G;
    int ntm = 0, ntn = 0;
    const bool has_next = pers_tile(next, G, p.ntiles, xg, total, ntm, ntn);
    if (!has_next) ntm = ntn = 0;
    // the next tile's prologue rides in the last K-tiles' idle DMA slots (big8_ktile) as K-tiles
    // nk, nk + 1 of one stream: for odd nk the next tile starts at the other buffer parity
    const bool cont = has_next && nk >= 2 && DBG != 16 && (DBG != 6 || !(nk & 1));
    const int npar = cont ? par ^ (nk & 1) : 0;
    auto last = [&]() {
      if constexpr (ER > 0) pers_resid_early<0, 1>(p, wm, wn, ln, m0, n0, rre);
    };
    auto last3 = [&]() {  // row pair 1 once the n-half-1 fragments are dead (phase 3)
      if constexpr (ER > 1) pers_resid_early<1, 2>(p, wm, wn, ln, m0, n0, rre);
    };
    if (early) {
      // this tile's LayerNorm coefficients by wave group 1 while it waits for group 0's first
      // phase; the next tile's statistics rows / column vectors DMA'd after K-tile 0 (PERS_RAW is
      // free once those coefficients are read: every later phase retires group 1's LDS ops)
      auto pre1 = [&]() { pers_coef<FL>(p, smem, tid - 256); };
      auto mid = [&]() {
        if (has_next) pers_coop_dma<FL>(p, smem, wave, lane, ntm * BIG_BM, ntn * BIG_BN);
      };
      if constexpr (DBG == 18)  // A/B: groups re-synchronised before the epilogue
        big8_loop<PERS_X>(p, smem, acc, wave, ln, wm, wn, m0, n0, nk, cont, ntm * BIG_BM,
                          ntn * BIG_BN, pre1, mid, {}, {}, par);
      else
        big8_loop<PERS_X, true, decltype(pre1), decltype(mid), (ER > 0 ? 4 : 0), decltype(last),
                  (ER > 1 ? 4 : 0), decltype(last3), P, KT2, U2>(
            p, smem, acc, wave, ln, wm, wn, m0, n0, nk, cont, ntm * BIG_BM, ntn * BIG_BN, pre1, mid,
            last, last3, par);
      stamp(1);
      if (has_next && !cont) big8_prologue(p, smem, wave, lane, ntm * BIG_BM, ntn * BIG_BN, nk);
    } else {
      big8_loop<PERS_X, false, NoOp, NoOp, (ER > 0 ? 4 : 0), decltype(last), (ER > 1 ? 4 : 0),
                decltype(last3), P, KT2, U2>(p, smem, acc, wave, ln, wm, wn, m0, n0, nk, cont, ntm * BIG_BM,
                                    ntn * BIG_BN, {}, {}, last, last3, par);
      stamp(1);
      pers_coef<FL>(p, smem, tid);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      big8_bar();
      if (has_next) {
        pers_coop_dma<FL>(p, smem, wave, lane, ntm * BIG_BM, ntn * BIG_BN);
        if (!cont) big8_prologue(p, smem, wave, lane, ntm * BIG_BM, ntn * BIG_BN, nk);
      }
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    stamp(2);
    const bool interior = (m0 + BIG_BM <= p.M) && (n0 + BIG_BN <= p.N);
    if constexpr (DBG == 6)  // A/B: the round-1 epilogue
      pers_epilogue_v1<FL, 0, PADN>(p, smem, acc, wave, wm, wn, m0, n0, tn, lane, interior);
    else
      pers_epilogue<FL, DBG, PADN, ER>(p, smem, acc, wave, wm, wn, m0, n0, tn, lane, interior,
                                       iter, rre, npar);
    stamp(7);
    ++iter;
    if (!has_next) break;
    if (!interior || DBG == 1 || DBG == 2) wait_vmcnt0();
    par = npar;
    tile = next;
    tm = ntm;
    tn = ntn;
  }
}

template <int FL, int DBG = 0, bool PADN = true>
__global__ __launch_bounds__(512, 2) void gemm_pers_kernel(GemmParams p, int total) {
  __shared__ __attribute__((aligned(16))) char smem[PERS_LDS_ALL];
  const int G = gridDim.x;  // XCD-aware order when a multiple of 8
  const int tile = (G & 7) ? (int)blockIdx.x : (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  {
    int tm, tn;
    if (!pers_tile(tile, G, p.ntiles, p.xgroups, total, tm, tn)) return;
  }
  if constexpr ((FL & EPI_GATHER) != 0) {
    MergeParams q;
    static_cast<GemmParams&>(q) = p;
    pers_run<FL, DBG, PADN>(q, total, tile, smem);
  } else if constexpr ((FL & EPI_SPLIT) != 0) {
    UnfoldParams q;
    static_cast<GemmParams&>(q) = p;
    pers_run<FL, DBG, PADN>(q, total, tile, smem);
  } else {
    pers_run<FL, DBG, PADN>(p, total, tile, smem);
  }
}

// ---------------------------------------------------------------------------------------------
// Persistent 128 x 384 kernel (gemm_p384_kernel): the same 8-phase main loop (big8_*, geometry
// GeoOf<P384Params>: 8 waves of 64 x 96, 6 x 4 fragments, A m-halves of 8 KiB and W n-halves of
// 24 KiB per 64 KiB K-tile stage, the same counted waits) for GEMMs whose width is a multiple of
// 384 and whose 256 x 256 grid quantises badly: D = 384 models (T2T-ViT-14, DeiT-small, Swin
// stage 3) have out-proj / FC2 at 1.54 tile rounds with the N = 384 -> 512 padding, and the
// DeiT-base out-proj / FC2 of a strong-scaling shard (64 images: 150 tiles on 256 CUs) leave CUs
// idle; 128 x 384 tiles need no padding and fill the rounds (launch_t's cost rule picks it).
// Epilogue straight from the accumulators as the 256 x 256 one (LN fold, bias, GELU, residual
// LayerNorm, row statistics), rows leaving through a per-wave 3 KiB LDS transpose in four
// 16-row steps: each row's 96 columns = one whole 128-B line + one 64-B half line.
// Statistics: one slot per 128-column slab (3 per tile); slab s of the tile is the sum of exactly
// two waves' partials (wave s, then wave s + 1), the slots past 3 * ntiles written as zero.
// ---------------------------------------------------------------------------------------------
constexpr int P3_RAW = 2 * BIG_STAGE;          // raw LN statistics of the tile rows [128][<=8] f32x2
constexpr int P3_COLRAW = P3_RAW + 8192;       // DMA'd column vectors [3][384] f32
constexpr int P3_COEF = P3_COLRAW + 4608;      // LayerNorm (mu, r) per tile row [128] f32x2
constexpr int P3_COLB = P3_COEF + 1024;        // column vectors of the tile being finished [3][384]
constexpr int P3_PART = P3_COLB + 4608;        // second-wave slab partials [3][128] f32x2
constexpr int P3_LDS_ALL = P3_PART + 3072;
constexpr int P3_X = 12;                       // output stores per wave per interior tile

constexpr bool p384_fl(int fl) {
  return fl == (EPI_BIAS | EPI_RESID | EPI_RESLN | EPI_STATS) ||
         fl == (EPI_BIAS | EPI_RESID | EPI_STATS) || fl == (EPI_LNIN | EPI_BIAS | EPI_GELU) ||
         fl == (EPI_LNIN | EPI_BIAS);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc_rows(const void* mat, int64_t ld, int M,
                                                                int m0, int n0, int rows) {
  m0 = __builtin_amdgcn_readfirstlane(m0);
  n0 = __builtin_amdgcn_readfirstlane(n0);
  const int nr = (min(M - m0, rows) * (int)ld - n0) * 2;
  return __builtin_amdgcn_make_buffer_rsrc((char*)const_cast<void*>(mat) + ((int64_t)m0 * ld + n0) * 2,
                                           0, nr, 0x00020000);
}

template <int FL>
__device__ __forceinline__ void p3_coop_dma(const GemmParams& p, char* smem, int wave, int lane,
                                            int m0, int n0) {
  typedef PersFlags<FL> F;
  asm volatile("" : "+v"(lane));
  if constexpr (F::ln) {
    const float* st = (FL & EPI_LNIN) ? p.stats_in : p.rstats;
    const int half = p.nslots >> 1;  // 16-B chunks per row
    const int nch = 128 * half;      // <= 512
    const int64_t c0 = (int64_t)m0 * half, clast = (int64_t)p.M * half - 1;
    const int c = wave * 64;
    if (c < nch) glds16(st + 4 * min(c0 + c + lane, clast), (EVT_LDS char*)smem + P3_RAW + c * 16);
  }
  const float* v = nullptr;
  if (wave == 0 && F::v0) v = p.bias;
  if (wave == 1 && (FL & EPI_LNIN)) v = p.colsum;
  if (wave == 1 && (FL & EPI_RESLN)) v = p.rgamma;
  if (wave == 2 && F::v2) v = p.rbeta;
  if (v) {  // 384 floats: 96 chunks of 16 B
    EVT_LDS char* d = (EVT_LDS char*)smem + P3_COLRAW + wave * 1536;
    glds16(v + min(n0 + 4 * lane, p.N - 4), d);
    if (lane < 32) glds16(v + min(n0 + 256 + 4 * lane, p.N - 4), d + 1024);
  }
}

// Per-row LayerNorm coefficients of the 128 tile rows and a copy of the 3 x 384 column vectors;
// `tid` in [0, 256) (wave group 1 in the main loop's slot) or [0, 512).
template <int FL>
__device__ __forceinline__ void p3_coef(const GemmParams& p, char* smem, int tid, int nthr) {
  typedef PersFlags<FL> F;
  asm volatile("" : "+v"(tid));
  if constexpr (F::ln) {
    if (tid < 128) {
      const EVT_LDS f32x2* st = (const EVT_LDS f32x2*)(smem + P3_RAW) + tid * p.nslots;
      float s1 = 0.f, s2 = 0.f;
      for (int j = 0; j < p.nslots; ++j) {
        const f32x2 v = st[j];
        s1 += v[0];
        s2 += v[1];
      }
      const float mu = s1 * p.inv_d;
      const float r = rsqrtf(fmaxf(s2 * p.inv_d - mu * mu, 0.f) + p.eps);
      ((EVT_LDS f32x2*)(smem + P3_COEF))[tid] = f32x2{mu, r};
    }
  }
  const EVT_LDS float* src = (const EVT_LDS float*)(smem + P3_COLRAW);
  EVT_LDS float* dst = (EVT_LDS float*)(smem + P3_COLB);
  for (int c = tid; c < 384; c += nthr) {
    if (F::v0) dst[c] = src[c];
    if (F::v1) dst[384 + c] = src[384 + c];
    if (F::v2) dst[768 + c] = src[768 + c];
  }
}

template <int FL>
__device__ __forceinline__ void p3_epilogue(const GemmParams& p, char* smem, f32x4 (&acc)[6][4],
                                            int wave, int wm, int wn, int m0, int n0, int tn,
                                            int lane, int spar) {
  asm volatile("" : "+v"(lane));
  const int frow = lane & 15, fg = lane >> 4;
  const EVT_LDS f32x2* coef = (const EVT_LDS f32x2*)(smem + P3_COEF);
  const EVT_LDS float* colb = (const EVT_LDS float*)(smem + P3_COLB);
  // 1. MFMA layout: row wm*64 + mt*16 + frow, columns wn*96 + nt*16 + 4 fg + j
  if constexpr ((FL & EPI_LNIN) != 0) {
#pragma unroll
    for (int nt = 0; nt < 6; ++nt) {
      const int c = wn * 96 + nt * 16 + 4 * fg;
      const f32x4 b4 = (FL & EPI_BIAS) ? lds4(colb + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 c4 = lds4(colb + 384 + c);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const f32x2 cf = coef[wm * 64 + mt * 16 + frow];
        const f32x2 nmu = {-cf[0], -cf[0]}, rr = {cf[1], cf[1]};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          f32x2 a = {acc[nt][mt][2 * h], acc[nt][mt][2 * h + 1]};
          const f32x2 cs = {c4[2 * h], c4[2 * h + 1]}, bb = {b4[2 * h], b4[2 * h + 1]};
          a = __builtin_elementwise_fma(cs, nmu, a);
          a = __builtin_elementwise_fma(a, rr, bb);
          acc[nt][mt][2 * h] = a[0];
          acc[nt][mt][2 * h + 1] = a[1];
        }
      }
    }
  } else if constexpr ((FL & EPI_BIAS) != 0) {
#pragma unroll
    for (int nt = 0; nt < 6; ++nt) {
      const int c = wn * 96 + nt * 16 + 4 * fg;
      f32x4 b4 = lds4(colb + c);
      if (FL & EPI_RESLN) b4 += lds4(colb + 768 + c);  // + beta of LN(resid)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[nt][mt] += b4;
    }
  }
  if constexpr ((FL & (EPI_GELU | EPI_GELU_ERF)) != 0) {
#pragma unroll
    for (int nt = 0; nt < 6; ++nt)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[nt][mt] = gelu4(acc[nt][mt], (FL & EPI_GELU) ? 0 : 2);
  }
  // 2. row pairs (2k, 2k+1): lane row wm*64 + (2k + (fg & 1))*16 + frow, columns
  //    wn*96 + nt*16 + (fg >> 1)*8 .. + 7
#pragma unroll
  for (int nt = 0; nt < 6; ++nt)
#pragma unroll
    for (int k = 0; k < 2; ++k) swap_rows16(acc[nt][2 * k], acc[nt][2 * k + 1]);
  const int rl = wm * 64 + (fg & 1) * 16 + frow;  // + 32 k
  const int cl = wn * 96 + (fg >> 1) * 8;           // + 16 nt
  u32x4 rr[2][6];
  if constexpr ((FL & EPI_RESID) != 0) {
    const __amdgpu_buffer_rsrc_t rs = tile_rsrc_rows(p.resid, p.ldr, p.M, m0, n0, 128);
    const int vo = (rl * (int)p.ldr + cl) * 2;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int so = __builtin_amdgcn_readfirstlane(32 * k * (int)p.ldr * 2);
#pragma unroll
      for (int nt = 0; nt < 6; ++nt)
        rr[k][nt] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo + 32 * nt, so, 0));
    }
  }
  // 3. values (+ residual), bf16 packing and the per-row statistics of the stored values, split
  //    by 128-column slab: part a = the slab of the wave's first column, part b = the next one
  const int sa = (wn * 96) >> 7;
  f32x2 sta[2], stb[2];
  u32x4 ov[2][6];
  const bf16x2 one2 = {(bf16)1.0f, (bf16)1.0f};
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    sta[k] = f32x2{0.f, 0.f};
    stb[k] = f32x2{0.f, 0.f};
    const f32x2 rc = (FL & EPI_RESLN) ? coef[rl + 32 * k] : f32x2{0.f, 0.f};
#pragma unroll
    for (int nt = 0; nt < 6; ++nt) {
      f32x4 v[2] = {acc[nt][2 * k], acc[nt][2 * k + 1]};
      if constexpr ((FL & EPI_RESID) != 0) {
        const int c = cl + 16 * nt;
        const bf16x8 r8 = __builtin_bit_cast(bf16x8, rr[k][nt]);
        const f32x2 rrow = {rc[1], rc[1]}, nrm = {-rc[1] * rc[0], -rc[1] * rc[0]};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          f32x4 g = f32x4{0.f, 0.f, 0.f, 0.f};
          if (FL & EPI_RESLN) g = lds4(colb + 384 + c + 4 * h);
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const f32x2 rv = {(float)r8[4 * h + 2 * q], (float)r8[4 * h + 2 * q + 1]};
            f32x2 a = {v[h][2 * q], v[h][2 * q + 1]};
            if (FL & EPI_RESLN) {  // + gamma (r resid - r mu)   (beta already in the bias)
              const f32x2 t = __builtin_elementwise_fma(rrow, rv, nrm);
              a = __builtin_elementwise_fma(f32x2{g[2 * q], g[2 * q + 1]}, t, a);
            } else {
              a += rv;
            }
            v[h][2 * q] = a[0];
            v[h][2 * q + 1] = a[1];
          }
        }
      }
      const bf16x8 o = {(bf16)v[0][0], (bf16)v[0][1], (bf16)v[0][2], (bf16)v[0][3],
                        (bf16)v[1][0], (bf16)v[1][1], (bf16)v[1][2], (bf16)v[1][3]};
      ov[k][nt] = __builtin_bit_cast(u32x4, o);
    }
  }
  // 4. output: per row pair k and lane-row half h (16 rows), the wave's 16 x 96 block goes through
  //    its 3 KiB of LDS (the W n-half-1 rows of the next tile's K-tile-1 buffer, not DMA'd before
  //    that tile's phase 1) and leaves as one whole 128-B line + one 64-B half line per row
  {
    EVT_LDS char* scr = (EVT_LDS char*)smem + (spar ^ 1) * BIG_STAGE + Geo<P384Params>::A_TILE +
                        ((wave & 3) * 96 + 48) * ROWB + (wave >> 2) * 3072;
    const __amdgpu_buffer_rsrc_t cs = tile_rsrc_rows(p.C, p.ldc, p.M, m0, n0, 128);
    const int fo = (wn & 1) ? 64 : 0, ho = (wn & 1) ? 0 : 128;  // line / half-line byte offsets
    const int lrow = lane >> 3, lch = lane & 7, hrow = lane >> 2, hch = lane & 3;
    const int wcol = wn * 96 * 2;  // the wave's first column, bytes
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if ((fg & 1) == h) {
#pragma unroll
          for (int nt = 0; nt < 6; ++nt) {
            const int ch = 2 * nt + (fg >> 1);
            *(EVT_LDS u32x4*)(scr + frow * 192 + ch * 16) = ov[k][nt];
          }
        }
        asm volatile("" ::: "memory");  // (a wave's LDS operations execute in order)
        const int r0 = wm * 64 + 32 * k + 16 * h;
        const int so = __builtin_amdgcn_readfirstlane(r0 * (int)p.ldc * 2);
#pragma unroll
        for (int i = 0; i < 2; ++i) {  // whole lines: 8 rows x 128 B per instruction
          const int r = i * 8 + lrow, ch = (fo >> 4) + lch;
          const u32x4 v = *(const EVT_LDS u32x4*)(scr + r * 192 + ch * 16);
          buffer_store_b128<2>(v, cs, r * (int)p.ldc * 2 + wcol + fo + lch * 16, so);
        }
        {  // half lines: 16 rows x 64 B
          const int ch = (ho >> 4) + hch;
          const u32x4 v = *(const EVT_LDS u32x4*)(scr + hrow * 192 + ch * 16);
          buffer_store_b128<2>(v, cs, hrow * (int)p.ldc * 2 + wcol + ho + hch * 16, so);
        }
        asm volatile("" ::: "memory");
      }
  }
  if constexpr ((FL & EPI_STATS) != 0) {
    // statistics of the stored values, after the stores (the slab split selects would otherwise
    // be scheduled between a wide store and its fence)
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int nt = 0; nt < 6; ++nt) {
        const bool inb = ((wn * 96 + nt * 16) >> 7) != sa;  // wave-uniform
        const bf16x8 o = __builtin_bit_cast(bf16x8, ov[k][nt]);
        f32x2 s = {0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          // (from the bf16x8, not bit_cast(bf16x2, ov[k][nt][e]): see pers_epilogue)
          const bf16x2 w = {o[2 * e], o[2 * e + 1]};
          s[0] = __builtin_amdgcn_fdot2_f32_bf16(w, one2, s[0], false);
          s[1] = __builtin_amdgcn_fdot2_f32_bf16(w, w, s[1], false);
        }
        if (inb) stb[k] += s;
        else sta[k] += s;
      }
    // lanes fg and fg ^ 2 hold the two 8-column halves of the same row's 16-column groups
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      sta[k][0] += __shfl_xor(sta[k][0], 32, 64);
      sta[k][1] += __shfl_xor(sta[k][1], 32, 64);
      stb[k][0] += __shfl_xor(stb[k][0], 32, 64);
      stb[k][1] += __shfl_xor(stb[k][1], 32, 64);
    }
    // slab s = first part (wave s: a for s = 0, b otherwise) + second (wave s + 1, its part a)
    EVT_LDS f32x2* part = (EVT_LDS f32x2*)(smem + P3_PART);
    if (wn >= 1 && lane < 32) {
#pragma unroll
      for (int k = 0; k < 2; ++k) part[(wn - 1) * 128 + wm * 64 + 32 * k + lane] = sta[k];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    big8_bar();
    if (lane < 32) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int m = m0 + wm * 64 + 32 * k + lane;
        if (m < p.M) {
          float* so = p.stats_out + 2 * (int64_t)p.nslots * m;
          if (wn <= 2) {
            const f32x2 o = part[wn * 128 + wm * 64 + 32 * k + lane];
            *(f32x2*)(so + 2 * (3 * tn + wn)) = (wn == 0 ? sta[k] : stb[k]) + o;
          } else if (tn == p.ntiles - 1) {  // slots past the last tile's slabs: zero
            for (int s = 3 * p.ntiles; s < p.nslots; ++s) *(f32x2*)(so + 2 * s) = f32x2{0.f, 0.f};
          }
        }
      }
    }
  }
}

template <int FL>
__device__ __forceinline__ void p3_run(const P384Params& p, int total, int tile, char* smem) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int G = gridDim.x;
  const int nk = p.K / 64;
  int tm = tile / p.ntiles, tn = tile - tm * p.ntiles;
  p3_coop_dma<FL>(p, smem, wave, lane, tm * 128, tn * 384);
  big8_prologue(p, smem, wave, lane, tm * 128, tn * 384, nk);
  wait_vmcnt0();  // the first K-tile's waits assume P3_X younger VMEM ops or a drain
  int par = 0;
  const bool early = nk >= 3;
  while (true) {
    const int m0 = tm * 128, n0 = tn * 384;
    f32x4 acc[6][4];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int next = tile + G;
    const bool has_next = next < total;
    int ntm = 0, ntn = 0;
    if (has_next) {
      ntm = next / p.ntiles;
      ntn = next - ntm * p.ntiles;
    }
    const bool cont = has_next && nk >= 2;
    const int npar = cont ? par ^ (nk & 1) : 0;
    if (early) {
      auto pre1 = [&]() { p3_coef<FL>(p, smem, tid - 256, 256); };
      auto mid = [&]() {
        if (has_next) p3_coop_dma<FL>(p, smem, wave, lane, ntm * 128, ntn * 384);
      };
      big8_loop<P3_X, true, decltype(pre1), decltype(mid), 0, NoOp, 0, NoOp, P384Params>(
          p, smem, acc, wave, ln, wm, wn, m0, n0, nk, cont, ntm * 128, ntn * 384, pre1, mid, {}, {},
          par);
      if (has_next && !cont) big8_prologue(p, smem, wave, lane, ntm * 128, ntn * 384, nk);
    } else {
      big8_loop<P3_X, false, NoOp, NoOp, 0, NoOp, 0, NoOp, P384Params>(
          p, smem, acc, wave, ln, wm, wn, m0, n0, nk, cont, ntm * 128, ntn * 384, {}, {}, {}, {},
          par);
      p3_coef<FL>(p, smem, tid, 512);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      big8_bar();
      if (has_next) {
        p3_coop_dma<FL>(p, smem, wave, lane, ntm * 128, ntn * 384);
        if (!cont) big8_prologue(p, smem, wave, lane, ntm * 128, ntn * 384, nk);
      }
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    p3_epilogue<FL>(p, smem, acc, wave, wm, wn, m0, n0, tn, lane, npar);
    if (!has_next) break;
    if (m0 + 128 > p.M) wait_vmcnt0();  // edge tile: fewer stores than P3_X issued
    par = npar;
    tile = next;
    tm = ntm;
    tn = ntn;
  }
}

template <int FL>
__global__ __launch_bounds__(512, 2) void gemm_p384_kernel(GemmParams p, int total) {
  __shared__ __attribute__((aligned(16))) char smem[P3_LDS_ALL];
  const int G = gridDim.x;  // XCD-aware order when a multiple of 8
  const int tile = (G & 7) ? (int)blockIdx.x : (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  if (tile >= total) return;
  P384Params q;
  static_cast<GemmParams&>(q) = p;
  p3_run<FL>(q, total, tile, smem);
}

// ---------------------------------------------------------------------------------------------
// Stream-K persistent kernel. The persistent kernel above runs every CU through identical tiles
// in lock step, so all 256 epilogues (32 MB of output stores, plus 32 MB of residual loads for
// out-proj / FC2) hit HBM in the same few microseconds while it idles during the main loops:
// measured (scripts/probe/pers_timeline.py) 10k of a 51k-cycle FC1 tile and 25k of a 60k-cycle
// out-proj tile are epilogue, HBM-write bound. Here the K-iterations of all tiles (total * nk)
// are split evenly over the G blocks: block r (XCD-major rank) takes the contiguous range
// [r I / G, (r+1) I / G). Ranges start part-way through a tile, so tile boundaries - and with
// them the epilogue bursts - are spread uniformly over the tile period across CUs, and the tail
// quantisation of the tile grid disappears (out-proj / FC2: 4.62 tiles per CU, not 5).
// A tile cut by a range boundary (at most two parts: requires total >= G) is finished by
// whichever of its two blocks gets there second:
//   flag[b] (b = the boundary's upper rank) 0 -> 1 by CAS (first arriver), which writes its fp32
//   partial accumulators to slot b (write-through sc1 stores, every wave drained, barrier) and
//   sets 2; the second arriver polls for 2 (the first is running, so this always completes),
//   resets the flag to 0 (self-cleaning: every flag is 0 again at kernel end), adds the partial
//   (sc1 loads) and runs the normal epilogue. The LayerNorm fold / bias / residual are applied
//   once, to the summed accumulators. Results are deterministic for a given (M, N, K, G); a split
//   tile sums its two K ranges in a different order than an unsplit one (fp32 reassociation).
// ---------------------------------------------------------------------------------------------
constexpr int SK_ROLE = PERS_LDS;          // LDS word: CAS result broadcast
constexpr int SK_LDS = PERS_LDS + 16;
constexpr int SK_SLOT_FLOATS = 256 * 256;  // fp32 partial tile per boundary

__device__ __forceinline__ __amdgpu_buffer_rsrc_t sk_rsrc(float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, SK_SLOT_FLOATS * 4, 0x00020000);
}

template <int FL>
__global__ __launch_bounds__(512, 2) void gemm_sk_kernel(GemmParams p, int total) {
  __shared__ __attribute__((aligned(16))) char smem[SK_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int G = gridDim.x;  // multiple of 8: ranks of one XCD are consecutive (shared A panels)
  const int r = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  const int nk = p.K / 64;
  const int64_t I = (int64_t)total * nk;
  int64_t it = I * r / G;
  const int64_t end = I * (r + 1) / G;
  // work item: K-tiles [kb, ke) of tile t; operands shifted to kb
  auto decode = [&](int64_t i, int& t, int& kb, int& ke) {
    t = (int)(i / nk);
    kb = (int)(i - (int64_t)t * nk);
    ke = (int)min<int64_t>(nk, kb + (end - i));
  };
  auto shifted = [&](int kb) {
    GemmParams q = p;
    q.A = (const bf16*)p.A + kb * 64;
    q.W = (const bf16*)p.W + kb * 64;
    return q;
  };
  int t, kb, ke;
  decode(it, t, kb, ke);
  int tm = t / p.ntiles, tn = t - tm * p.ntiles;
  pers_coop_dma<FL>(p, smem, wave, lane, tm * BIG_BM, tn * BIG_BN);
  big8_prologue(shifted(kb), smem, wave, lane, tm * BIG_BM, tn * BIG_BN, ke - kb);
  wait_vmcnt0();
  while (true) {
    const int m0 = tm * BIG_BM, n0 = tn * BIG_BN;
    f32x4 acc[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int ln = lane;
    asm volatile("" : "+v"(ln));
    big8_loop<PERS_X>(shifted(kb), smem, acc, wave, ln, wm, wn, m0, n0, ke - kb);
    pers_coef<FL>(p, smem, tid);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    big8_bar();
    const int64_t nit = it + (ke - kb);
    const bool has_next = nit < end;
    int nt_ = 0, nkb = 0, nke = 0, ntm = 0, ntn = 0;
    if (has_next) {
      decode(nit, nt_, nkb, nke);
      ntm = nt_ / p.ntiles;
      ntn = nt_ - ntm * p.ntiles;
      pers_coop_dma<FL>(p, smem, wave, lane, ntm * BIG_BM, ntn * BIG_BN);
      big8_prologue(shifted(nkb), smem, wave, lane, ntm * BIG_BM, ntn * BIG_BN, nke - nkb);
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const bool interior = (m0 + BIG_BM <= p.M) && (n0 + BIG_BN <= p.N);
    const bool whole = kb == 0 && ke == nk;
    bool finish = whole;
    if (!whole) {
      const int b = kb > 0 ? r : r + 1;  // boundary inside this tile
      int* flag = p.sk_flags + b;
      const __amdgpu_buffer_rsrc_t rs = sk_rsrc(p.sk_part + (int64_t)b * SK_SLOT_FLOATS);
      const int off0 = (wave * 32 * 64 + lane) * 16;  // + (nt * 8 + mt) * 1024
      if (tid == 0) {
        int expect = 0;
        __hip_atomic_compare_exchange_strong(flag, &expect, 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        *(EVT_LDS int*)(smem + SK_ROLE) = expect;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      big8_bar();
      finish = *(const EVT_LDS int*)(smem + SK_ROLE) != 0;
      if (!finish) {  // first arriver: publish the partial
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int mt = 0; mt < 8; ++mt)
            buffer_store_b128<16>(__builtin_bit_cast(u32x4, acc[nt][mt]), rs, off0,
                                  (nt * 8 + mt) * 1024);
        wait_vmcnt0();  // every storing wave drained
        big8_bar();
        if (tid == 0) __hip_atomic_store(flag, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {  // second arriver: wait for the partial and add it
        if (tid == 0) {  // bounded (~1 s): a corrupted flag block must not hang the GPU
          for (int i = 0; i < (1 << 23); ++i) {
            if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 2) break;
            __builtin_amdgcn_s_sleep(2);
          }
          __hip_atomic_store(flag, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        big8_bar();
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int h = 0; h < 2; ++h) {  // 4 loads in flight: bounded register footprint
            u32x4 v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
              v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, off0, (nt * 8 + h * 4 + j) * 1024, 16);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[nt][h * 4 + j] += __builtin_bit_cast(f32x4, v[j]);
            __builtin_amdgcn_sched_barrier(0);
          }
      }
    }
    if (finish) pers_epilogue<FL>(p, smem, acc, wave, wm, wn, m0, n0, tn, lane, interior);
    if (!whole || !interior) wait_vmcnt0();
    if (!has_next) break;
    it = nit;
    t = nt_;
    kb = nkb;
    ke = nke;
    tm = ntm;
    tn = ntn;
  }
}

template <int FL>
hipError_t launch_big(const GemmParams& p, hipStream_t s) {
  const int mtiles = (p.M + BIG_BM - 1) / BIG_BM;
  GemmParams q = p;
  q.ntiles = (p.ntiles * GEMM_BN) / BIG_BN;
  const dim3 grid(mtiles * q.ntiles);
  if (g_gemm_variant == 2)
    hipLaunchKernelGGL((gemm_big_kernel<FL, 0>), grid, dim3(512), 0, s, q);
  else if (g_gemm_variant == 8)
    hipLaunchKernelGGL((gemm_big_kernel<FL, 8>), grid, dim3(512), 0, s, q);
#ifdef EVT_GEMM_LAB
  else if (g_gemm_variant == 106)
    hipLaunchKernelGGL((gemm_big_kernel<FL, 6, true>), grid, dim3(512), 0, s, q);
  else if (g_gemm_variant == 108)
    hipLaunchKernelGGL((gemm_big_kernel<FL, 8, true>), grid, dim3(512), 0, s, q);
#endif
  else if constexpr ((FL & EPI_POS) != 0)  // patch embedding: 8-phase loop (153 vs 179 us, bs512)
    hipLaunchKernelGGL((gemm_big_kernel<FL, 8>), grid, dim3(512), 0, s, q);
  else
    hipLaunchKernelGGL((gemm_big_kernel<FL, 6>), grid, dim3(512), 0, s, q);
  return hipGetLastError();
}

int g_num_cus = 0;
// persistent grid balancing (launch_pers): 1 = for launches of 2-4 tile rounds (default),
// 0 = never, 2 = always; EVT_GRID_BALANCE, read once (A/B switch)
const int g_grid_balance = [] {
  const char* e = std::getenv("EVT_GRID_BALANCE");
  return (e && e[0] >= '0' && e[0] <= '2') ? e[0] - '0' : 1;
}();

int num_cus() {
  if (!g_num_cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  return g_num_cus;
}


constexpr bool pers_fl(int fl) {
  return fl == 0 || fl == EPI_BIAS || fl == (EPI_BIAS | EPI_GELU) || fl == (EPI_LNIN | EPI_BIAS) ||
         fl == (EPI_BIAS | EPI_POS | EPI_STATS) ||
         fl == (EPI_LNIN | EPI_BIAS | EPI_GELU) ||
         fl == (EPI_BIAS | EPI_RESID | EPI_RESLN | EPI_STATS) ||
         fl == (EPI_LNIN | EPI_BIAS | EPI_GELU_ERF) || fl == (EPI_BIAS | EPI_RESID | EPI_STATS) ||
         fl == (EPI_LNIN | EPI_BIAS | EPI_STATS) ||
         fl == (EPI_LNIN | EPI_BIAS | EPI_STATS | EPI_GATHER) ||
         fl == (EPI_LNIN | EPI_BIAS | EPI_SPLIT) || fl == (EPI_BIAS | EPI_POS | EPI_STATS | EPI_SPLIT) ||
         fl == (EPI_LNIN | EPI_BIAS | EPI_HM);
}

// persistent kernel: supported epilogue, 8-column output groups, LN rows of <= 8 slots
bool gemm_lab_pers_variant(int v) {
#ifdef EVT_GEMM_LAB
  return v == 10 || v == 11 || v == 13 || v == 15 || (v >= 17 && v <= 25);
#else
  (void)v;
  return false;
#endif
}

bool use_pers(const GemmParams& p, int flags) {
  const int v = g_gemm_variant;
  if (v != 0 && v != 9 && v != 16 && v != 31 && v != 36 && !gemm_lab_pers_variant(v))
    return false;
  // timeline variants stamp s_memtime through p.pos: never on the patch GEMM (p.pos = the table)
  if ((v == 13 || v == 15) && (flags & EPI_POS)) return false;
  if (p.N % 8 || p.vec_ok < 2) return false;
  if ((flags & (EPI_LNIN | EPI_RESLN)) && (p.nslots > 8 || p.nslots % 2 || p.stats_step > 1))
    return false;
  // POS: the bf16 copy of the position table rides in resid / ldr (else the staged-epilogue kernel)
  if ((flags & EPI_POS) && (!p.resid || p.ldr % 8 || p.P <= 0 || p.M >= (1 << 22))) return false;
  return true;
}

// XCD groups of the persistent walk (pers_tile): 2 where the weight panels split evenly over
// two groups of four XCDs and the launch has more than one round (FC1 of the D = 768 models: 12
// panels -> 6 per group; measured round 4: one group 484.5 us, two 479.9, four 479.3 per FC1 launch)
int pers_xgroups(int ntiles, int G, int total) {
  if (G != 256 || total <= G) return 1;  // the walk arithmetic assumes 8 XCDs of 32 blocks
  return (ntiles % 2 == 0 && ntiles / 2 >= 3) ? 2 : 1;
}

template <int FL>
hipError_t launch_pers(const GemmParams& p, hipStream_t s) {
  num_cus();
  GemmParams q = p;
  q.ntiles = (p.ntiles * GEMM_BN) / BIG_BN;
  const int total = ((p.M + BIG_BM - 1) / BIG_BM) * q.ntiles;
  int G = min(total, g_gemm_variant == 10 ? 8 : g_num_cus);  // 10: few blocks, many tiles each
  if (G >= 8 && total > G) G &= ~7;
  // 2-4 tile rounds: as few blocks as keep the round count (multiple of 8), every block the same
  // number of tiles. Measured round 6 (r6f, alternating): DeiT-base at 64 images 22.67k -> 23.30k
  // img/s (FC1 600 tiles: 200 blocks x 3 instead of 256 with 88 taking a third; QKV 450: 232 x 2),
  // the CUs left idle let the busy ones hold a higher clock; at 512 images (>= 5 rounds) -0.3 %,
  // not applied there. evt_set_gemm_variant 36: never (the tile -> block assignment only: bitwise
  // the same outputs); EVT_GRID_BALANCE=0 / 2: never / always (A/B)
  const int rounds = (total + G - 1) / G;
  const int bal = (g_gemm_variant == 36 || p.no_balance) ? 0 : g_grid_balance;
  if (total > G && G >= 8 && (bal == 2 || (bal == 1 && rounds <= 4)))
    G = min(G, (((total + rounds - 1) / rounds) + 7) & ~7);
  // one round (one block per tile): up to a multiple of 8 blocks (the surplus exits at once) so
  // that the XCD-major start order applies and an m-panel's n-tiles run on one XCD, its A panel
  // fetched once into that L2 (DeiT-base FC2 at 64 images: 150 tiles, 3 per 1.5 MB A panel; in
  // block order the 3 went to 3 XCDs: 292 MB fetched per launch for ~100 MB of operands)
  else if (total <= G && (G & 7) && ((G + 7) & ~7) <= max(g_num_cus, 8)) G = (G + 7) & ~7;
  q.xgroups = pers_xgroups(q.ntiles, G, total);
  if (false) {
  }
#ifdef EVT_GEMM_LAB
  else if (g_gemm_variant == 11)
    hipLaunchKernelGGL((gemm_pers_kernel<FL, 1>), dim3(G), dim3(512), 0, s, q, total);
  else if (g_gemm_variant == 13)  // timeline probe: p.pos = u64 [blocks][16][8]
    hipLaunchKernelGGL((gemm_pers_kernel<FL, 3>), dim3(G), dim3(512), 0, s, q, total);
  else if (g_gemm_variant == 15)  // timeline probe + staggered block start
    hipLaunchKernelGGL((gemm_pers_kernel<FL, 5>), dim3(G), dim3(512), 0, s, q, total);
  else if (g_gemm_variant == 19)  // A/B: round-1 epilogue
    hipLaunchKernelGGL((gemm_pers_kernel<FL, 6, false>), dim3(G), dim3(512), 0, s, q, total);
  else if (g_gemm_variant == 17)  // ablation: main loop + tile loop only (no epilogue)
    hipLaunchKernelGGL((gemm_pers_kernel<FL, 2, false>), dim3(G), dim3(512), 0, s, q, total);
  else if (g_gemm_variant == 23)  // A/B: wave groups re-synchronised before the epilogue
    hipLaunchKernelGGL((gemm_pers_kernel<FL, 18, false>), dim3(G), dim3(512), 0, s, q, total);
  else if (g_gemm_variant == 22)  // A/B: LN coefficients / statistics DMA after the main loop
    hipLaunchKernelGGL((gemm_pers_kernel<FL, 17, false>), dim3(G), dim3(512), 0, s, q, total);
  else if (g_gemm_variant == 21)  // A/B: next-tile prologue issued after the main loop
    hipLaunchKernelGGL((gemm_pers_kernel<FL, 16, false>), dim3(G), dim3(512), 0, s, q, total);
  else if (g_gemm_variant == 24)  // A/B: the whole residual loaded in the epilogue
    hipLaunchKernelGGL((gemm_pers_kernel<FL, 20, false>), dim3(G), dim3(512), 0, s, q, total);
  else if (g_gemm_variant == 25)  // A/B: one residual quarter early (not two)
    hipLaunchKernelGGL((gemm_pers_kernel<FL, 21, false>), dim3(G), dim3(512), 0, s, q, total);
  else if (g_gemm_variant == 20)  // ablation: no residual loads (out-proj 153 -> 115 us)
    hipLaunchKernelGGL((gemm_pers_kernel<FL, 7, false>), dim3(G), dim3(512), 0, s, q, total);
  else if (g_gemm_variant == 18)  // ablation: epilogue without the GELU
    hipLaunchKernelGGL((gemm_pers_kernel<(FL & ~(EPI_GELU | EPI_GELU_ERF)), 0, false>), dim3(G),
                       dim3(512), 0, s, q, total);
#endif
  else if (p.N % BIG_BN == 0)
    hipLaunchKernelGGL((gemm_pers_kernel<FL, 0, false>), dim3(G), dim3(512), 0, s, q, total);
  else
    hipLaunchKernelGGL((gemm_pers_kernel<FL>), dim3(G), dim3(512), 0, s, q, total);
  return hipGetLastError();
}

// 128 x 384 persistent tiles (gemm_p384_kernel) where the width is a multiple of 384 and their
// tile rounds cost less than the 256 x 256 grid's: rounds x tile work, a 128 x 384 tile = 0.75 of
// a 256 x 256 one (e.g. T2T-ViT-14 out-proj / FC2: 2 x 0.75 against 2 rounds of half-padded
// tiles; DeiT-base out-proj / FC2 at 64 images: 1 x 0.75 against one round on 150 CUs).
// evt_set_gemm_variant 30 forces it wherever it applies, 31 never.
bool use_p384(const GemmParams& p, int flags) {
  const int v = g_gemm_variant;
  if ((v != 0 && v != 30) || p.N % 384 || p.vec_ok < 2 || p.K < 64) return false;
  if (std::max(std::max(p.lda, p.ldw), std::max(p.ldc, p.resid ? p.ldr : (int64_t)0)) > BIG_MAX_LD)
    return false;
  if ((flags & (EPI_LNIN | EPI_RESLN)) && (p.nslots > 8 || p.nslots % 2 || p.stats_step > 1))
    return false;
  if ((flags & EPI_STATS) && 3 * (p.N / 384) > p.nslots) return false;
  // automatic selection: never. Measured (round 4, rocprofv3, same box): a 128 x 384 tile takes
  // as long per K-tile as a 256 x 256 one (the main loop is bound by its 8 LDS-DMA instructions
  // per wave per K-tile, the same for both shapes, not by its MFMAs), so 0.75 of the work runs at
  // 0.75 of the FLOP rate: T2T-ViT-14 out-proj / FC2 53.1 vs 52.8 us, Swin-T 65.2 vs 65.1 us,
  // DeiT-base at 64 images 80.8 vs 70.6 us (128x128). Kept as the forced diagnostic variant 30.
  return v == 30;
}

template <int FL>
hipError_t launch_p384(const GemmParams& p, hipStream_t s) {
  GemmParams q = p;
  q.ntiles = p.N / 384;
  const int total = ((p.M + 127) / 128) * q.ntiles;
  int G = min(total, num_cus());
  if (G >= 8 && total > G) G &= ~7;
  hipLaunchKernelGGL((gemm_p384_kernel<FL>), dim3(G), dim3(512), 0, s, q, total);
  return hipGetLastError();
}

constexpr int SK_MAX_G = 256;

int sk_grid() { return min(num_cus(), SK_MAX_G) & ~7; }

// stream-K: scratch bound, auto (0) or forced (16), every range of K-iterations at least one
// tile long (each tile has at most two parts)
bool use_sk(const GemmParams& p) {
  // explicit diagnostic only: an automatic stream-K split breaks bitwise batch-position
  // independence ("Stream-K for the 1.5-round D = 384 GEMMs")
  if (!p.sk_flags || !p.sk_part || g_gemm_variant != 16) return false;
  const int G = sk_grid();
  const int total = ((p.M + BIG_BM - 1) / BIG_BM) * ((p.ntiles * GEMM_BN) / BIG_BN);
  return G >= 8 && total >= G;
}

template <int FL>
hipError_t launch_sk(const GemmParams& p, hipStream_t s) {
  GemmParams q = p;
  q.ntiles = (p.ntiles * GEMM_BN) / BIG_BN;
  const int total = ((p.M + BIG_BM - 1) / BIG_BM) * q.ntiles;
  hipLaunchKernelGGL((gemm_sk_kernel<FL>), dim3(sk_grid()), dim3(512), 0, s, q, total);
  return hipGetLastError();
}

bool headmajor_fits(const GemmParams& p) {
  return p.N % 192 == 0 && p.P > 0 && p.M % p.P == 0 && p.M < (1 << 22) &&
         (int64_t)p.M * p.N * 2 < ((int64_t)1 << 31) && g_gemm_variant != 16 && g_gemm_variant != 30;
}

template <typename T, int FL>
hipError_t launch_t(const GemmParams& p, hipStream_t s) {
  if constexpr ((FL & EPI_HM) != 0) {  // head-major store: the persistent kernel or nothing
    if constexpr (std::is_same<T, bf16>::value && pers_fl(FL)) {
      if (headmajor_fits(p) && use_big(p, FL) && use_pers(p, FL)) return launch_pers<FL>(p, s);
    }
    return hipErrorNotSupported;
  } else if constexpr ((FL & (EPI_GATHER | EPI_SPLIT)) != 0) {  // gathering loader: persistent kernel
    if constexpr (std::is_same<T, bf16>::value) {
      constexpr bool MERGE = (FL & EPI_GATHER) != 0;
      const bool merge = MERGE && p.gmode == 1 && p.gR % 2 == 0 && p.gOW == p.gR / 2 &&
                         p.gC % 8 == 0 && p.K == 4 * p.gC;
      const bool unfold = !MERGE && p.gmode == 2 && p.gC == 64 && p.K == 9 * 64 && p.gzero &&
                          p.gOW == (p.gR + 1) / 2;
      // the gathered loaders decode rows with float reciprocals: exact for rows < 2^22
      if ((merge || unfold) && p.gR > 0 && p.M < (1 << 22) && use_big(p, FL) && use_pers(p, FL) &&
          !use_sk(p))
        return launch_pers<FL>(p, s);
    }
    return hipErrorNotSupported;
  } else {
    if constexpr (std::is_same<T, bf16>::value) {
      if constexpr (p384_fl(FL)) {
        if (use_p384(p, FL)) return launch_p384<FL>(p, s);
      }
      if (use_big(p, FL)) {
        if constexpr (pers_fl(FL)) {
          if (use_pers(p, FL)) return use_sk(p) ? launch_sk<FL>(p, s) : launch_pers<FL>(p, s);
        }
        return launch_big<FL>(p, s);
      }
    }
    const int mtiles = (p.M + GEMM_BM - 1) / GEMM_BM;
    hipLaunchKernelGGL((gemm_nt_kernel<T, FL>), dim3(mtiles * p.ntiles), dim3(256), 0, s, p);
    return hipGetLastError();
  }
}

template <typename T>
hipError_t dispatch(int flags, const GemmParams& p, hipStream_t s) {
  switch (flags) {
#define EVT_CASE(F) \
  case (F): return launch_t<T, (F)>(p, s);
    EVT_CASE(0)                                              // plain (op-level)
    EVT_CASE(EPI_BIAS)
    EVT_CASE(EPI_BIAS | EPI_GELU)                            // head1
    EVT_CASE(EPI_BIAS | EPI_OUT_F32)                         // head2 (logits)
    EVT_CASE(EPI_BIAS | EPI_RESID | EPI_OUT_F32)             // op-level residual
    EVT_CASE(EPI_BIAS | EPI_POS | EPI_OUT_F32)               // op-level patch embed
    EVT_CASE(EPI_BIAS | EPI_POS | EPI_STATS)                 // patch embed -> stream + stats
    EVT_CASE(EPI_LNIN | EPI_BIAS)                            // LN1-folded QKV
    EVT_CASE(EPI_LNIN | EPI_BIAS | EPI_GELU)                 // LN2-folded FC1 + GELU
    EVT_CASE(EPI_LNIN | EPI_BIAS | EPI_OUT_F32)              // LN-folded classifier (T2T)
    EVT_CASE(EPI_BIAS | EPI_RESID | EPI_RESLN | EPI_STATS)   // out-proj / FC2 + LN residual
    EVT_CASE(EPI_LNIN | EPI_BIAS | EPI_GELU_ERF)             // Swin LN2-folded FC1 + erf GELU
    EVT_CASE(EPI_LNIN | EPI_BIAS | EPI_STATS | EPI_GATHER)   // Swin PatchMerging (gathered A)
    EVT_CASE(EPI_LNIN | EPI_BIAS | EPI_SPLIT)                // T2T soft_split1 + kqv (gathered A)
    EVT_CASE(EPI_BIAS | EPI_POS | EPI_STATS | EPI_SPLIT)     // T2T soft_split2 + project
    EVT_CASE(EPI_BIAS | EPI_RESID | EPI_STATS)               // Swin proj / FC2 + plain residual
    EVT_CASE(EPI_LNIN | EPI_BIAS | EPI_STATS)                // Swin LN-folded patch-merge reduction
    EVT_CASE(EPI_LNIN | EPI_BIAS | EPI_HM)                   // LN1-folded QKV, head-major output
#undef EVT_CASE
    default: return hipErrorInvalidValue;
  }
}

// out[m][n] = epilogue(sum_z part[z][m][n] + bias[n]), z in order (4 columns per thread)
template <typename T, bool GELU>
__global__ void splitk_reduce_kernel(const float* __restrict__ part, int S, int64_t stride,
                                     int ldp, const float* __restrict__ bias, T* __restrict__ out,
                                     int64_t ldo, int M, int N) {
  const int n4 = (N + 3) >> 2;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)M * n4) return;
  const int m = (int)(i / n4), n = (int)(i - (int64_t)m * n4) * 4;
  f32x4 v = *(const f32x4*)(part + (int64_t)m * ldp + n);
  for (int z = 1; z < S; ++z) v += *(const f32x4*)(part + z * stride + (int64_t)m * ldp + n);
  if (bias) v += *(const f32x4*)(bias + n);  // bias: >= ntiles*128 floats (zero padded)
  if (GELU) v = gelu4(v, 0);
  for (int j = 0; j < 4; ++j)
    if (n + j < N) out[(int64_t)m * ldo + n + j] = (T)v[j];
}

template <typename T>
hipError_t splitk_t(int flags, const GemmParams& p, int S, float* part, hipStream_t s) {
  GemmParams q = p;
  const int ldp = p.ntiles * GEMM_BN;
  q.ks_chunk = p.K / S;
  q.ks_stride = (int64_t)p.M * ldp;
  q.C = part;
  q.ldc = ldp;
  q.N = ldp;
  q.vec_ok = 2;
  q.bias = nullptr;
  const int mtiles = (p.M + GEMM_BM - 1) / GEMM_BM;
  hipLaunchKernelGGL((gemm_nt_kernel<T, EPI_OUT_F32>), dim3(mtiles * p.ntiles, S), dim3(256), 0, s, q);
  const int64_t n = (int64_t)p.M * ((p.N + 3) / 4);
  const dim3 grid((unsigned)((n + 255) / 256));
  const bool gelu = (flags & EPI_GELU) != 0;
  if (flags & EPI_OUT_F32) {
    if (gelu)
      hipLaunchKernelGGL((splitk_reduce_kernel<float, true>), grid, dim3(256), 0, s, part, S,
                         q.ks_stride, ldp, p.bias, (float*)p.C, p.ldc, p.M, p.N);
    else
      hipLaunchKernelGGL((splitk_reduce_kernel<float, false>), grid, dim3(256), 0, s, part, S,
                         q.ks_stride, ldp, p.bias, (float*)p.C, p.ldc, p.M, p.N);
  } else {
    if (gelu)
      hipLaunchKernelGGL((splitk_reduce_kernel<T, true>), grid, dim3(256), 0, s, part, S,
                         q.ks_stride, ldp, p.bias, (T*)p.C, p.ldc, p.M, p.N);
    else
      hipLaunchKernelGGL((splitk_reduce_kernel<T, false>), grid, dim3(256), 0, s, part, S,
                         q.ks_stride, ldp, p.bias, (T*)p.C, p.ldc, p.M, p.N);
  }
  return hipGetLastError();
}


// Wp[n][k] = W[k][n] * (scale ? scale[k] : 1) (fp32 [K][N] in) converted to T, zero outside
// [N) x [K). `scale` folds a LayerNorm gamma into the weight rows.
template <typename T>
__global__ void pack_kernel(const float* __restrict__ W, const float* __restrict__ scale, int K,
                            int N, T* __restrict__ Wp, int Kpad, int Npad) {
  __shared__ float tile[32][33];
  const int k0 = blockIdx.x * 32, n0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 8 rows per pass
  for (int r = ty; r < 32; r += 8) {
    const int k = k0 + r, n = n0 + tx;
    tile[r][tx] = (k < K && n < N) ? W[(int64_t)k * N + n] * (scale ? scale[k] : 1.f) : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int n = n0 + r, k = k0 + tx;
    if (n < Npad && k < Kpad) Wp[(int64_t)n * Kpad + k] = from_f32<T>(tile[tx][r]);
  }
}

// LayerNorm-fold vectors: colsum[n] = sum_k Wp[n][k] (of the packed, rounded weights, so that
// r (x.W') - r mu colsum == r ((x - mu).W') exactly w.r.t. the weights the GEMM uses) and
// cvec[n] = sum_k beta[k] W[k][n] + bias[n]. One wave per output column n.
template <typename T>
__global__ void fold_kernel(const T* __restrict__ Wp, int Kpad, const float* __restrict__ W,
                            const float* __restrict__ beta, const float* __restrict__ bias, int K,
                            int N, float* __restrict__ colsum, float* __restrict__ cvec, int Npad) {
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (n >= Npad) return;
  float s = 0.f, c = 0.f;
  if (n < N) {
    for (int k = lane; k < K; k += 64) {
      s += to_f32(Wp[(int64_t)n * Kpad + k]);
      c += beta[k] * W[(int64_t)k * N + n];
    }
  }
  s = wave_sum(s);
  c = wave_sum(c);
  if (lane == 0) {
    colsum[n] = s;
    cvec[n] = (n < N) ? c + (bias ? bias[n] : 0.f) : 0.f;
  }
}

}  // namespace

int device_cus() { return num_cus(); }
void gemm_set_variant(int v) { g_gemm_variant = v; }
bool gemm_variant_supported(int v) {
  return v == 0 || v == 1 || v == 2 || v == 6 || v == 8 || v == 9 || v == 16 || v == 30 || v == 31 ||
         v == 36 ||
         gemm_lab_pers_variant(v)
#ifdef EVT_GEMM_LAB
         || v == 106 || v == 108
#endif
      ;
}
int gemm_variant() { return g_gemm_variant; }

size_t gemm_sk_bytes() { return 4096 + (size_t)SK_MAX_G * SK_SLOT_FLOATS * sizeof(float); }

void gemm_sk_bind(void* ws, GemmParams& p) {
  p.sk_flags = ws ? (int*)ws : nullptr;
  p.sk_part = ws ? (float*)((char*)ws + 4096) : nullptr;
}

bool gemm_headmajor_ok(int dtype, int flags, const GemmParams& p) {
  constexpr int F = EPI_LNIN | EPI_BIAS | EPI_HM;
  return dtype == DT_BF16 && (flags | EPI_HM) == F && p.K % PAD_K == 0 && p.K > 0 &&
         p.ntiles * GEMM_BN >= p.N && headmajor_fits(p) && use_big(p, F) && use_pers(p, F);
}

hipError_t gemm_launch(int dtype, int flags, const GemmParams& p, hipStream_t s) {
  if (p.M <= 0 || p.N <= 0) return hipSuccess;
  if (p.K % PAD_K != 0 || p.K <= 0) return hipErrorInvalidValue;
  if (p.ntiles * GEMM_BN < p.N) return hipErrorInvalidValue;
  return dtype == DT_BF16 ? dispatch<bf16>(flags, p, s) : dispatch<float>(flags, p, s);
}

hipError_t gemm_splitk_launch(int dtype, int flags, const GemmParams& p, int S, float* part,
                              hipStream_t s) {
  if (p.M <= 0 || p.N <= 0) return hipSuccess;
  if (S < 1 || p.K % (S * PAD_K) || (flags & ~(EPI_BIAS | EPI_GELU | EPI_OUT_F32)) || !part)
    return hipErrorInvalidValue;
  return dtype == DT_BF16 ? splitk_t<bf16>(flags, p, S, part, s) : splitk_t<float>(flags, p, S, part, s);
}

namespace {
__global__ void to_bf16_kernel(const float* __restrict__ x, bf16* __restrict__ y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = (bf16)x[i];
}
}  // namespace

hipError_t to_bf16_launch(const float* x, void* y, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(to_bf16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, (bf16*)y, n);
  return hipGetLastError();
}

hipError_t pack_weight(int dtype, const float* W, const float* row_scale, int K, int N, void* Wp,
                       int Kpad, int Npad, hipStream_t s) {
  dim3 grid((Kpad + 31) / 32, (Npad + 31) / 32);
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(pack_kernel<bf16>, grid, dim3(256), 0, s, W, row_scale, K, N, (bf16*)Wp,
                       Kpad, Npad);
  else
    hipLaunchKernelGGL(pack_kernel<float>, grid, dim3(256), 0, s, W, row_scale, K, N, (float*)Wp,
                       Kpad, Npad);
  return hipGetLastError();
}

hipError_t ln_fold(int dtype, const void* Wp, int Kpad, const float* W, const float* beta,
                   const float* bias, int K, int N, float* colsum, float* cvec, int Npad,
                   hipStream_t s) {
  dim3 grid((Npad + 3) / 4);
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(fold_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)Wp, Kpad, W, beta,
                       bias, K, N, colsum, cvec, Npad);
  else
    hipLaunchKernelGGL(fold_kernel<float>, grid, dim3(256), 0, s, (const float*)Wp, Kpad, W, beta,
                       bias, K, N, colsum, cvec, Npad);
  return hipGetLastError();
}

}  // namespace evt
