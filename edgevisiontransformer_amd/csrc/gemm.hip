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
    if (FL & EPI_GELU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = gelu_tanh(v[j]);
    }
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
    if (FL & EPI_GELU) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[h][j] = gelu_tanh(v[h][j]);
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
      if (full) __builtin_nontemporal_store(__builtin_bit_cast(u32x4, o), (u32x4*)cp);
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

int g_gemm_variant = 0;  // 0 auto, 1 force 128x128, 2 / 6 256x256 VAR 0 / 6

bool use_big(const GemmParams& p, int flags) {
  if ((p.ntiles * GEMM_BN) % BIG_BN) return false;
  if (!(flags & EPI_OUT_F32) && p.vec_ok < 2) return false;  // big epilogue: 16-B bf16 stores only
  if (g_gemm_variant == 1) return false;
  if (g_gemm_variant >= 2) return true;
  // enough 256x256 tiles to fill the chip at least once
  return (int64_t)((p.M + 255) / 256) * (p.ntiles * GEMM_BN / 256) >= 256;
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

template <int FL, int VAR>
__global__ __launch_bounds__(512, 2) void gemm_big_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * BIG_STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably uniform -> SGPR math
  const int wm = wave & 1, wn = wave >> 1;
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

  big_epilogue<FL>(p, smem, acc, wm, wn, m0, n0, tn, wave, lane);
}

template <int FL>
hipError_t launch_big(const GemmParams& p, hipStream_t s) {
  const int mtiles = (p.M + BIG_BM - 1) / BIG_BM;
  GemmParams q = p;
  q.ntiles = (p.ntiles * GEMM_BN) / BIG_BN;
  const dim3 grid(mtiles * q.ntiles);
  if (g_gemm_variant == 2)
    hipLaunchKernelGGL((gemm_big_kernel<FL, 0>), grid, dim3(512), 0, s, q);
  else
    hipLaunchKernelGGL((gemm_big_kernel<FL, 6>), grid, dim3(512), 0, s, q);
  return hipGetLastError();
}

template <typename T, int FL>
hipError_t launch_t(const GemmParams& p, hipStream_t s) {
  if constexpr (std::is_same<T, bf16>::value) {
    if (use_big(p, FL)) return launch_big<FL>(p, s);
  }
  const int mtiles = (p.M + GEMM_BM - 1) / GEMM_BM;
  hipLaunchKernelGGL((gemm_nt_kernel<T, FL>), dim3(mtiles * p.ntiles), dim3(256), 0, s, p);
  return hipGetLastError();
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
#undef EVT_CASE
    default: return hipErrorInvalidValue;
  }
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

void gemm_set_variant(int v) { g_gemm_variant = v; }

hipError_t gemm_launch(int dtype, int flags, const GemmParams& p, hipStream_t s) {
  if (p.M <= 0 || p.N <= 0) return hipSuccess;
  if (p.K % PAD_K != 0 || p.K <= 0) return hipErrorInvalidValue;
  if (p.ntiles * GEMM_BN < p.N) return hipErrorInvalidValue;
  return dtype == DT_BF16 ? dispatch<bf16>(flags, p, s) : dispatch<float>(flags, p, s);
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
