// Swin Transformer kernels for gfx950 (reference `utils.py:14-47` get_swin -> microsoft
// Swin-Transformer `SwinTransformer`, benchmarked as swin_tiny_patch4_window7_224 NCHW by
// `tools.py:272-282`; the algorithm restated in oracle/swin_ref.py).
//
// The token stream stays in raster order [B][R*R][Cst] (Cst = C rounded up to 64, pad columns
// kept at exactly 0) for the whole stage: LayerNorm, QKV, proj and the MLP are per-token, so the
// cyclic shift and the window partition / reverse only change WHICH rows one window's attention
// reads and writes. window_attn_* computes those row indices itself (torch.roll(-s) + 7x7
// partition on the way in, the inverse on the way out) - no roll, partition or reverse pass ever
// touches HBM.
//
//   swin_patch_kernel    Conv2d(k = s = patch) as im2col: NCHW fp32 -> rows (c, kh, kw), zero pad
//   ln_rows_kernel       LayerNorm of act-dtype rows -> act dtype + slot statistics (embed norm)
//   merge_kernel         PatchMerging gather x[0::2,0::2] | x[1::2,0::2] | x[0::2,1::2] |
//                        x[1::2,1::2] -> [B*(R/2)^2][4C] + row statistics (its LayerNorm is folded
//                        into the reduction GEMM)
//   window_attn_bf16     one wave per (window, head): S^T = K Q^T and O^T = V^T P^T on
//                        v_mfma_f32_16x16x32_bf16 (head size 32 = one MFMA k-step), + relative
//                        position bias + SW-MSA mask (one precomputed table per window type),
//                        exact softmax
//   window_attn_f32      the exact fp32 parity path (VALU dot products, K / V in LDS)
//   ln_pool_kernel       final LayerNorm + mean over tokens (AdaptiveAvgPool1d) -> [B][Cst]
#include <algorithm>

#include "common.h"
#include "evt_internal.h"

namespace evt {

namespace {

constexpr float kLog2e = 1.4426950408889634f;

// ---- patch embedding im2col ----------------------------------------------------------------
// One block per (patch row py, image b): the [C][ps][S] fp32 strip of the image is staged in LDS
// with coalesced 16-B loads, then the S/ps output rows (c, kh, kw) leave as 16-B chunks of 8
// (coalesced row-contiguous stores), zero padded to ldo.
template <typename TO>
__global__ __launch_bounds__(256) void swin_patch_kernel(const float* __restrict__ img, int C,
                                                         int S, int ps, TO* __restrict__ out,
                                                         int ldo) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* strip = (float*)smem;
  const int py = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int np = S / ps, per_c = ps * S, pd = C * ps * ps;
  for (int c = 0; c < C; ++c) {
    const float* src = img + (((int64_t)b * C + c) * S + (int64_t)py * ps) * S;
    for (int i = tid * 4; i < per_c; i += 256 * 4) *(f32x4*)(strip + c * per_c + i) = load4(src + i);  // LDS
  }
  __syncthreads();
  TO* orow = out + ((int64_t)b * np + py) * np * ldo;
  const int cpr = ldo / 8;  // 8-element chunks per output row
  for (int e = tid; e < np * cpr; e += 256) {
    const int px = e / cpr, f0 = (e - px * cpr) * 8;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = f0 + j;
      v[j] = 0.f;
      if (f < pd) {
        const int c = f / (ps * ps), r = f - c * ps * ps, kh = r / ps, kw = r - kh * ps;
        v[j] = strip[c * per_c + kh * S + px * ps + kw];
      }
    }
    TO* op = orow + (int64_t)px * ldo + f0;
    store4(op, f32x4{v[0], v[1], v[2], v[3]});
    store4(op + 4, f32x4{v[4], v[5], v[6], v[7]});
  }
}

// ---- LayerNorm rows (act dtype in / out) + statistics of the stored output -----------------
// LPR lanes per row (power of 2 <= 64), each lane NC 16-B chunks (ld <= LPR * NC * V); 64 / LPR
// rows per wave; reductions over the row's lanes with xor shuffles.
template <typename T, int LPR, int NC>
__global__ __launch_bounds__(256) void ln_rows_kernel(const T* __restrict__ x, int64_t ld,
                                                      T* __restrict__ y,
                                                      const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, int rows,
                                                      int D, float eps,
                                                      float* __restrict__ stats, int nslots) {
  constexpr int V = 16 / sizeof(T);
  const int lane = threadIdx.x & 63, sub = lane % LPR;
  const int row = (blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / LPR) + lane / LPR;
  const bool live = row < rows;
  const T* xr = x + (int64_t)min(row, rows - 1) * ld;
  float v[NC][V];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c0 = (i * LPR + sub) * V;
    u32x4 raw = u32x4{0u, 0u, 0u, 0u};
    if (c0 < ld) raw = *(const u32x4*)(xr + c0);
    const T* tv = (const T*)&raw;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      v[i][j] = (c0 + j < D) ? to_f32(tv[j]) : 0.f;
      s += v[i][j];
    }
  }
#pragma unroll
  for (int o = 1; o < LPR; o <<= 1) s += __shfl_xor(s, o, 64);
  const float inv_d = 1.0f / (float)D;
  const float mean = s * inv_d;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i)
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c = (i * LPR + sub) * V + j;
      if (c < D) q += (v[i][j] - mean) * (v[i][j] - mean);
    }
#pragma unroll
  for (int o = 1; o < LPR; o <<= 1) q += __shfl_xor(q, o, 64);
  const float rstd = rsqrtf(q * inv_d + eps);
  T* yr = y + (int64_t)row * ld;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c0 = (i * LPR + sub) * V;
    if (c0 >= ld) continue;
    T o[V];
    float gv[V], bv[V];  // 16-B loads of gamma / beta (D is a multiple of V here)
#pragma unroll
    for (int j = 0; j < V; j += 4) {
      const f32x4 gq = c0 + j < D ? load4(gamma + c0 + j) : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 bq = c0 + j < D ? load4(beta + c0 + j) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        gv[j + u] = gq[u];
        bv[j + u] = bq[u];
      }
    }
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c = c0 + j;
      o[j] = from_f32<T>(c < D ? (v[i][j] - mean) * rstd * gv[j] + bv[j] : 0.f);
      const float f = to_f32(o[j]);
      s1 += f;
      s2 += f * f;
    }
    if (live) store_b128(yr + c0, *(const u32x4*)o);
  }
#pragma unroll
  for (int o = 1; o < LPR; o <<= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  if (live && sub < nslots) {
    float* st = stats + 2 * ((int64_t)nslots * row + sub);
    st[0] = sub == 0 ? s1 : 0.f;
    st[1] = sub == 0 ? s2 : 0.f;
  }
}

// ---- PatchMerging gather: one wave per output row, 16-B chunks (C % 8 == 0) -----------------
template <typename T>
__global__ __launch_bounds__(256) void merge_kernel(const T* __restrict__ x, int64_t ldx, int B,
                                                    int R, int C, T* __restrict__ out,
                                                    float* __restrict__ stats, int nslots) {
  constexpr int V = 16 / sizeof(T);  // elements per 16-B chunk
  const int lane = threadIdx.x & 63;
  const int64_t orow = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int R2 = R / 2;
  if (orow >= (int64_t)B * R2 * R2) return;
  const int b = (int)(orow / (R2 * R2)), t = (int)(orow - (int64_t)b * R2 * R2);
  const int oy = t / R2, ox = t - oy * R2;
  T* op = out + orow * 4 * C;
  const int cq = C / V;  // chunks per quadrant
  float s1 = 0.f, s2 = 0.f;
  // quadrant q: (dy, dx) = (q & 1, q >> 1) (reference order x0, x1, x2, x3)
  for (int e = lane; e < 4 * cq; e += 64) {
    const int q = e / cq, c = (e - q * cq) * V;
    const int y = 2 * oy + (q & 1), xx = 2 * ox + (q >> 1);
    const u32x4 v = *(const u32x4*)(x + ((int64_t)b * R * R + (int64_t)y * R + xx) * ldx + c);
    store_b128(op + q * C + c, v);
    const T* tv = (const T*)&v;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float f = to_f32(tv[j]);
      s1 += f;
      s2 += f * f;
    }
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (lane < nslots) {
    float* st = stats + 2 * ((int64_t)nslots * orow + lane);
    st[0] = lane == 0 ? s1 : 0.f;
    st[1] = lane == 0 ? s2 : 0.f;
  }
}

// ---- statistics of the gathered PatchMerging rows (for the EPI_GATHER reduction GEMM) ----------
// Row (b, y, x) of the R/2 grid is the concatenation of 4 source tokens, so its (sum, sumsq) is the
// sum of their slot statistics (written by the previous stage's last sublayer): slot 0, the other
// slots zero.
__global__ __launch_bounds__(256) void merge_stats_kernel(const float* __restrict__ src, int ns,
                                                          int B, int R, float* __restrict__ dst,
                                                          int nd) {
  const int R2 = R / 2;
  const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (m >= (int64_t)B * R2 * R2) return;
  const int b = (int)(m / (R2 * R2)), r = (int)(m - (int64_t)b * R2 * R2), y = r / R2, x = r - y * R2;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t row = ((int64_t)b * R + 2 * y + (q & 1)) * R + 2 * x + (q >> 1);
    for (int j = 0; j < ns; ++j) {
      const f32x2 v = *(const f32x2*)(src + (row * ns + j) * 2);
      s1 += v[0];
      s2 += v[1];
    }
  }
  float* d = dst + m * nd * 2;
  *(f32x2*)d = f32x2{s1, s2};
  for (int j = 1; j < nd; ++j) *(f32x2*)(d + 2 * j) = f32x2{0.f, 0.f};
}

// ---- relative position bias + shift mask, expanded once per block at model creation ----------
// dense[type][h][q][k] = table[(qy-ky+w-1)*(2w-1) + (qx-kx+w-1)][h] * log2(e), -100 * log2(e) more
// where q and k lie in different SW-MSA regions, -inf for k >= w*w. With a shift the windows of
// the last window row / column see the 3x3 region split (region of a window-local row i: 1 if
// i < w - shift else 2; 0 elsewhere): type = 2 * (last window row) + (last window column).
// Without a shift there is one type (no mask).
__global__ void rpb_dense_kernel(const float* __restrict__ table, int H, int w, int shift,
                                 float* __restrict__ dense) {
  const int n = w * w;
  const int ntypes = shift ? 4 : 1;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= ntypes * H * n * 64) return;
  const int type = e / (H * n * 64), r0 = e - type * H * n * 64;
  const int h = r0 / (n * 64), r = r0 - h * n * 64, q = r / 64, k = r - q * 64;
  float v = -INFINITY;
  if (k < n) {
    const int qy = q / w, qx = q - qy * w, ky = k / w, kx = k - ky * w;
    v = table[((qy - ky + w - 1) * (2 * w - 1) + (qx - kx + w - 1)) * H + h] * kLog2e;
    const bool lr = type & 2, lc = type & 1;  // last window row / column
    const int rq = (lr ? (qy < w - shift ? 1 : 2) : 0) * 3 + (lc ? (qx < w - shift ? 1 : 2) : 0);
    const int rk = (lr ? (ky < w - shift ? 1 : 2) : 0) * 3 + (lc ? (kx < w - shift ? 1 : 2) : 0);
    if (rq != rk) v += -100.0f * kLog2e;
  }
  dense[e] = v;
}

// Compact relative-position table per head (the bf16 window kernel's bias source): RPB_CROW
// floats per head, entries 0 .. 168 = table[r][h] * log2(e), stored after the dense tables.
constexpr int RPB_CROW = 192;
__host__ __device__ __forceinline__ const float* rpb_compact(const float* dense, int H, int shift) {
  return dense + (size_t)(shift ? 4 : 1) * H * 49 * 64;
}
__global__ void rpb_compact_kernel(const float* __restrict__ table, int H, float* __restrict__ out) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= H * RPB_CROW) return;
  const int h = e / RPB_CROW, r = e - h * RPB_CROW;
  out[e] = r < 169 ? table[r * H + h] * kLog2e : 0.f;
}

// Row of window-local token t (t < 49) of window `win` of image b, with the cyclic shift; and
// the bias / mask table type of the window.
struct WinGeom {
  int R, s;
  int y0, x0;       // shifted-frame origin of the window (wy * 7 + s, wx * 7 + s)
  int64_t base;     // first token row of the image
  int wtype;        // bias / mask table type (rpb_dense_kernel): last window row / column
  __device__ __forceinline__ WinGeom(int R_, int nwx, int s_, int b, int win) : R(R_), s(s_) {
    const int wy = win / nwx, wx = win - wy * nwx;
    y0 = wy * 7 + s;
    x0 = wx * 7 + s;
    base = (int64_t)b * R * R;
    wtype = s ? (wy == nwx - 1 ? 2 : 0) + (wx == nwx - 1 ? 1 : 0) : 0;
  }
  __device__ __forceinline__ int64_t row(int t) const {
    const int i = t / 7, j = t - i * 7;
    int y = y0 + i, x = x0 + j;
    if (y >= R) y -= R;
    if (x >= R) x -= R;
    return base + (y * R + x);
  }
  __device__ __forceinline__ int type() const { return wtype; }
};

// Butterfly max / sum over lanes l ^ 16 and l ^ 32 on the VALU: v_permlane16_swap / 32_swap of a
// value with itself leave the two halves of each row pair (of the wave) in the two results, so one
// max / add gives every lane the reduction (no LDS round trip as with ds_bpermute).
__device__ __forceinline__ float bfly_max_16_32(float x) {
  unsigned u = __builtin_bit_cast(unsigned, x);
  const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  x = fmaxf(__builtin_bit_cast(float, (unsigned)a[0]), __builtin_bit_cast(float, (unsigned)a[1]));
  u = __builtin_bit_cast(unsigned, x);
  const auto c = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)c[0]), __builtin_bit_cast(float, (unsigned)c[1]));
}
__device__ __forceinline__ float bfly_sum_16_32(float x) {
  unsigned u = __builtin_bit_cast(unsigned, x);
  const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  x = __builtin_bit_cast(float, (unsigned)a[0]) + __builtin_bit_cast(float, (unsigned)a[1]);
  u = __builtin_bit_cast(unsigned, x);
  const auto c = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __builtin_bit_cast(float, (unsigned)c[0]) + __builtin_bit_cast(float, (unsigned)c[1]);
}

// bf16 window attention. 4 waves per block, wave = one (image, window, head); head size 32,
// window 7x7 = 49 tokens padded to 64 (4 tiles of 16). Q / K fragments are 16-B loads straight
// from the QKV rows; V goes to the wave's 4 KiB of LDS (LDS-DMA, chunk swizzle (row >> 2) & 3) for
// the transposed ds_read_b64_tr_b16 reads of the V^T operand. Every global access goes through a
// buffer descriptor of the image (SGPR base) with a 32-bit row offset per lane and the q / k / v
// column block in soffset.
// The relative position bias comes from the head's compact table (169 entries x log2 e, 768 B,
// LDS-DMA'd per wave): bias(q, k) = T[(qi - ki + 6) 13 + (qj - kj + 6)] = T[a(q) - b(k)] with
// a(q) = 6 qi + q + 84, b(k) = 6 ki + k, one ds_read_b32 per score; the SW-MSA region mask (and the
// keys past 49) set the score to -inf (the reference's -100 leaves e^-100 relative weights, below
// fp32 resolution against the row maximum's 1). Round-4 counters (profiles/r04_pmc_swin_*): the
// texture-address unit was busy 75 % of the kernel, half of that stalled on the L1, and the
// kernel without its dense-table bias reads (16 x 16 B per lane per wave, L2 hits) ran 25 %
// faster: those reads are gone; the VALU butterflies and v_rcp_f32 cut its VALU count by 29 %.
__global__ __launch_bounds__(256) void window_attn_bf16_kernel(SwinAttnParams p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * 64 * 64 + 4 * 768];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: scalar index math
  const int pair = blockIdx.x * 4 + wave;  // (B * windows * H < 2^31: checked at launch)
  const int nw = p.nwx * p.nwx;
  if (pair >= p.B * nw * p.H) return;
  const int h = pair % p.H;
  const int bw = pair / p.H;
  const int win = bw % nw, b = bw / nw;
  const int R = p.R, s0 = p.shift;
  const int wy = win / p.nwx, wx = win - wy * p.nwx;
  const int y0 = wy * 7 + s0, x0 = wx * 7 + s0;
  const int wtype = s0 ? (wy == p.nwx - 1 ? 2 : 0) + (wx == p.nwx - 1 ? 1 : 0) : 0;
  // image-local raster row of window token t (with the cyclic shift)
  auto lrow = [&](int t) {
    const int i = (t * 37) >> 8, j = t - 7 * i;  // t / 7 for t < 64
    int y = y0 + i, x = x0 + j;
    if (y >= R) y -= R;
    if (x >= R) x -= R;
    return y * R + x;
  };
  const int ldq2 = (int)p.ldq * 2, ldo2 = (int)p.ldo * 2;
  const int64_t img0 = (int64_t)b * R * R;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (char*)const_cast<void*>(p.qkv) + img0 * ldq2, 0, R * R * ldq2, 0x00020000);
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
      (char*)p.out + img0 * ldo2, 0, R * R * ldo2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(rpb_compact(p.bias, p.H, s0)) + h * RPB_CROW, 0, RPB_CROW * 4, 0x00020000);
  const int g = lane >> 4, c16 = lane & 15;
  EVT_LDS char* Vs = (EVT_LDS char*)smem + wave * 4096;
  EVT_LDS char* Ts = (EVT_LDS char*)smem + 4 * 4096 + wave * 768;
  const int C2 = p.C * 2;

  // the head's compact bias table -> LDS (3 x 64 lanes x 4 B)
#pragma unroll
  for (int i = 0; i < 3; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rt, Ts + i * 256, 4, lane * 4, i * 256, 0, 0);
  // V rows (keys) -> LDS: instruction i covers rows 16 i + (lane >> 2), 16-B chunk lane & 3
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 16 * i + (lane >> 2), ch = (lane & 3) ^ ((r >> 2) & 3);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, Vs + i * 1024, 16,
                                             lrow(min(r, 48)) * ldq2 + (h * 32 + ch * 8) * 2,
                                             2 * C2, 0, 0);
  }
  // Q and K fragments: tile i, lane (token 16 i + c16, d 8 g .. 8 g + 7)
  u32x4 qf[4], kf[4];
  int qoff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = min(16 * i + c16, 48);
    const int lr = lrow(t);
    qoff[i] = lr * ldo2 + (h * 32 + 4 * g) * 2;  // query token t's output row, this lane's columns
    const int vo = lr * ldq2 + (h * 32 + 8 * g) * 2;
    qf[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 0, 0));
    kf[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, C2, 0));
  }
  // per-lane table offsets b(k) of its 16 keys k = 16 kt + 4 g + j (keys past 48 read key 48's:
  // masked below) and, for SW-MSA windows, their region codes (bit 0: lower part of the last
  // window row, bit 1: right part of the last window column), one byte per j
  int kofs[4][4];
  unsigned kc[4] = {0u, 0u, 0u, 0u};
  const int cut = 7 - s0;
  const bool lr_ = wtype & 2, lc_ = wtype & 1;
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = min(16 * kt + 4 * g + j, 48), ki = (k * 37) >> 8, kj = k - 7 * ki;
      kofs[kt][j] = (6 * ki + k) * 4;
      kc[kt] |= (unsigned)((lr_ && ki >= cut ? 1 : 0) | (lc_ && kj >= cut ? 2 : 0)) << (8 * j);
    }
  wait_vmcnt0();

  const int tq = (lane >> 2) & 3, tp = lane & 3;
  const float NEG = -INFINITY;
#pragma unroll
  for (int qt = 0; qt < 4; ++qt) {
    const int q = 16 * qt + c16;
    const int qq = min(q, 48), qi = (qq * 37) >> 8, qj = qq - 7 * qi;
    const EVT_LDS char* Tq = Ts + (6 * qi + qq + 84) * 4;
    const unsigned cq = ((lr_ && qi >= cut ? 1u : 0u) | (lc_ && qj >= cut ? 2u : 0u)) * 0x01010101u;
    f32x4 s[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kf[kt]),
                                                      __builtin_bit_cast(bf16x8, qf[qt]), acc, 0,
                                                      0, 0);
    }
    // s[kt][j] = S^T[key 16 kt + 4 g + j][query q]: scores in the log2 domain + bias on packed
    // pairs, then the masks
    const f32x2 sc2 = {p.scale_log2, p.scale_log2};
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      f32x4 bv;
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = *(const EVT_LDS float*)(Tq - kofs[kt][j]);
      const f32x2 lo = f32x2{s[kt][0], s[kt][1]} * sc2 + f32x2{bv[0], bv[1]};
      const f32x2 hi = f32x2{s[kt][2], s[kt][3]} * sc2 + f32x2{bv[2], bv[3]};
      s[kt] = f32x4{lo[0], lo[1], hi[0], hi[1]};
      if (wtype) {  // SW-MSA window on the last row / column: keys of another region
        const unsigned x = kc[kt] ^ cq;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if ((x >> (8 * j)) & 3u) s[kt][j] = NEG;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)  // keys 49 .. 63 (the padding of tile 3: all but key 48)
      if (4 * g + j > 0) s[3][j] = NEG;
    float m4[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) m4[kt] = fmaxf(fmaxf(s[kt][0], s[kt][1]), fmaxf(s[kt][2], s[kt][3]));
    const float mx = bfly_max_16_32(fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3])));
    float p4[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int j = 0; j < 4; ++j) s[kt][j] = __builtin_amdgcn_exp2f(s[kt][j] - mx);
      p4[kt] = (s[kt][0] + s[kt][1]) + (s[kt][2] + s[kt][3]);
    }
    const float sum = bfly_sum_16_32((p4[0] + p4[1]) + (p4[2] + p4[3]));

    f32x4 o[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 pf;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pf[j] = (bf16)s[2 * ks][j];
        pf[4 + j] = (bf16)s[2 * ks + 1][j];
      }
      const int key0 = ks * 32 + 4 * g + tq;  // and key0 + 16: same (row >> 2) & 3 swizzle
      const int sw = (key0 >> 2) & 3;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int chunk = 2 * dt + (tp >> 1);
        const int off = ((chunk ^ sw) * 16) + (tp & 1) * 8;
        const i16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((EVT_LDS i16x4*)(Vs + key0 * 64 + off));
        const i16x4 v1 =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((EVT_LDS i16x4*)(Vs + (key0 + 16) * 64 + off));
        const i16x8 vv = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vv), pf, o[dt],
                                                        0, 0, 0);
      }
    }
    // o[dt][j] = O^T[d = 16 dt + 4 g + j][query q]
    if (q < 49) {
      const float inv = __builtin_amdgcn_rcpf(sum);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const f32x4 v = o[dt] * inv;
        const bf16x4 ob = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
        buffer_store_b64<0>(__builtin_bit_cast(u32x2, ob), ro, qoff[qt], 32 * dt);
      }
      if (h == 0)  // pad columns [C, ldo) of the attention output (the proj GEMM's K padding)
        for (int c = p.C + 4 * g; c < p.ldo; c += 16)
          buffer_store_b64<0>(u32x2{0u, 0u}, ro, qoff[qt] + (c - 4 * g) * 2, 0);
    }
  }
}

// fp32 window attention (parity path): wave = (image, window, head), lane = query (49 of 64).
__global__ __launch_bounds__(256) void window_attn_f32_kernel(SwinAttnParams p) {
  __shared__ float smem[4][2][49][33];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t pair = (int64_t)blockIdx.x * 4 + wave;
  const int nw = p.nwx * p.nwx;
  if (pair >= (int64_t)p.B * nw * p.H) return;
  const int h = (int)(pair % p.H);
  const int64_t bw = pair / p.H;
  const int win = (int)(bw % nw), b = (int)(bw / nw);
  const WinGeom G(p.R, p.nwx, p.shift, b, win);
  const float* qkv = (const float*)p.qkv;
  float(*Ks)[33] = smem[wave][0];
  float(*Vs)[33] = smem[wave][1];
  for (int e = lane; e < 49 * 32; e += 64) {
    const int t = e >> 5, d = e & 31;
    const float* rp = qkv + G.row(t) * p.ldq + h * 32 + d;
    Ks[t][d] = rp[p.C];
    Vs[t][d] = rp[2 * p.C];
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // wave-private LDS: no barrier
  __builtin_amdgcn_wave_barrier();
  const int t = min(lane, 48);
  const int64_t qrow = G.row(t);
  float q[32];
#pragma unroll
  for (int d = 0; d < 32; ++d) q[d] = qkv[qrow * p.ldq + h * 32 + d];
  const float* br = p.bias + (((int64_t)G.type() * p.H + h) * 49 + t) * 64;
  float sc[49];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < 49; ++k) {
    float a = 0.f;
#pragma unroll
    for (int d = 0; d < 32; ++d) a += q[d] * Ks[k][d];
    const float v = a * p.scale_log2 + br[k];
    sc[k] = v;
    mx = fmaxf(mx, v);
  }
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < 49; ++k) {
    sc[k] = exp2f(sc[k] - mx);
    sum += sc[k];
  }
  float o[32];
#pragma unroll
  for (int d = 0; d < 32; ++d) o[d] = 0.f;
#pragma unroll
  for (int k = 0; k < 49; ++k)
#pragma unroll
    for (int d = 0; d < 32; ++d) o[d] += sc[k] * Vs[k][d];
  if (lane < 49) {
    float* op = (float*)p.out + qrow * p.ldo;
    const float inv = 1.0f / sum;
#pragma unroll
    for (int d = 0; d < 32; ++d) op[h * 32 + d] = o[d] * inv;
    if (h == 0)
      for (int c = p.C; c < p.ldo; ++c) op[c] = 0.f;
  }
}

// ---- final LayerNorm + token mean: one block per image -------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void ln_pool_kernel(const T* __restrict__ x, int64_t ldx, int T_,
                                                      int D, const float* __restrict__ stats,
                                                      int nslots, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, float eps,
                                                      T* __restrict__ out, int64_t ldo) {
  __shared__ float coef[256][2];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float inv_d = 1.0f / (float)D;
  for (int t = tid; t < T_; t += 256) {
    const float* st = stats + 2 * (int64_t)nslots * ((int64_t)b * T_ + t);
    float s1 = 0.f, s2 = 0.f;
    for (int j = 0; j < nslots; ++j) {
      s1 += st[2 * j];
      s2 += st[2 * j + 1];
    }
    const float mu = s1 * inv_d;
    coef[t][0] = mu;
    coef[t][1] = rsqrtf(fmaxf(s2 * inv_d - mu * mu, 0.f) + eps);
  }
  __syncthreads();
  const T* xb = x + (int64_t)b * T_ * ldx;
  for (int c = tid; c < ldo; c += 256) {
    float acc = 0.f;
    if (c < D)
      for (int t = 0; t < T_; ++t) acc += (to_f32(xb[(int64_t)t * ldx + c]) - coef[t][0]) * coef[t][1];
    out[(int64_t)b * ldo + c] = from_f32<T>(c < D ? acc / (float)T_ * gamma[c] + beta[c] : 0.f);
  }
}

// ---- fused MLP of the C = 96 stage (Swin-T / Swin-S stage 1) -------------------------------
// x = xm + fc2(GELU(LN2(xm) W1 + b1)) + b2 (+ row statistics of x) in one pass: the 384-wide
// hidden never leaves the CU. The separate GEMMs move 1.7 GB per stage-1 block (FC1 writes the
// 617 MB hidden, FC2 reads it back) and serialise the erf-GELU VALU work behind the tiles' MFMA;
// here it is xm in + x out (0.3 GB) and each SIMD runs two waves whose MFMA and VALU phases
// interleave.
//   LDS (whole block, loaded once): W1 = the LN2-folded FC1 weights, 384 hidden rows x 96 k
//   (224-B rows), and W2 = FC2, 96 output
//   rows x 384 hidden (800-B rows) with the hidden axis permuted per 32-chunk so that the FC1
//   accumulators ARE the FC2 B operand: chunk position 8g + s holds hidden 4g + s (s < 4) or
//   16 + 4g + (s - 4) - the two 16-row FC1 tiles of the chunk, as lane group g holds them.
//   Wave = 32 tokens (2 tiles of 16), their rows normalised once in registers ((x - mu) r; gamma
//   folded into W1). Per 32-hidden chunk: H^T = W1 . LN(xm)^T seeded with beta.W1 + b1 (12 MFMAs),
//   GELU on the 16 accumulators per lane, bf16 pack, Out^T += W2 . H^T (12 MFMAs, seeded with b2).
//   Products are transposed (C^T = A . B) so one token is one lane column throughout. The
//   per-lane VALU work (GELU) is the bound: erf GELU in its fast bf16-path form.
constexpr int MLP96_C = 96, MLP96_F = 384;
// row pitches from scripts/probe/lds_conflicts.py's lane-group model: 208 / 784 put two 16-B
// reads on one bank group in half of the W1 and W2 fragment reads (measured round 4: 48 % of the
// LDS-active cycles were bank conflicts); 224 / 800 have none (162816 B of the 163840)
constexpr int MLP96_W1_ROW = 224, MLP96_W2_ROW = 800;
constexpr int MLP96_LDS = MLP96_F * MLP96_W1_ROW + MLP96_C * MLP96_W2_ROW;  // 162816 B
// 12 waves (3 per SIMD, <= 168 VGPRs): the MFMA -> GELU -> MFMA chain of one wave leaves the
// SIMD idle on latencies that a third wave fills
constexpr int MLP96_WAVES = 12;

__global__ __launch_bounds__(64 * MLP96_WAVES, 1) void swin_mlp96_kernel(SwinMlpParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  EVT_LDS char* W1s = (EVT_LDS char*)smem;
  EVT_LDS char* W2s = W1s + MLP96_F * MLP96_W1_ROW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const bf16* w1 = (const bf16*)p.w1;
  const bf16* w2 = (const bf16*)p.w2;
  // ---- stage the weights (once per block) ----
  for (int e = tid; e < MLP96_F * 12; e += 64 * MLP96_WAVES) {  // W1: row n, 16-B chunk j of 12
    const int n = e / 12, j = e - n * 12;
    *(EVT_LDS u32x4*)(W1s + n * MLP96_W1_ROW + j * 16) = *(const u32x4*)(w1 + (int64_t)n * p.ldw1 + j * 8);
  }
  for (int e = tid; e < MLP96_C * 48; e += 64 * MLP96_WAVES) {  // W2: row c, chunk (hc, gg) of 12 x 4
    const int c = e / 48, r = e - c * 48, hc = r >> 2, gg = r & 3;
    const bf16* src = w2 + (int64_t)c * p.ldw2 + hc * 32 + 4 * gg;
    const uint2 lo = *(const uint2*)src;         // hidden 32 hc + 4 gg .. + 3
    const uint2 hi = *(const uint2*)(src + 16);  // hidden 32 hc + 16 + 4 gg .. + 3
    *(EVT_LDS u32x4*)(W2s + c * MLP96_W2_ROW + hc * 64 + gg * 16) = u32x4{lo.x, lo.y, hi.x, hi.y};
  }
  __syncthreads();
  const float inv_d = 1.0f / (float)MLP96_C;
  const int ntiles = (p.M + 31) / 32;
  // tile t of round k goes to wave (t mod W) / G of block t mod G (W = G waves x 12): the last,
  // partial round spreads over every block (Swin-T bs256: 512 tiles past 8 full rounds = waves 0-1
  // of all 256 blocks) instead of filling 43 blocks while the others idle
  for (int t = wave * gridDim.x + blockIdx.x; t < ntiles; t += gridDim.x * MLP96_WAVES) {
    const int tok0 = t * 32;
    // B operand of FC1: LN2(xm) of token (16 tt + c16), k 32 ks + 8 g .. + 7, normalised in
    // registers ((x - mu) r; gamma is folded into W1, beta.W1 + b1 = cvec seeds the accumulator)
    u32x4 a[2][3];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int m = min(tok0 + 16 * tt + c16, p.M - 1);
      const bf16* ar = (const bf16*)p.xm + (int64_t)m * MLP96_C;
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) a[tt][ks] = *(const u32x4*)(ar + 32 * ks + 8 * g);
      const float* st = p.stats_in + (int64_t)m * 2 * p.nslots;
      float s1 = 0.f, s2 = 0.f;
      for (int j = 0; j < p.nslots; ++j) {
        s1 += st[2 * j];
        s2 += st[2 * j + 1];
      }
      const float mu = s1 * inv_d;
      const float rs = rsqrtf(fmaxf(s2 * inv_d - mu * mu, 0.f) + p.eps);
      const f32x2 r2 = {rs, rs}, o2 = {-mu * rs, -mu * rs};
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const bf16x8 xv = __builtin_bit_cast(bf16x8, a[tt][ks]);
        u32x4 nv;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x2 f = f32x2{(float)xv[2 * q], (float)xv[2 * q + 1]} * r2 + o2;
          nv[q] = __builtin_bit_cast(unsigned, __builtin_convertvector(f, bf16x2));
        }
        a[tt][ks] = nv;
      }
    }
    f32x4 out[6][2];
#pragma unroll
    for (int ct = 0; ct < 6; ++ct) out[ct][0] = out[ct][1] = load4(p.b2 + ct * 16 + 4 * g);
#pragma unroll 2
    for (int hc = 0; hc < 12; ++hc) {
      f32x4 h[2][2];
#pragma unroll
      for (int ht = 0; ht < 2; ++ht) {
        const EVT_LDS char* wr = W1s + (hc * 32 + ht * 16 + c16) * MLP96_W1_ROW + 16 * g;
        h[ht][0] = h[ht][1] = load4(p.cvec + hc * 32 + ht * 16 + 4 * g);
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
          const u32x4 wv = *(const EVT_LDS u32x4*)(wr + 64 * ks);
#pragma unroll
          for (int tt = 0; tt < 2; ++tt)
            h[ht][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, wv), __builtin_bit_cast(bf16x8, a[tt][ks]), h[ht][tt], 0, 0, 0);
        }
      }
      // h[ht][tt][jj]: hidden 32 hc + 16 ht + 4 g + jj, token 16 tt + c16 (bias included) -> GELU,
      // packed straight into the FC2 B operand (k slots 8 g .. 8 g + 7 = [ht 0 jj 0..3 | ht 1])
      u32x4 pf[2];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int ht = 0; ht < 2; ++ht) {
          const f32x2 lo = gelu_erf_fast2(f32x2{h[ht][tt][0], h[ht][tt][1]});
          const f32x2 hi = gelu_erf_fast2(f32x2{h[ht][tt][2], h[ht][tt][3]});
          pf[tt][2 * ht] = __builtin_bit_cast(unsigned, __builtin_convertvector(lo, bf16x2));
          pf[tt][2 * ht + 1] = __builtin_bit_cast(unsigned, __builtin_convertvector(hi, bf16x2));
        }
#pragma unroll
      for (int ct = 0; ct < 6; ++ct) {
        const u32x4 wv = *(const EVT_LDS u32x4*)(W2s + (ct * 16 + c16) * MLP96_W2_ROW + hc * 64 + 16 * g);
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
          out[ct][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, wv), __builtin_bit_cast(bf16x8, pf[tt]), out[ct][tt], 0, 0, 0);
      }
    }
    // out[ct][tt][jj]: feature 16 ct + 4 g + jj, token 16 tt + c16: + b2 + xm, store x, stats
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int m = tok0 + 16 * tt + c16;
      const bool ok = m < p.M;
      const int mc = min(m, p.M - 1);
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int ct = 0; ct < 6; ++ct) {
        const int c = ct * 16 + 4 * g;
        const f32x4 r = load4((const bf16*)p.xm + (int64_t)mc * MLP96_C + c);
        const f32x4 v = out[ct][tt] + r;  // (b2 seeded the accumulator)
        const bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
        if (ok) *(bf16x4*)((bf16*)p.x + (int64_t)m * MLP96_C + c) = o;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float f = (float)o[jj];
          s1 += f;
          s2 += f * f;
        }
      }
      s1 += __shfl_xor(s1, 16, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (ok && g < p.nslots) {
        float* so = p.stats_out + (int64_t)m * 2 * p.nslots + 2 * g;
        so[0] = g == 0 ? s1 : 0.f;
        so[1] = g == 0 ? s2 : 0.f;
      }
    }
  }
}


// ---- fused attention sublayer of the C = 96 stage (Swin-T / Swin-S stage 1) --------------------
// xm = x + proj(WMSA(LN1(x))) for one 7x7 window per block iteration, everything between the x
// read and the xm write on chip: the separate QKV GEMM, window attention and proj move 1.7 GB per
// stage-1 block (qkv 462 MB written + read, o 154 MB written + read, x / xm); here 0.3 GB.
// The per-window work is small and latency-bound (three short phases separated by barriers), so
// the kernel is sized for TWO blocks per CU, whose phases interleave: 4 waves and 71 KiB of LDS
// per block. The QKV weights (288 x 96, LN1 gamma folded) live in registers, split by feature
// tile over the waves (5 / 5 / 4 / 4 of 18 tiles: 60 VGPRs); LDS holds the proj weights (96 x 96),
// the window's qkv [64][288] and one [64][96] buffer that is Xn = LN1(x) of the 49 (64) window
// tokens (gathered with the cyclic shift) in P1, the attention output O in P2 / P3 and the xm
// staging rows at the end.
//   P0  Xn ((x - mu) r, rows past 49 zero) from the x chunks prefetched during the previous
//       window's attention                                                       -> barrier
//   P1  QKV^T = Wq . Xn^T (+ beta.W + b seeds), wave = its feature tiles x all 4 token tiles
//                                                                                -> barrier
//   P2  attention units (head h, query tile `wave`) for h = 0..2, exactly as window_attn_bf16 with
//       Q / K / V from LDS; O rows 16 wave .. 16 wave + 15 are written by this wave only, so
//   P3  (no barrier) proj = Wp . O^T + b + x (rows re-read from L2) -> bf16 xm, full-row
//       statistics in the wave (lane groups hold the 4 column quarters), xm staged through the
//       wave's own O rows and stored as whole 192-B rows (16-B pieces).
constexpr int AT96_ROW = 208;                       // 96-element rows (+ 8 pad)
constexpr int AT96_QROW = 592;                      // 288-element qkv rows (+ 8 pad)
constexpr int AT96_WP = 0;                          // proj weights [96][AT96_ROW]
constexpr int AT96_QKV = AT96_WP + 96 * AT96_ROW;   // 19968: window qkv [64][AT96_QROW]
constexpr int AT96_XO = AT96_QKV + 64 * AT96_QROW;  // 57856: Xn / O / xm staging [64][AT96_ROW]
constexpr int AT96_CV = AT96_XO + 64 * AT96_ROW;    // 71168: cqkv [288], bproj [96] (f32)
constexpr int AT96_TB = AT96_CV + 384 * 4;          // 72704: compact bias tables [3][RPB_CROW]
constexpr int AT96_LDS = AT96_TB + 3 * RPB_CROW * 4;  // 75008: two blocks per CU

__global__ __launch_bounds__(256, 2) void swin_attn96_kernel(SwinAttnBlockParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  EVT_LDS char* L = (EVT_LDS char*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  const bf16* x = (const bf16*)p.x;
  // ---- once per block: Wp / cqkv / bproj -> LDS, this wave's Wq fragments -> registers ----
  for (int e = tid; e < 96 * 12; e += 256) {
    const int n = e / 12, j = e - n * 12;
    *(EVT_LDS u32x4*)(L + AT96_WP + n * AT96_ROW + j * 16) =
        *(const u32x4*)((const bf16*)p.wproj + (int64_t)n * p.ldp + j * 8);
  }
  for (int e = tid; e < 384; e += 256)
    ((EVT_LDS float*)(L + AT96_CV))[e] = e < 288 ? p.cqkv[e] : p.bproj[e - 288];
  {  // the three heads' compact relative-position tables (window_attn_bf16_kernel)
    const float* cb = rpb_compact(p.bias, 3, p.shift);
    for (int e = tid; e < 3 * RPB_CROW; e += 256) ((EVT_LDS float*)(L + AT96_TB))[e] = cb[e];
  }
  // per-lane table offsets b(k) of the 16 keys k = 16 kt + 4 g + j (past 48: key 48's, masked)
  int kofs[4][4], kij[4][4];
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = min(16 * kt + 4 * g + j, 48), ki = (k * 37) >> 8;
      kofs[kt][j] = (6 * ki + k) * 4;
      kij[kt][j] = ki * 8 + (k - 7 * ki);  // row, column in the window
    }
  const int cut = 7 - p.shift;
  const int ft0 = wave * 5 - (wave > 2 ? 1 : 0), nft = wave < 2 ? 5 : 4;  // 0 / 5 / 10 / 14
  u32x4 wq[5][3];
#pragma unroll
  for (int f = 0; f < 5; ++f)
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      const int ft = min(ft0 + f, 17);
      wq[f][ks] = *(const u32x4*)((const bf16*)p.wqkv + (int64_t)(16 * ft + c16) * p.ldq + 32 * ks + 8 * g);
    }
  const int nwx = p.R / 7, nw = nwx * nwx, nwin = p.B * nw;
  const float inv_d = 1.0f / 96.0f;
  const float scale_log2 = 0.17677669529663687f * kLog2e;
  // x chunks (token e / 12, 16-B chunk e % 12; e = tid + 256 k) and their row statistics of the
  // NEXT window, loaded during the current window's attention phase
  u32x4 xc[3];
  f32x4 sc[3];
  auto prefetch = [&](int wgn) {
    const int bn = wgn / nw, wn = wgn - bn * nw;
    const WinGeom Gn(p.R, nwx, p.shift, bn, wn);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int e = tid + 256 * k, t = e / 12, j = e - t * 12;
      xc[k] = u32x4{0u, 0u, 0u, 0u};
      sc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (t < 49) {
        const int64_t row = Gn.row(t);
        xc[k] = *(const u32x4*)(x + row * 96 + j * 8);
        const float* st = p.stats_in + row * 2 * p.nslots;
        sc[k] = f32x4{st[0], st[1], p.nslots > 1 ? st[2] : 0.f, p.nslots > 1 ? st[3] : 0.f};
      }
    }
  };
  if (blockIdx.x < nwin) prefetch(blockIdx.x);
  const int tq = (lane >> 2) & 3, tp = lane & 3;
  for (int wg = blockIdx.x; wg < nwin; wg += gridDim.x) {
    const int b = wg / nw, win = wg - b * nw;
    const WinGeom G(p.R, nwx, p.shift, b, win);
    __syncthreads();  // the previous window's qkv / XO readers are done
    // ---- P0: Xn = LN1(x) of the window tokens ((x - mu) r; gamma is in Wq, beta in cqkv) ----
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int e = tid + 256 * k, t = e / 12, j = e - t * 12;
      u32x4 nv = u32x4{0u, 0u, 0u, 0u};
      if (t < 49) {  // (nslots <= 2 here: C = 96)
        const float s1 = sc[k][0] + sc[k][2], s2 = sc[k][1] + sc[k][3];
        const float mu = s1 * inv_d;
        const float r = rsqrtf(fmaxf(s2 * inv_d - mu * mu, 0.f) + p.eps);
        const bf16x8 xv = __builtin_bit_cast(bf16x8, xc[k]);
        const f32x2 r2 = {r, r}, o2 = {-mu * r, -mu * r};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x2 f = f32x2{(float)xv[2 * q], (float)xv[2 * q + 1]} * r2 + o2;
          nv[q] = __builtin_bit_cast(unsigned, __builtin_convertvector(f, bf16x2));
        }
      }
      *(EVT_LDS u32x4*)(L + AT96_XO + t * AT96_ROW + j * 16) = nv;
    }
    __syncthreads();
    // ---- P1: QKV^T = Wq . Xn^T + cqkv: this wave's feature tiles x the 4 token tiles ----
    {
      u32x4 bx[4][3];
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int ks = 0; ks < 3; ++ks)
          bx[tt][ks] = *(const EVT_LDS u32x4*)(L + AT96_XO + (16 * tt + c16) * AT96_ROW + 64 * ks + 16 * g);
#pragma unroll
      for (int f = 0; f < 5; ++f) {
        if (f >= nft) break;
        const int ft = ft0 + f;
        const f32x4 cq = *(const EVT_LDS f32x4*)(L + AT96_CV + (16 * ft + 4 * g) * 4);
        f32x4 acc[4] = {cq, cq, cq, cq};
#pragma unroll
        for (int ks = 0; ks < 3; ++ks)
#pragma unroll
          for (int tt = 0; tt < 4; ++tt)
            acc[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wq[f][ks]),
                                                              __builtin_bit_cast(bf16x8, bx[tt][ks]),
                                                              acc[tt], 0, 0, 0);
        // acc[tt][jj]: feature 16 ft + 4 g + jj, token 16 tt + c16
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          const f32x2 lo = {acc[tt][0], acc[tt][1]}, hi = {acc[tt][2], acc[tt][3]};
          const u32x2 pk = {__builtin_bit_cast(unsigned, __builtin_convertvector(lo, bf16x2)),
                            __builtin_bit_cast(unsigned, __builtin_convertvector(hi, bf16x2))};
          *(EVT_LDS u32x2*)(L + AT96_QKV + (16 * tt + c16) * AT96_QROW + (16 * ft + 4 * g) * 2) = pk;
        }
      }
    }
    __syncthreads();
    // ---- P2: attention units (h, query tile `wave`), h = 0..2 ----
    // the bias from the LDS tables as in window_attn_bf16_kernel (T[a(q) - b(k)], the SW-MSA
    // region mask and the keys past 48 as -inf); the next window's x prefetch lands during P2 / P3
    const int qt = wave;
    if (wg + (int)gridDim.x < nwin) prefetch(wg + gridDim.x);
    const int wtype = G.type();
    const bool lr_ = wtype & 2, lc_ = wtype & 1;
    const int qq = min(16 * qt + c16, 48), qi = (qq * 37) >> 8, qj = qq - 7 * qi;
    const int toff = AT96_TB + (6 * qi + qq + 84) * 4;
    const unsigned cq = (lr_ && qi >= cut ? 1u : 0u) | (lc_ && qj >= cut ? 2u : 0u);
    const EVT_LDS char* Q = L + AT96_QKV;
#pragma unroll
    for (int h = 0; h < 3; ++h) {
      const u32x4 qf = *(const EVT_LDS u32x4*)(Q + (16 * qt + c16) * AT96_QROW + (32 * h + 8 * g) * 2);
      f32x4 sv[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const u32x4 kf = *(const EVT_LDS u32x4*)(Q + (16 * kt + c16) * AT96_QROW + (96 + 32 * h + 8 * g) * 2);
        sv[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kf),
                                                         __builtin_bit_cast(bf16x8, qf),
                                                         f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      }
      const f32x2 sc2 = {scale_log2, scale_log2};
      const EVT_LDS char* Tq = L + toff + h * RPB_CROW * 4;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        f32x4 bv;
#pragma unroll
        for (int j = 0; j < 4; ++j) bv[j] = *(const EVT_LDS float*)(Tq - kofs[kt][j]);
        const f32x2 lo = f32x2{sv[kt][0], sv[kt][1]} * sc2 + f32x2{bv[0], bv[1]};
        const f32x2 hi = f32x2{sv[kt][2], sv[kt][3]} * sc2 + f32x2{bv[2], bv[3]};
        sv[kt] = f32x4{lo[0], lo[1], hi[0], hi[1]};
        if (wtype) {  // SW-MSA window on the last row / column: keys of another region
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int ki = kij[kt][j] >> 3, kj = kij[kt][j] & 7;
            const unsigned ck = (lr_ && ki >= cut ? 1u : 0u) | (lc_ && kj >= cut ? 2u : 0u);
            if (ck != cq) sv[kt][j] = -INFINITY;
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)  // keys 49 .. 63
        if (4 * g + j > 0) sv[3][j] = -INFINITY;
      float m4[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
        m4[kt] = fmaxf(fmaxf(sv[kt][0], sv[kt][1]), fmaxf(sv[kt][2], sv[kt][3]));
      const float mx = bfly_max_16_32(fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3])));
      float p4[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
        for (int j = 0; j < 4; ++j) sv[kt][j] = __builtin_amdgcn_exp2f(sv[kt][j] - mx);
        p4[kt] = (sv[kt][0] + sv[kt][1]) + (sv[kt][2] + sv[kt][3]);
      }
      const float sum = bfly_sum_16_32((p4[0] + p4[1]) + (p4[2] + p4[3]));
      f32x4 o[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 pf;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pf[j] = (bf16)sv[2 * ks][j];
          pf[4 + j] = (bf16)sv[2 * ks + 1][j];
        }
        const int key0 = ks * 32 + 4 * g + tq;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int col = (192 + 32 * h + 16 * dt + 4 * tp) * 2;
          const i16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((EVT_LDS i16x4*)(Q + key0 * AT96_QROW + col));
          const i16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((EVT_LDS i16x4*)(Q + (key0 + 16) * AT96_QROW + col));
          const i16x8 vv = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
          o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vv), pf, o[dt], 0, 0, 0);
        }
      }
      // o[dt][j] = O^T[d = 16 dt + 4 g + j][query 16 qt + c16]
      const float inv = __builtin_amdgcn_rcpf(sum);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const f32x2 lo = f32x2{o[dt][0], o[dt][1]} * f32x2{inv, inv};
        const f32x2 hi = f32x2{o[dt][2], o[dt][3]} * f32x2{inv, inv};
        const u32x2 pk = {__builtin_bit_cast(unsigned, __builtin_convertvector(lo, bf16x2)),
                          __builtin_bit_cast(unsigned, __builtin_convertvector(hi, bf16x2))};
        *(EVT_LDS u32x2*)(L + AT96_XO + (16 * qt + c16) * AT96_ROW + (32 * h + 16 * dt + 4 * g) * 2) = pk;
      }
    }
    // ---- P3: proj + bias + residual -> xm and its row statistics (token tile `wave`) ----
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's O rows are in LDS
    {
      const int t = 16 * qt + c16;
      const int64_t row = G.row(min(t, 48));
      bf16x4 xr[6];  // residual rows (L2-resident: read by this window's prefetch)
#pragma unroll
      for (int f = 0; f < 6; ++f) xr[f] = *(const bf16x4*)(x + row * 96 + 16 * f + 4 * g);
      u32x4 bo[3];
#pragma unroll
      for (int ks = 0; ks < 3; ++ks)
        bo[ks] = *(const EVT_LDS u32x4*)(L + AT96_XO + t * AT96_ROW + 64 * ks + 16 * g);
      float s1 = 0.f, s2 = 0.f;
      u32x2 ov[6];
#pragma unroll
      for (int f = 0; f < 6; ++f) {
        f32x4 acc = *(const EVT_LDS f32x4*)(L + AT96_CV + (288 + 16 * f + 4 * g) * 4);
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
          const u32x4 wv = *(const EVT_LDS u32x4*)(L + AT96_WP + (16 * f + c16) * AT96_ROW + 64 * ks + 16 * g);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wv),
                                                        __builtin_bit_cast(bf16x8, bo[ks]), acc, 0, 0, 0);
        }
        const f32x4 v = acc + f32x4{(float)xr[f][0], (float)xr[f][1], (float)xr[f][2], (float)xr[f][3]};
        const bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float fv = (float)o[jj];
          s1 += fv;
          s2 += fv * fv;
        }
        ov[f] = __builtin_bit_cast(u32x2, o);
      }
      s1 += __shfl_xor(s1, 16, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 32, 64);
      // xm rows of this token tile staged over its (dead) O rows, then whole-row 16-B stores
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int f = 0; f < 6; ++f)
        *(EVT_LDS u32x2*)(L + AT96_XO + t * AT96_ROW + (16 * f + 4 * g) * 2) = ov[f];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int idx = 64 * i + lane, r = idx / 12, j = idx - r * 12, tr = 16 * qt + r;
        if (tr < 49) {
          const u32x4 v = *(const EVT_LDS u32x4*)(L + AT96_XO + tr * AT96_ROW + j * 16);
          store_b128((bf16*)p.xm + G.row(tr) * 96 + 8 * j, v);
        }
      }
      if (g == 0 && t < 49) {
        float* so = p.stats_out + row * 2 * p.nslots;
        *(f32x2*)so = f32x2{s1, s2};
        for (int k = 1; k < p.nslots; ++k) *(f32x2*)(so + 2 * k) = f32x2{0.f, 0.f};
      }
    }
  }
}

// ---- fused patch embedding of the 3-channel, 4x4-patch, C = 96 stem (Swin-T / Swin-S) ---------
// Conv2d(3, 96, k = s = 4) + the embedding LayerNorm(96) -> stage-1 stream x (bf16) and its row
// statistics in one pass. The three-kernel path (im2col rows, the Dense GEMM writing the bf16
// conv output, ln_rows_kernel reading it back) moves the 154 MB fp32 image plus 3 x 154 MB of
// bf16 rows at bs256; this one reads the image and writes x.
//   Persistent blocks (4 per CU) walk patch rows (image b, row py); the fp32 image strip
//   [c][kh][S] of the NEXT patch row is loaded into registers while the current one is computed
//   (coalesced 16-B loads), then written to LDS. Wave = token tile (16 patches); per tile
//   C^T = W . P^T on v_mfma_f32_16x16x32_bf16 (K = 48 in two k-steps; the packed weight's K
//   padding is zero, W in LDS with 144-B rows), the B operand built from two LDS float4 reads per
//   lane (8 consecutive k = (c, kh, kw) are kh = 2q, 2q + 1 of one channel, 4 kw each). Conv output
//   + bias stays fp32 into the LayerNorm (two-pass mean / variance over the token's 96 features:
//   24 per lane, 4 lane groups); the stored bf16 values' (sum, sumsq) go to slot 0; x rows are
//   staged in LDS and leave as whole 192-B rows.
constexpr int EMB96_WROW = 144;  // W rows: 64 bf16 (48 + zero pad) + 16 B against bank conflicts
constexpr int EMB96_XROW = 208;  // staged x rows: 96 bf16 + pad
constexpr int EMB96_PF = 3;      // strip float4 per thread in flight (12 rows x S/4 <= 768)

__global__ __launch_bounds__(256) void swin_embed96_kernel(SwinEmbedParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int S = p.S, R = S / 4, q4 = S / 4;
  EVT_LDS char* ws = (EVT_LDS char*)smem;
  EVT_LDS float* strip = (EVT_LDS float*)(smem + 96 * EMB96_WROW);  // [12][S]
  EVT_LDS char* xs = (EVT_LDS char*)strip + 12 * S * 4;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  const int nrow = p.B * R;  // patch rows (b, py)
  for (int e = tid; e < 96 * 8; e += 256) {
    const int n = e >> 3, c = e & 7;
    *(EVT_LDS u32x4*)(ws + n * EMB96_WROW + 16 * c) =
        *(const u32x4*)((const bf16*)p.w + (int64_t)n * p.ldw + 8 * c);
  }
  f32x4 pf[EMB96_PF];
  auto fetch = [&](int pr) {  // strip of patch row pr: row (c, kh) = img[b][c][4 py + kh][0 .. S)
    const int b = pr / R, py = pr - b * R;
#pragma unroll
    for (int k = 0; k < EMB96_PF; ++k) {
      const int e = tid + 256 * k, r = e / q4, i = e - r * q4;
      if (r < 12) {
        const int c = r >> 2, kh = r & 3;
        pf[k] = *(const f32x4*)(p.img + (((int64_t)b * 3 + c) * S + 4 * py + kh) * S + 4 * i);
      }
    }
  };
  if ((int)blockIdx.x < nrow) fetch(blockIdx.x);
  const float inv_d = 1.0f / 96.0f;
  const int ntt = (R + 15) / 16;
  for (int pr = blockIdx.x; pr < nrow; pr += gridDim.x) {
    __syncthreads();  // the previous row's strip / staging readers are done
#pragma unroll
    for (int k = 0; k < EMB96_PF; ++k) {
      const int e = tid + 256 * k;
      if (e < 12 * q4) *(EVT_LDS f32x4*)(strip + 4 * e) = pf[k];  // [r][S] = e / q4, 4 (e % q4)
    }
    __syncthreads();
    if (pr + (int)gridDim.x < nrow) fetch(pr + gridDim.x);  // lands during this row's compute
    const int b = pr / R, py = pr - b * R;
    for (int tt = wave; tt < ntt; tt += 4) {
      const int j = 16 * tt + c16;  // this lane's patch (token) in the row
      const bool ok = j < R;
      u32x4 bx[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int gq = 4 * ks + g;  // k = 8 gq .. 8 gq + 7: channel gq >> 1, kh 2 (gq & 1) + {0, 1}
        bx[ks] = u32x4{0u, 0u, 0u, 0u};
        if (gq < 6 && ok) {
          const int r0 = (gq >> 1) * 4 + 2 * (gq & 1);
          const f32x4 a0 = *(const EVT_LDS f32x4*)(strip + r0 * S + 4 * j);
          const f32x4 a1 = *(const EVT_LDS f32x4*)(strip + (r0 + 1) * S + 4 * j);
          bx[ks][0] = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a0[0], a0[1]}, bf16x2));
          bx[ks][1] = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a0[2], a0[3]}, bf16x2));
          bx[ks][2] = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a1[0], a1[1]}, bf16x2));
          bx[ks][3] = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a1[2], a1[3]}, bf16x2));
        }
      }
      f32x4 acc[6];
#pragma unroll
      for (int ft = 0; ft < 6; ++ft) {
        acc[ft] = load4(p.bias + 16 * ft + 4 * g);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const u32x4 wv = *(const EVT_LDS u32x4*)(ws + (16 * ft + c16) * EMB96_WROW + 64 * ks + 16 * g);
          acc[ft] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wv),
                                                            __builtin_bit_cast(bf16x8, bx[ks]), acc[ft], 0, 0, 0);
        }
      }
      // acc[ft][jj]: feature 16 ft + 4 g + jj of patch j; LayerNorm over the 96 features
      float s = 0.f;
#pragma unroll
      for (int ft = 0; ft < 6; ++ft) s += (acc[ft][0] + acc[ft][1]) + (acc[ft][2] + acc[ft][3]);
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      const float mean = s * inv_d;
      float v2 = 0.f;
#pragma unroll
      for (int ft = 0; ft < 6; ++ft)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) v2 += (acc[ft][jj] - mean) * (acc[ft][jj] - mean);
      v2 += __shfl_xor(v2, 16, 64);
      v2 += __shfl_xor(v2, 32, 64);
      const float rstd = rsqrtf(v2 * inv_d + p.eps);
      float s1 = 0.f, s2 = 0.f;
      EVT_LDS char* xrow = xs + (16 * wave + c16) * EMB96_XROW;
#pragma unroll
      for (int ft = 0; ft < 6; ++ft) {
        const f32x4 gm = load4(p.gamma + 16 * ft + 4 * g), bt = load4(p.beta + 16 * ft + 4 * g);
        const f32x4 y = (acc[ft] - mean) * rstd * gm + bt;
        const bf16x4 o = {(bf16)y[0], (bf16)y[1], (bf16)y[2], (bf16)y[3]};
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float f = (float)o[jj];
          s1 += f;
          s2 += f * f;
        }
        *(EVT_LDS bf16x4*)(xrow + (16 * ft + 4 * g) * 2) = o;
      }
      s1 += __shfl_xor(s1, 16, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 32, 64);
      const int64_t row0 = ((int64_t)b * R + py) * R + 16 * tt;  // stream row of patch 16 tt
      if (g == 0 && ok) {
        float* st = p.stats + (row0 + c16) * 2 * p.nslots;
        *(f32x2*)st = f32x2{s1, s2};
        for (int k = 1; k < p.nslots; ++k) *(f32x2*)(st + 2 * k) = f32x2{0.f, 0.f};
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // the wave's 16 staged rows leave as whole 192-B rows (12 lanes x 16 B each)
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int idx = 64 * i + lane, r = idx / 12, c = idx - r * 12;
        if (16 * tt + r < R) {
          const u32x4 v = *(const EVT_LDS u32x4*)(xs + (16 * wave + r) * EMB96_XROW + 16 * c);
          store_b128((bf16*)p.x + (row0 + r) * 96 + 8 * c, v);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staging reads done before reuse
    }
  }
}

template <typename T, int LPR, int NC>
hipError_t ln_rows_lc(const void* x, int64_t ld, void* y, const float* g, const float* bb,
                      int rows, int D, float eps, float* stats, int nslots, hipStream_t s) {
  const int rows_per_block = 4 * (64 / LPR);
  hipLaunchKernelGGL((ln_rows_kernel<T, LPR, NC>), dim3((rows + rows_per_block - 1) / rows_per_block),
                     dim3(256), 0, s, (const T*)x, ld, (T*)y, g, bb, rows, D, eps, stats, nslots);
  return hipGetLastError();
}

template <typename T>
hipError_t ln_rows_t(const void* x, int64_t ld, void* y, const float* g, const float* bb, int rows,
                     int D, float eps, float* stats, int nslots, hipStream_t s) {
  constexpr int V = 16 / sizeof(T);
  // lanes per row: enough to cover the row in <= 4 chunks each, and >= nslots (slot writers)
  if (ld <= 8 * V && nslots <= 8)
    return ln_rows_lc<T, 8, 1>(x, ld, y, g, bb, rows, D, eps, stats, nslots, s);
  if (ld <= 16 * V && nslots <= 16)
    return ln_rows_lc<T, 16, 1>(x, ld, y, g, bb, rows, D, eps, stats, nslots, s);
  if (ld <= 32 * V)
    return ln_rows_lc<T, 32, 1>(x, ld, y, g, bb, rows, D, eps, stats, nslots, s);
  if (ld <= 64 * V) return ln_rows_lc<T, 64, 1>(x, ld, y, g, bb, rows, D, eps, stats, nslots, s);
  if (ld <= 128 * V) return ln_rows_lc<T, 64, 2>(x, ld, y, g, bb, rows, D, eps, stats, nslots, s);
  return ln_rows_lc<T, 64, 4>(x, ld, y, g, bb, rows, D, eps, stats, nslots, s);
}

}  // namespace

hipError_t swin_patch_launch(int dtype, const float* img, int B, int C, int S, int ps, void* out,
                             int ldo, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (S % ps || C * ps * ps > ldo || ldo % 8 || (ps * S) % 4) return hipErrorInvalidValue;
  const size_t lds = (size_t)C * ps * S * sizeof(float);
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  const dim3 grid(S / ps, B);
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(swin_patch_kernel<bf16>, grid, dim3(256), lds, s, img, C, S, ps,
                       (bf16*)out, ldo);
  else
    hipLaunchKernelGGL(swin_patch_kernel<float>, grid, dim3(256), lds, s, img, C, S, ps,
                       (float*)out, ldo);
  return hipGetLastError();
}

hipError_t ln_rows_launch(int dtype, const void* x, int64_t ld, void* y, const float* gamma,
                          const float* beta, int rows, int D, float eps, float* stats, int nslots,
                          hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  if (D <= 0 || D > ld || ld > 1024 || nslots > 64 || ld % (dtype == DT_BF16 ? 8 : 4) ||
      D % (dtype == DT_BF16 ? 8 : 4))
    return hipErrorInvalidValue;
  return dtype == DT_BF16 ? ln_rows_t<bf16>(x, ld, y, gamma, beta, rows, D, eps, stats, nslots, s)
                          : ln_rows_t<float>(x, ld, y, gamma, beta, rows, D, eps, stats, nslots, s);
}

hipError_t merge_launch(int dtype, const void* x, int64_t ldx, int B, int R, int C, void* out,
                        float* stats, int nslots, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (R % 2 || C <= 0 || C > ldx || nslots > 64 || C % 8 || ldx % 8) return hipErrorInvalidValue;
  const int64_t rows = (int64_t)B * (R / 2) * (R / 2);
  const dim3 grid((unsigned)((rows + 3) / 4));
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(merge_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)x, ldx, B, R, C,
                       (bf16*)out, stats, nslots);
  else
    hipLaunchKernelGGL(merge_kernel<float>, grid, dim3(256), 0, s, (const float*)x, ldx, B, R, C,
                       (float*)out, stats, nslots);
  return hipGetLastError();
}

hipError_t rpb_dense_launch(const float* table, int H, int w, int shift, float* dense,
                            hipStream_t s) {
  const int n = (shift ? 4 : 1) * H * w * w * 64;
  hipLaunchKernelGGL(rpb_dense_kernel, dim3((n + 255) / 256), dim3(256), 0, s, table, H, w, shift,
                     dense);
  if (w == 7)  // + the compact per-head tables of the bf16 window kernel
    hipLaunchKernelGGL(rpb_compact_kernel, dim3((H * RPB_CROW + 255) / 256), dim3(256), 0, s, table,
                       H, const_cast<float*>(rpb_compact(dense, H, shift)));
  return hipGetLastError();
}

size_t rpb_table_floats(int H, int w, int shift) {
  return (size_t)(shift ? 4 : 1) * H * w * w * 64 + (size_t)H * RPB_CROW;
}

hipError_t window_attn_launch(int dtype, const SwinAttnParams& p, hipStream_t s) {
  if (p.B <= 0) return hipSuccess;
  if (p.R % 7 || p.nwx * 7 != p.R || p.C != p.H * 32 || p.ldo < p.C || p.shift < 0 ||
      p.shift >= 7 || (p.ldq % 8) || (p.ldo % 4))
    return hipErrorInvalidValue;
  const int64_t pairs = (int64_t)p.B * p.nwx * p.nwx * p.H;
  const dim3 grid((unsigned)((pairs + 3) / 4));
  // bf16 kernel: 32-bit (image, window, head) index and per-image 32-bit buffer offsets
  if (dtype == DT_BF16 && (pairs + 4 >= (int64_t)1 << 31 ||
                           (int64_t)p.R * p.R * std::max(p.ldq, p.ldo) * 2 >= (int64_t)1 << 31))
    return hipErrorInvalidValue;
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(window_attn_bf16_kernel, grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(window_attn_f32_kernel, grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t swin_mlp96_launch(const SwinMlpParams& p, hipStream_t s) {
  if (p.M <= 0) return hipSuccess;
  if (p.nslots < 1 || p.nslots > 4 || p.ldw1 < MLP96_C || p.ldw2 < MLP96_F || p.ldw1 % 8 ||
      p.ldw2 % 8)
    return hipErrorInvalidValue;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipFuncSetAttribute((const void*)swin_mlp96_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, MLP96_LDS);
  }
  const int waves = (p.M + 31) / 32;
  const int grid = std::max(1, std::min(ncu, (waves + MLP96_WAVES - 1) / MLP96_WAVES));
  hipLaunchKernelGGL(swin_mlp96_kernel, dim3(grid), dim3(64 * MLP96_WAVES), MLP96_LDS, s, p);
  return hipGetLastError();
}

hipError_t swin_attn96_launch(const SwinAttnBlockParams& p, hipStream_t s) {
  if (p.B <= 0) return hipSuccess;
  if (p.R % 7 || p.shift < 0 || p.shift >= 7 || p.nslots < 1 || p.nslots > 4 || p.ldq < 96 ||
      p.ldp < 96 || p.ldq % 8 || p.ldp % 8)
    return hipErrorInvalidValue;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipFuncSetAttribute((const void*)swin_attn96_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, AT96_LDS);
  }
  const int windows = p.B * (p.R / 7) * (p.R / 7);
  hipLaunchKernelGGL(swin_attn96_kernel, dim3(std::min(windows, 2 * ncu)), dim3(256), AT96_LDS, s, p);
  return hipGetLastError();
}

hipError_t swin_embed96_launch(const SwinEmbedParams& p, hipStream_t s) {
  if (p.B <= 0) return hipSuccess;
  if (p.S % 16 || 3 * p.S > 256 * EMB96_PF || p.ldw < 64 || p.ldw % 8 || p.nslots < 1 ||
      p.nslots > 4)
    return hipErrorInvalidValue;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  }
  const size_t lds = (size_t)96 * EMB96_WROW + 12 * p.S * 4 + 64 * EMB96_XROW;
  const int rows = p.B * (p.S / 4);
  hipLaunchKernelGGL(swin_embed96_kernel, dim3(std::min(rows, 4 * ncu)), dim3(256), lds, s, p);
  return hipGetLastError();
}

hipError_t merge_stats_launch(const float* src, int ns, int B, int R, float* dst, int nd,
                              hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (R % 2 || ns < 1 || nd < 1) return hipErrorInvalidValue;
  const int64_t rows = (int64_t)B * (R / 2) * (R / 2);
  hipLaunchKernelGGL(merge_stats_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, src,
                     ns, B, R, dst, nd);
  return hipGetLastError();
}

hipError_t ln_pool_launch(int dtype, const void* x, int64_t ldx, int B, int T, int D,
                          const float* stats, int nslots, const float* gamma, const float* beta,
                          void* out, int64_t ldo, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (T <= 0 || T > 256 || D > ldo) return hipErrorInvalidValue;
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(ln_pool_kernel<bf16>, dim3(B), dim3(256), 0, s, (const bf16*)x, ldx, T, D,
                       stats, nslots, gamma, beta, 1e-5f, (bf16*)out, ldo);
  else
    hipLaunchKernelGGL(ln_pool_kernel<float>, dim3(B), dim3(256), 0, s, (const float*)x, ldx, T, D,
                       stats, nslots, gamma, beta, 1e-5f, (float*)out, ldo);
  return hipGetLastError();
}

}  // namespace evt
