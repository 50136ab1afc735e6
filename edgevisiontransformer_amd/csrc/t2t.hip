// Tokens-to-token (T2T) stage of T2T-ViT on gfx950: soft split (unfold) and TokenPerformer.
//
// Reference: `modeling/models/t2t_vit.py:7-88` (tf_Unfold, T2T_module) and
// `modeling/layers/transformer_encoder.py:39-101` (TokenPerformer). Per performer:
//
//   unfold_kernel       NHWC [B,H,W,C] -> rows [B*OH*OW][ldo] in (kh, kw, c) order (extract_patches,
//                       channel_last), zero padded past k*k*C, + per-row (sum, sumsq) for the
//                       LayerNorm norm1 that is folded into the kqv GEMM (gemm.hip, EPI_LNIN)
//   kqv GEMM            (gemm.hip) LN1-folded Dense(3*64) + bias -> [rows][192] = (k | q | v)
//   performer_kv_kernel per (image, token chunk): kp = prm_exp(k); partial sum_t kp [m] and
//                       kptv = v^T kp [64][m] (fixed-order, no atomics)
//   performer_out_kernel per (image, token range): kptv, ksum = fixed-order sum of the chunk
//                       partials; per token qp = prm_exp(q), D = qp . ksum,
//                       y = v + Dense(qp kptv^T / (D + 1e-8)), out = y + FFN(LN2(y)) -> [rows][64]
//
// The per-token chains in the performer kernels run on MFMA with the operands never leaving
// registers: products are formed transposed (out^T = W^T in^T), so the 16x16 accumulator of one
// step (lane l: 4 consecutive features 4(l>>4)+j of token l&15) is exactly the B operand of the
// next 16x16x16 step (bf16: v_mfma_f32_16x16x16_bf16; f32: 4 x v_mfma_f32_16x16x4_f32 over the
// same k-permutation). Weights live in LDS as [out][in] fp32 rows with the 16-B chunk q of row r
// stored at q ^ (r & 15) (conflict-free fragment reads).
#include <type_traits>

#include "common.h"
#include "evt_internal.h"

namespace evt {

namespace {

constexpr int PF_HS = 64;  // TokenPerformer head size (token_size)
constexpr int PF_M = 32;   // random features m = int(64 * 0.5)
constexpr int PF_PART = PF_HS * PF_M + PF_M;  // floats per (image, chunk) partial: kptv + ksum

// acc[n][col] += sum_{k<16} A[n][k] B[k][col]. Lane l supplies a[s] = A[l&15][4(l>>4)+s] and
// b[s] = B[4(l>>4)+s][l&15] (s = 0..3): b is a 16x16 accumulator fragment of the previous step.
// The A fragment comes pre-converted (Afrag<T>): weight fragments are loop-invariant and get
// hoisted into registers, so the bf16 path keeps them at 2 VGPRs each.
template <typename T> struct Afrag;
template <> struct Afrag<bf16> {
  i16x4 v;
  Afrag() = default;
  __device__ __forceinline__ explicit Afrag(const f32x4& a) {
    const bf16x4 h = {(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3]};
    v = __builtin_bit_cast(i16x4, h);
  }
};
template <> struct Afrag<float> {
  f32x4 v;
  Afrag() = default;
  __device__ __forceinline__ explicit Afrag(const f32x4& a) : v(a) {}
};
template <typename T> __device__ __forceinline__ void chain16(f32x4& acc, const Afrag<T>& a, const f32x4& b);
template <> __device__ __forceinline__ void chain16<bf16>(f32x4& acc, const Afrag<bf16>& a, const f32x4& b) {
  const bf16x4 bh = {(bf16)b[0], (bf16)b[1], (bf16)b[2], (bf16)b[3]};
  acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a.v, __builtin_bit_cast(i16x4, bh), acc, 0, 0, 0);
}
template <> __device__ __forceinline__ void chain16<float>(f32x4& acc, const Afrag<float>& a, const f32x4& b) {
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[s], b[s], acc, 0, 0, 0);
}

// Swizzled fp32 LDS matrix with 64-float rows: element (r, c) at r*64 + (((c>>2) ^ (r&15))<<2) + (c&3).
__device__ __forceinline__ int swz64(int r, int c) { return r * 64 + ((((c >> 2) ^ (r & 15))) << 2) + (c & 3); }

// A fragment of rows [16*rt, 16*rt+16), k columns [16*kc, 16*kc+16) of a swz64 matrix.
__device__ __forceinline__ f32x4 afrag(const EVT_LDS float* M, int rt, int kc, int lane) {
  const int r = 16 * rt + (lane & 15);
  const int q = 4 * kc + (lane >> 4);
  return *(const EVT_LDS f32x4*)(M + r * 64 + ((q ^ (r & 15)) << 2));
}

// Sum over the 4 lanes that hold one token (lanes l, l^16, l^32, l^48).
__device__ __forceinline__ float token_sum(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

// One wave per output row, RPW consecutive rows per wave (neighbouring windows overlap, so the
// input stays cache-resident). Every lane owns VW consecutive output elements per access
// (VW = 4: 4 channels of one pixel, C % 4 == 0; VW = 2: an element pair, which may straddle a
// pixel, ldo even; VW = 1 otherwise), decomposed into (kh, kw, c) once per lane; per row only the
// window origin changes. At most 4 accesses per lane (ldo <= 256 * VW).
template <typename TI, typename TO, int VW>
__global__ __launch_bounds__(256) void unfold_kernel(const TI* __restrict__ in, int B, int H, int W,
                                                     int C, int k, int s, int p, int OH, int OW,
                                                     TO* __restrict__ out, int ldo,
                                                     float* __restrict__ stats, int nslots,
                                                     int rpw) {
  constexpr int NE = VW == 4 ? 1 : VW;  // independently decomposed elements per access
  const int lane = threadIdx.x & 63;
  const int kc = k * C, kk = k * kc;
  int rel[4][NE], ekh[4][NE], ekw[4][NE];
  bool inw[4][NE], col[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    col[i] = (lane + 64 * i) * VW < ldo;
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const int e = (lane + 64 * i) * VW + j;
      inw[i][j] = e < kk;
      const int kh = inw[i][j] ? e / kc : 0, r2 = e - kh * kc, kw = inw[i][j] ? r2 / C : 0;
      ekh[i][j] = kh;
      ekw[i][j] = kw;
      rel[i][j] = (kh * W + kw) * C + (r2 - kw * C);
    }
  }
  const int rows = B * OH * OW;  // < 2^31 (checked on the host)
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * rpw;
  if (row0 >= rows) return;
  // window of the first row, then stepped (no per-row integer division)
  int b = row0 / (OH * OW), rem = row0 - b * OH * OW;
  int oh = rem / OW, ow = rem - oh * OW;
  for (int r = 0; r < rpw; ++r, ++ow) {
    const int row = row0 + r;
    if (row >= rows) return;
    if (ow == OW) {
      ow = 0;
      if (++oh == OH) {
        oh = 0;
        ++b;
      }
    }
    const int ih0 = oh * s - p, iw0 = ow * s - p;
    const TI* win = in + (int64_t)b * H * W * C + ((int64_t)ih0 * W + iw0) * C;
    TO* orow = out + (int64_t)row * ldo;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (!col[i]) continue;
      const int e = (lane + 64 * i) * VW;
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < NE; ++j) {
        const int ih = ih0 + ekh[i][j], iw = iw0 + ekw[i][j];
        const bool ok = inw[i][j] && ih >= 0 && ih < H && iw >= 0 && iw < W;
        if constexpr (VW == 4) {
          if (ok) v = load4(win + rel[i][j]);
        } else {
          v[j] = ok ? to_f32(win[rel[i][j]]) : 0.f;
        }
      }
      if constexpr (VW == 4) {
        store4(orow + e, v);
      } else if constexpr (VW == 2) {
        if constexpr (sizeof(TO) == 2) {
          const bf16x2 o = {(bf16)v[0], (bf16)v[1]};
          *(bf16x2*)(orow + e) = o;
        } else {
          *(f32x2*)(orow + e) = f32x2{v[0], v[1]};
        }
      } else {
        orow[e] = from_f32<TO>(v[0]);
      }
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        const float q = to_f32(from_f32<TO>(v[j]));
        s1 += q;
        s2 += q * q;
      }
    }
    if (stats) {
      s1 = wave_sum(s1);
      s2 = wave_sum(s2);
      if (lane < nslots) {
        float* st = stats + 2 * ((int64_t)row * nslots + lane);
        st[0] = lane == 0 ? s1 : 0.f;
        st[1] = lane == 0 ? s2 : 0.f;
      }
    }
  }
}

// kp = prm_exp(k) of one 16-token tile from the random-feature fragments fw (2 m tiles x 4 k
// chunks): returns the 2 accumulator fragments (m tiles).
template <typename T>
__device__ __forceinline__ void prm_tile(const Afrag<T> (&fw)[2][4], const f32x4 (&z)[4], float zd,
                                         float inv_sqrt_m, f32x4 (&out)[2]) {
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c) chain16<T>(acc, fw[mt][c], z[c]);
#pragma unroll
    for (int j = 0; j < 4; ++j) out[mt][j] = __expf(acc[j] - zd) * inv_sqrt_m;
  }
}

template <typename T, int R, int K>
__device__ __forceinline__ void load_afrags(const EVT_LDS float* M, int lane, Afrag<T> (&f)[R][K]) {
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int k = 0; k < K; ++k) f[r][k] = Afrag<T>(afrag(M, r, k, lane));
}

// One token row's 64 features of column block `col0` of the kqv matrix as 4 B fragments.
template <typename T>
__device__ __forceinline__ void load_frags(const T* rowp, bool valid, int lane, f32x4 (&f)[4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c)
    f[c] = valid ? load4(rowp + 16 * c + 4 * (lane >> 4)) : f32x4{0.f, 0.f, 0.f, 0.f};
}

// kptv^T-tile contraction over 16 tokens on MFMA: acc[j] += sum_t A[l&15][t] B[t][...] with A frags
// (i = l & 15, k = t = 4(l>>4)+s) and B frags (k = t, j = l & 15) read as 4 consecutive tokens
// from the per-wave transposed LDS tiles.
template <typename T> __device__ __forceinline__ void tmma(f32x4& acc, const f32x4& a, const f32x4& b);
template <> __device__ __forceinline__ void tmma<bf16>(f32x4& acc, const f32x4& a, const f32x4& b) {
  const bf16x4 ah = {(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3]};
  const bf16x4 bh = {(bf16)b[0], (bf16)b[1], (bf16)b[2], (bf16)b[3]};
  acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(i16x4, ah),
                                                  __builtin_bit_cast(i16x4, bh), acc, 0, 0, 0);
}
template <> __device__ __forceinline__ void tmma<float>(f32x4& acc, const f32x4& a, const f32x4& b) {
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], acc, 0, 0, 0);
}

// grid (nchunk, B), block 256 (4 waves; wave w takes tiles w, w+4, ... of the chunk).
// Per 16-token tile: kp = prm_exp(k) (MFMA chain), ksum partial (VALU), and
// kptv[n][m] += sum_t v[t][n] kp[t][m] as 8 MFMAs (n tiles x m tiles, k = the 16 tokens): v and kp
// are written transposed ([feature][token], fp32) to the wave's LDS so that each lane reads 4
// consecutive tokens of one feature as its operand fragment.
// PERM (bf16 model path): the kqv GEMM's output columns are stored permuted within each 64-feature
// block (kqv_col): lane group g's 16 features {16 c + 4 g + j} sit at columns 16 g .. 16 g + 15,
// so a lane reads its 4 fragments of a row as two 16-B loads instead of four 8-B ones (round-4
// counters: both performer kernels were texture-data-unit bound on the 8-B loads).
__host__ __device__ constexpr int kqv_col(int f) { return 16 * ((f >> 2) & 3) + 4 * (f >> 4) + (f & 3); }

// the lane's 4 fragments (features 16 c + 4 (lane >> 4) + j) of one 64-feature block of a row
template <typename T, bool PERM>
__device__ __forceinline__ void load_block(const T* rowp, bool valid, int lane, f32x4 (&f)[4]) {
  if constexpr (PERM) {
    u32x4 h[2] = {u32x4{0u, 0u, 0u, 0u}, u32x4{0u, 0u, 0u, 0u}};
    if (valid) {
      h[0] = *(const u32x4*)(rowp + 16 * (lane >> 4));
      h[1] = *(const u32x4*)(rowp + 16 * (lane >> 4) + 8);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bf16x8 v = __builtin_bit_cast(bf16x8, h[c >> 1]);
      const int o = 4 * (c & 1);
      f[c] = f32x4{(float)v[o], (float)v[o + 1], (float)v[o + 2], (float)v[o + 3]};
    }
  } else {
    load_frags(rowp, valid, lane, f);
  }
}

template <typename T, bool PERM = false>
__global__ __launch_bounds__(256) void performer_kv_kernel(const T* __restrict__ kqv, int64_t ldq,
                                                           int ntok, int chunk,
                                                           const float* __restrict__ prmw,
                                                           float* __restrict__ part) {
  static_assert(!PERM || std::is_same<T, bf16>::value, "permuted kqv: bf16 path");
  constexpr int TS = 20;  // floats per transposed row (16 tokens + 4 pad: conflict-light writes)
  constexpr int TILES = 4 * (PF_HS + PF_M) * TS;
  __shared__ __attribute__((aligned(16))) float smem[PF_M * 64 + (TILES > 4 * PF_PART ? TILES : 4 * PF_PART)];
  EVT_LDS float* wS = (EVT_LDS float*)smem;                          // [32][64] swz64
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  EVT_LDS float* vT = wS + PF_M * 64 + wave * (PF_HS + PF_M) * TS;  // [64 n][TS] (tokens)
  EVT_LDS float* kT = vT + PF_HS * TS;                               // [32 m][TS]
  EVT_LDS float* red = wS + PF_M * 64;  // [4][PF_PART], over the tiles once every wave is done
  const int b = blockIdx.y, ci = blockIdx.x;
  for (int i = tid; i < PF_M * PF_HS; i += 256) wS[swz64(i >> 6, i & 63)] = prmw[i];
  __syncthreads();
  Afrag<T> fw[2][4];
  load_afrags<T>(wS, lane, fw);
  const int t_lo = ci * chunk, t_hi = min(ntok, t_lo + chunk);
  const float inv_sqrt_m = 1.0f / sqrtf((float)PF_M);
  f32x4 acc[4][2];  // kptv[n = 16 nt + 4 (l>>4) + j][m = 16 mt + (l & 15)]
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) acc[nt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ks[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // ksum partial, m = 16mt + 4(l>>4) + j
  const int tr = lane & 15, g4 = 4 * (lane >> 4);
  // PERM (the model's bf16 path): the next tile's raw k / v pieces are loaded while this one runs
  // (round 5: the loads were issued and consumed in the same iteration, 65 % of the wave cycles in
  // s_waitcnt); a row past the chunk loads the chunk's first row and is zeroed on use
  u32x4 rk[2], rv[2];
  auto raw = [&](int t0n) {
    const int tn = t0n + tr;
    const T* rowp = kqv + ((int64_t)b * ntok + (tn < t_hi ? tn : t_lo)) * ldq + 16 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      rk[i] = *(const u32x4*)(rowp + 8 * i);
      rv[i] = *(const u32x4*)(rowp + 2 * PF_HS + 8 * i);
    }
  };
  if constexpr (PERM) {
    if (t_lo + 16 * wave < t_hi) raw(t_lo + 16 * wave);
  }
  for (int t0 = t_lo + 16 * wave; t0 < t_hi; t0 += 64) {
    const int t = t0 + tr;
    const bool valid = t < t_hi;
    const T* rowp = kqv + ((int64_t)b * ntok + t) * ldq;
    f32x4 kf[4], vf[4];
    if constexpr (PERM) {  // the same fragments as load_block<T, true>
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const bf16x8 kv8 = __builtin_bit_cast(bf16x8, rk[c >> 1]), vv8 = __builtin_bit_cast(bf16x8, rv[c >> 1]);
        const int o = 4 * (c & 1);
        kf[c] = valid ? f32x4{(float)kv8[o], (float)kv8[o + 1], (float)kv8[o + 2], (float)kv8[o + 3]}
                      : f32x4{0.f, 0.f, 0.f, 0.f};
        vf[c] = valid ? f32x4{(float)vv8[o], (float)vv8[o + 1], (float)vv8[o + 2], (float)vv8[o + 3]}
                      : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      if (t0 + 64 < t_hi) raw(t0 + 64);
    } else {
      load_block<T, PERM>(rowp, valid, lane, kf);              // k = columns [0, 64) (split order k, q, v)
      load_block<T, PERM>(rowp + 2 * PF_HS, valid, lane, vf);  // v = columns [128, 192)
    }
    float kd = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) kd += kf[c][0] * kf[c][0] + kf[c][1] * kf[c][1] + kf[c][2] * kf[c][2] + kf[c][3] * kf[c][3];
    kd = 0.5f * token_sum(kd);
    f32x4 kp[2];
    prm_tile<T>(fw, kf, kd, inv_sqrt_m, kp);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      if (!valid) kp[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        ks[mt * 4 + j] += kp[mt][j];
        kT[(16 * mt + g4 + j) * TS + tr] = kp[mt][j];
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) vT[(16 * c + g4 + j) * TS + tr] = vf[c][j];
    __builtin_amdgcn_wave_barrier();
    f32x4 kb[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) kb[mt] = *(const EVT_LDS f32x4*)(kT + (16 * mt + tr) * TS + g4);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const f32x4 va = *(const EVT_LDS f32x4*)(vT + (16 * nt + tr) * TS + g4);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) tmma<T>(acc[nt][mt], va, kb[mt]);
    }
    __builtin_amdgcn_wave_barrier();
  }
  // ksum: reduce over the 16 lanes sharing (l >> 4)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) ks[i] += __shfl_xor(ks[i], o, 64);
  }
  __syncthreads();  // every wave's tile loop is done: `red` reuses the tile area
  EVT_LDS float* myred = red + wave * PF_PART;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) myred[(16 * nt + g4 + j) * PF_M + 16 * mt + tr] = acc[nt][mt][j];
  if ((lane & 15) == 0) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) myred[PF_HS * PF_M + 16 * mt + 4 * (lane >> 4) + j] = ks[mt * 4 + j];
  }
  __syncthreads();
  float* dst = part + ((int64_t)b * gridDim.x + ci) * PF_PART;
  for (int i = tid; i < PF_PART; i += 256)
    dst[i] = ((red[i] + red[PF_PART + i]) + red[2 * PF_PART + i]) + red[3 * PF_PART + i];
}

// grid (ceil(ntok / span), B), block 256. LDS ~74 KB.
template <typename T>
__global__ __launch_bounds__(256, sizeof(T) == 2 ? 2 : 1) void performer_out_kernel(const T* __restrict__ kqv, int64_t ldq,
                                                            int ntok, int span,
                                                            const float* __restrict__ part,
                                                            int nchunk, PerformerWeights pw,
                                                            T* __restrict__ out, int64_t ldo) {
  extern __shared__ __attribute__((aligned(16))) float dsm[];
  EVT_LDS float* wS = (EVT_LDS float*)dsm;     // [32][64]
  EVT_LDS float* kvS = wS + PF_M * 64;         // [64][64] (m < 32 used)
  EVT_LDS float* woS = kvS + 64 * 64;          // [n][k]
  EVT_LDS float* w1S = woS + 64 * 64;
  EVT_LDS float* w2S = w1S + 64 * 64;
  EVT_LDS float* vec = w2S + 64 * 64;          // ksum[64 (32 used)], bo, b1, b2, g2, be2
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.y;
  for (int i = tid; i < PF_M * PF_HS; i += 256) wS[swz64(i >> 6, i & 63)] = pw.prmw[i];
  for (int i = tid; i < 64 * 64; i += 256) {
    const int kr = i >> 6, nc = i & 63;  // Keras [in = kr][out = nc] -> LDS [out][in]
    woS[swz64(nc, kr)] = pw.out_w[i];
    w1S[swz64(nc, kr)] = pw.fc1_w[i];
    w2S[swz64(nc, kr)] = pw.fc2_w[i];
  }
  // kptv / ksum of this image: fixed-order sum of the chunk partials
  const float* pb = part + (int64_t)b * nchunk * PF_PART;
  for (int i = tid; i < PF_PART; i += 256) {
    float v = 0.f;
    for (int c = 0; c < nchunk; ++c) v += pb[(int64_t)c * PF_PART + i];
    if (i < PF_HS * PF_M) kvS[swz64(i / PF_M, i % PF_M)] = v;
    else vec[i - PF_HS * PF_M] = v;
  }
  for (int i = tid; i < 64; i += 256) {
    vec[64 + i] = pw.out_b[i];
    vec[128 + i] = pw.fc1_b[i];
    vec[192 + i] = pw.fc2_b[i];
    vec[256 + i] = pw.ln2_g[i];
    vec[320 + i] = pw.ln2_b[i];
  }
  __syncthreads();
  // all weight fragments in registers for the whole token loop
  Afrag<T> fw[2][4], fkv[4][2], fo[4][4], f1[4][4], f2[4][4];
  load_afrags<T>(wS, lane, fw);
  load_afrags<T>(kvS, lane, fkv);
  load_afrags<T>(woS, lane, fo);
  load_afrags<T>(w1S, lane, f1);
  load_afrags<T>(w2S, lane, f2);
  const float inv_sqrt_m = 1.0f / sqrtf((float)PF_M);
  const int t_lo = blockIdx.x * span, t_hi = min(ntok, t_lo + span);
  const int g4 = 4 * (lane >> 4);  // this lane's feature offset inside a 16-feature tile
  for (int t0 = t_lo + 16 * wave; t0 < t_hi; t0 += 64) {
    const int t = t0 + (lane & 15);
    const bool valid = t < t_hi;
    const T* rowp = kqv + ((int64_t)b * ntok + t) * ldq;
    f32x4 qf[4], vf[4];
    load_frags(rowp + PF_HS, valid, lane, qf);
    load_frags(rowp + 2 * PF_HS, valid, lane, vf);
    float qd = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) qd += qf[c][0] * qf[c][0] + qf[c][1] * qf[c][1] + qf[c][2] * qf[c][2] + qf[c][3] * qf[c][3];
    qd = 0.5f * token_sum(qd);
    f32x4 qp[2];
    prm_tile<T>(fw, qf, qd, inv_sqrt_m, qp);
    float dn = 0.f;  // D_t = qp . ksum  (transformer_encoder.py:86)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) dn += qp[mt][j] * vec[16 * mt + g4 + j];
    const float rden = 1.0f / (token_sum(dn) + 1e-8f);
    f32x4 y[4];  // y^T = kptv . qp^T / (D + eps)   (:88-90)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int mc = 0; mc < 2; ++mc) chain16<T>(acc, fkv[nt][mc], qp[mc]);
      y[nt] = acc * rden;
    }
    f32x4 y2[4];  // y2 = v + attn_output(y)   (:93)
    float s1 = 0.f;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c) chain16<T>(acc, fo[nt][c], y[c]);
      const f32x4 bo = *(const EVT_LDS f32x4*)(vec + 64 + 16 * nt + g4);
      y2[nt] = acc + bo + vf[nt];
      s1 += y2[nt][0] + y2[nt][1] + y2[nt][2] + y2[nt][3];
    }
    const float mu = token_sum(s1) * (1.0f / 64.0f);
    float s2 = 0.f;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const f32x4 d = y2[nt] - mu;
      s2 += d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3];
    }
    const float rstd = rsqrtf(token_sum(s2) * (1.0f / 64.0f) + 1e-5f);
    f32x4 hn[4];  // LN2(y2)   (:99 norm2)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const f32x4 g = *(const EVT_LDS f32x4*)(vec + 256 + 16 * nt + g4);
      const f32x4 be = *(const EVT_LDS f32x4*)(vec + 320 + 16 * nt + g4);
      hn[nt] = (y2[nt] - mu) * rstd * g + be;
    }
    f32x4 h1[4];  // gelu(Dense(64))   (ffn.py:8)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c) chain16<T>(acc, f1[nt][c], hn[c]);
      acc += *(const EVT_LDS f32x4*)(vec + 128 + 16 * nt + g4);
#pragma unroll
      for (int j = 0; j < 4; ++j) h1[nt][j] = gelu_tanh(acc[j]);
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {  // out = y2 + Dense(64)(h1)   (ffn.py:9, :99)
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c) chain16<T>(acc, f2[nt][c], h1[c]);
      acc += *(const EVT_LDS f32x4*)(vec + 192 + 16 * nt + g4) + y2[nt];
      if (valid) store4(out + ((int64_t)b * ntok + t) * ldo + 16 * nt + g4, acc);
    }
  }
}

// bf16 out pass with fewer registers and more waves: the weight fragments are read from LDS per
// use (bf16 rows, 16-B chunks swizzled by row & 7; 34 KB per workgroup instead of 74 KB of fp32,
// and ~128 fewer VGPRs than the register-resident fragments of performer_out_kernel), so three
// workgroups share a CU, and the next tile's q / v rows are loaded while the current one runs.
// Same arithmetic (bf16 operands, fp32 accumulation, same k order) as performer_out_kernel<bf16>.
constexpr int PO_W = 0;                        // bf16 element offsets in the weight area:
constexpr int PO_KV = PO_W + PF_M * 64;        // prm w [32][64], kptv [64][32],
constexpr int PO_O = PO_KV + 64 * PF_M;        // out_w, fc1_w, fc2_w [64 out][64 in]
constexpr int PO_1 = PO_O + 64 * 64;
constexpr int PO_2 = PO_1 + 64 * 64;
constexpr int PO_END = PO_2 + 64 * 64;
constexpr size_t PF_OUT16_LDS = PO_END * 2 + 6 * 64 * sizeof(float);

// element (r, c) of a bf16 matrix with `cols` columns (multiple of 8): row-major, 16-B chunk
// (c / 8) stored at chunk index (c / 8) ^ (r & 7) (cols / 8 >= 4: chunk ^ (r & 3) when cols == 32)
__device__ __forceinline__ int po_idx(int r, int c, int cols) {
  const int nch = cols >> 3, q = (c >> 3) ^ (r & (nch - 1) & 7);
  return r * cols + (q << 3) + (c & 7);
}
// A fragment (rows 16 rt + (l & 15), k columns 16 kc + 4 (l >> 4) .. + 3) as one 8-B LDS read
__device__ __forceinline__ Afrag<bf16> po_frag(const EVT_LDS bf16* M, int cols, int rt, int kc, int lane) {
  const int r = 16 * rt + (lane & 15), c = 16 * kc + 4 * (lane >> 4);
  Afrag<bf16> f;
  f.v = *(const EVT_LDS i16x4*)(M + po_idx(r, c, cols));
  return f;
}

template <bool PERM>
__global__ __launch_bounds__(256, 4) void performer_out16_kernel(const bf16* __restrict__ kqv,
                                                                int64_t ldq, int ntok, int span,
                                                                const float* __restrict__ part,
                                                                PerformerWeights pw,
                                                                bf16* __restrict__ out, int64_t ldo,
                                                                float* __restrict__ tstats) {
  extern __shared__ __attribute__((aligned(16))) char dsm16[];
  EVT_LDS bf16* Wl = (EVT_LDS bf16*)dsm16;
  EVT_LDS float* vec = (EVT_LDS float*)(dsm16 + PO_END * 2);  // ksum[64 (32 used)], bo, b1, b2, g2, be2
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.y;
  for (int i = tid; i < PF_M * PF_HS; i += 256)  // prm w [m][k]
    Wl[PO_W + po_idx(i >> 6, i & 63, 64)] = (bf16)pw.prmw[i];
  for (int i = tid; i < 64 * 64; i += 256) {
    const int kr = i >> 6, nc = i & 63;  // Keras [in = kr][out = nc] -> LDS [out][in]
    Wl[PO_O + po_idx(nc, kr, 64)] = (bf16)pw.out_w[i];
    Wl[PO_1 + po_idx(nc, kr, 64)] = (bf16)pw.fc1_w[i];
    Wl[PO_2 + po_idx(nc, kr, 64)] = (bf16)pw.fc2_w[i];
  }
  const float* pb = part + (int64_t)b * PF_PART;  // the image's summed kptv / ksum
  for (int i = tid; i < PF_PART; i += 256) {
    const float v = pb[i];
    if (i < PF_HS * PF_M) Wl[PO_KV + po_idx(i / PF_M, i % PF_M, PF_M)] = (bf16)v;
    else vec[i - PF_HS * PF_M] = v;
  }
  for (int i = tid; i < 64; i += 256) {
    vec[64 + i] = pw.out_b[i];
    vec[128 + i] = pw.fc1_b[i];
    vec[192 + i] = pw.fc2_b[i];
    vec[256 + i] = pw.ln2_g[i];
    vec[320 + i] = pw.ln2_b[i];
  }
  __syncthreads();
  const float inv_sqrt_m = 1.0f / sqrtf((float)PF_M);
  const int t_lo = blockIdx.x * span, t_hi = min(ntok, t_lo + span);
  const int g4 = 4 * (lane >> 4);
  // raw bf16 q / v of a tile: 4 + 4 pieces of 4 features (8 B each; PERM: two 16-B loads per
  // block, kqv_col)
  auto load_raw = [&](int t0, u32x2 (&r)[8]) {
    const int t = t0 + (lane & 15);
    const bool valid = t < t_hi;
    const bf16* rowp = kqv + ((int64_t)b * ntok + (valid ? t : t_lo)) * ldq;
    if constexpr (PERM) {
#pragma unroll
      for (int blk = 0; blk < 2; ++blk) {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const u32x4 v = *(const u32x4*)(rowp + (1 + blk) * PF_HS + 16 * (lane >> 4) + 8 * hh);
          r[4 * blk + 2 * hh] = u32x2{v[0], v[1]};
          r[4 * blk + 2 * hh + 1] = u32x2{v[2], v[3]};
        }
      }
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        r[c] = *(const u32x2*)(rowp + PF_HS + 16 * c + g4);
        r[4 + c] = *(const u32x2*)(rowp + 2 * PF_HS + 16 * c + g4);
      }
    }
  };
  auto f4 = [](u32x2 v) {
    const bf16x4 h = __builtin_bit_cast(bf16x4, v);
    return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
  };
  u32x2 raw[8];
  int t0 = t_lo + 16 * wave;
  if (t0 < t_hi) load_raw(t0, raw);
  for (; t0 < t_hi; t0 += 64) {
    const int t = t0 + (lane & 15);
    const bool valid = t < t_hi;
    // the weight fragments are re-read from LDS every tile, not hoisted into registers
    const EVT_LDS bf16* Wt = Wl;
    asm volatile("" : "+v"(Wt));
    f32x4 qf[4], vf[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      qf[c] = valid ? f4(raw[c]) : f32x4{0.f, 0.f, 0.f, 0.f};
      vf[c] = valid ? f4(raw[4 + c]) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (t0 + 64 < t_hi) load_raw(t0 + 64, raw);  // next tile in flight under this one
    float qd = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) qd += qf[c][0] * qf[c][0] + qf[c][1] * qf[c][1] + qf[c][2] * qf[c][2] + qf[c][3] * qf[c][3];
    qd = 0.5f * token_sum(qd);
    f32x4 qp[2];  // prm_exp(q)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c) chain16<bf16>(acc, po_frag(Wt + PO_W, 64, mt, c, lane), qf[c]);
#pragma unroll
      for (int j = 0; j < 4; ++j) qp[mt][j] = __expf(acc[j] - qd) * inv_sqrt_m;
    }
    float dn = 0.f;  // D_t = qp . ksum  (transformer_encoder.py:86)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) dn += qp[mt][j] * vec[16 * mt + g4 + j];
    const float rden = 1.0f / (token_sum(dn) + 1e-8f);
    f32x4 y[4];  // y^T = kptv . qp^T / (D + eps)   (:88-90)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int mc = 0; mc < 2; ++mc) chain16<bf16>(acc, po_frag(Wt + PO_KV, PF_M, nt, mc, lane), qp[mc]);
      y[nt] = acc * rden;
    }
    f32x4 y2[4];  // y2 = v + attn_output(y)   (:93)
    float s1 = 0.f;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c) chain16<bf16>(acc, po_frag(Wt + PO_O, 64, nt, c, lane), y[c]);
      const f32x4 bo = *(const EVT_LDS f32x4*)(vec + 64 + 16 * nt + g4);
      y2[nt] = acc + bo + vf[nt];
      s1 += y2[nt][0] + y2[nt][1] + y2[nt][2] + y2[nt][3];
    }
    const float mu = token_sum(s1) * (1.0f / 64.0f);
    float s2 = 0.f;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const f32x4 d = y2[nt] - mu;
      s2 += d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3];
    }
    const float rstd = rsqrtf(token_sum(s2) * (1.0f / 64.0f) + 1e-5f);
    f32x4 hn[4];  // LN2(y2)   (:99 norm2)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const f32x4 g = *(const EVT_LDS f32x4*)(vec + 256 + 16 * nt + g4);
      const f32x4 be = *(const EVT_LDS f32x4*)(vec + 320 + 16 * nt + g4);
      hn[nt] = (y2[nt] - mu) * rstd * g + be;
    }
    f32x4 h1[4];  // gelu(Dense(64))   (ffn.py:8)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c) chain16<bf16>(acc, po_frag(Wt + PO_1, 64, nt, c, lane), hn[c]);
      acc += *(const EVT_LDS f32x4*)(vec + 128 + 16 * nt + g4);
#pragma unroll
      for (int j = 0; j < 4; ++j) h1[nt][j] = gelu_tanh(acc[j]);
    }
    float o1 = 0.f, o2 = 0.f;  // (sum, sumsq) of the token's stored output (tstats)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {  // out = y2 + Dense(64)(h1)   (ffn.py:9, :99)
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c) chain16<bf16>(acc, po_frag(Wt + PO_2, 64, nt, c, lane), h1[c]);
      acc += *(const EVT_LDS f32x4*)(vec + 192 + 16 * nt + g4) + y2[nt];
      const bf16x4 ob = {(bf16)acc[0], (bf16)acc[1], (bf16)acc[2], (bf16)acc[3]};
      if (valid) *(bf16x4*)(out + ((int64_t)b * ntok + t) * ldo + 16 * nt + g4) = ob;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float f = (float)ob[j];
        o1 += f;
        o2 += f * f;
      }
    }
    if (tstats) {  // per-token statistics for the next soft split's gathered rows
      o1 = token_sum(o1);
      o2 = token_sum(o2);
      if (valid && lane < 16) *(f32x2*)(tstats + 2 * ((int64_t)b * ntok + t)) = f32x2{o1, o2};
    }
  }
}

template <typename T>
__global__ __launch_bounds__(64) void cls_rows_kernel(T* __restrict__ x, int ntok, int D,
                                                      const float* __restrict__ cls,
                                                      const float* __restrict__ pos,
                                                      float* __restrict__ stats, int nslots) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int64_t row = (int64_t)b * ntok;
  float s1 = 0.f, s2 = 0.f;
  for (int n = lane; n < D; n += 64) {
    const T v = from_f32<T>(cls[n] + pos[n]);
    x[row * D + n] = v;
    const float q = to_f32(v);
    s1 += q;
    s2 += q * q;
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (stats && lane < nslots) {
    float* st = stats + 2 * (row * nslots + lane);
    st[0] = lane == 0 ? s1 : 0.f;
    st[1] = lane == 0 ? s2 : 0.f;
  }
}


// soft_split0 of the fp32 image (k 7, s 4, p 2, C 3: every T2T-ViT, t2t_vit.py:50): one block per
// (output row oh, image). The 7 input rows the band needs are staged once in LDS with coalesced
// 16-B loads ([7][W + 2p + pad][3] fp32, zero outside the image: the padding), then every output
// row (one pixel's 147-vector, zero padded to ldo) leaves as 16-B chunks of 8 elements, 32 lanes
// per row (ldo / 8 <= 32 chunks); row statistics by shuffles within the 32 lanes. The generic
// kernel above gathers 4-B elements from 7 image rows per row (1.6 TB/s measured).
template <typename TO>
__global__ __launch_bounds__(256) void unfold_k7s4c3_kernel(const float* __restrict__ in, int H,
                                                            int W, int OW, TO* __restrict__ out,
                                                            int ldo, float* __restrict__ stats,
                                                            int nslots) {
  extern __shared__ __attribute__((aligned(16))) float band[];  // [7][Wp][3]
  const int oh = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int Wp = W + 8;  // staged columns: iw = -2 .. W + 5 (zero outside [0, W))
  const int ih0 = oh * 4 - 2;
  for (int e = tid; e < 7 * Wp; e += 256) {
    const int kh = e / Wp, cw = e - kh * Wp, ih = ih0 + kh, iw = cw - 2;
    float v0 = 0.f, v1 = 0.f, v2 = 0.f;
    if (ih >= 0 && ih < H && iw >= 0 && iw < W) {
      const float* src = in + (((int64_t)b * H + ih) * W + iw) * 3;
      v0 = src[0];
      v1 = src[1];
      v2 = src[2];
    }
    float* d = band + (kh * Wp + cw) * 3;
    d[0] = v0;
    d[1] = v1;
    d[2] = v2;
  }
  __syncthreads();
  const int lane = tid & 63, half = lane >> 5, sub = lane & 31, wave = tid >> 6;
  const int nch = ldo / 8;
  // this lane's 8 (kh, kw, c) offsets inside a window (relative to the window origin), -1 = pad
  int off[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int e = sub * 8 + u;
    const int kh = e / 21, r = e - kh * 21, kw = r / 3, c = r - kw * 3;
    off[u] = (sub < nch && e < 147) ? (kh * Wp + kw) * 3 + c : -1;
  }
  for (int ow = wave * 2 + half; ow < OW; ow += 8) {
    const float* win = band + ow * 4 * 3;  // staged column of iw = ow * 4 - 2 is ow * 4
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = off[u] >= 0 ? win[off[u]] : 0.f;
    const int64_t row = ((int64_t)b * (gridDim.x) + oh) * OW + ow;
    float s1 = 0.f, s2 = 0.f;
    if (sub < nch) {
      TO* op = out + row * ldo + sub * 8;
      if constexpr (sizeof(TO) == 2) {
        const bf16x8 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3],
                          (bf16)v[4], (bf16)v[5], (bf16)v[6], (bf16)v[7]};
        store_b128(op, __builtin_bit_cast(u32x4, o));
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float q = (float)o[u];
          s1 += q;
          s2 += q * q;
        }
      } else {
        store4(op, f32x4{v[0], v[1], v[2], v[3]});
        store4(op + 4, f32x4{v[4], v[5], v[6], v[7]});
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          s1 += v[u];
          s2 += v[u] * v[u];
        }
      }
    }
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      s1 += __shfl_xor(s1, o, 64);
      s2 += __shfl_xor(s2, o, 64);
    }
    if (stats && sub < nslots) {
      float* st = stats + 2 * (row * nslots + sub);
      st[0] = sub == 0 ? s1 : 0.f;
      st[1] = sub == 0 ? s2 : 0.f;
    }
  }
}

template <typename TI, typename TO>
hipError_t unfold_t(const void* in, int B, int H, int W, int C, int k, int s, int p, void* out,
                    int ldo, float* stats, int nslots, hipStream_t st) {
  const int OH = (H + 2 * p - k) / s + 1, OW = (W + 2 * p - k) / s + 1;
  const int64_t rows = (int64_t)B * OH * OW;
  if (rows >= (int64_t)1 << 31) return hipErrorInvalidValue;
  if constexpr (std::is_same<TI, float>::value) {
    if (k == 7 && s == 4 && p == 2 && C == 3 && ldo % 8 == 0 && ldo <= 256 && nslots <= 32 &&
        (OH - 1) * 4 - 2 + 7 <= H + 6) {
      const size_t lds = (size_t)7 * (W + 8) * 3 * sizeof(float);
      if (lds <= 64 * 1024) {
        hipLaunchKernelGGL(unfold_k7s4c3_kernel<TO>, dim3(OH, B), dim3(256), lds, st, (const float*)in,
                           H, W, OW, (TO*)out, ldo, stats, nslots);
        return hipGetLastError();
      }
    }
  }
  const int vw = (C % 4 == 0 && ldo % 4 == 0) ? 4 : (ldo % 2 == 0 ? 2 : 1);
  if (ldo > 256 * vw) return hipErrorInvalidValue;  // <= 4 accesses per lane
  const int rpw = 4;
  const dim3 grid((unsigned)((rows + 4 * rpw - 1) / (4 * rpw)));
#define EVT_UNFOLD(V)                                                                          \
  hipLaunchKernelGGL((unfold_kernel<TI, TO, V>), grid, dim3(256), 0, st, (const TI*)in, B, H, W, \
                     C, k, s, p, OH, OW, (TO*)out, ldo, stats, nslots, rpw)
  if (vw == 4) EVT_UNFOLD(4);
  else if (vw == 2) EVT_UNFOLD(2);
  else EVT_UNFOLD(1);
#undef EVT_UNFOLD
  return hipGetLastError();
}

constexpr size_t PF_OUT_LDS = (size_t)(PF_M * 64 + 4 * 64 * 64 + 6 * 64) * sizeof(float);

// fixed-order sum of an image's chunk partials: part[b][c][i] -> fin[b][i] (c ascending)
__global__ __launch_bounds__(256) void performer_reduce_kernel(const float* __restrict__ part,
                                                               int nchunk, float* __restrict__ fin) {
  const int b = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
  if (i >= PF_PART) return;
  const float* pb = part + (int64_t)b * nchunk * PF_PART + i;
  float v = 0.f;
  for (int c = 0; c < nchunk; ++c) v += pb[(int64_t)c * PF_PART];
  fin[(int64_t)b * PF_PART + i] = v;
}

template <typename T, bool PERM = false>
hipError_t performer_t(const void* kqv, int64_t ldq, int B, int ntok, int chunk, int nchunk,
                       float* part, const PerformerWeights& w, int span, void* out, int64_t ldo,
                       hipStream_t s, float* tstats) {
  hipLaunchKernelGGL((performer_kv_kernel<T, PERM>), dim3(nchunk, B), dim3(256), 0, s,
                     (const T*)kqv, ldq, ntok, chunk, w.prmw, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // the chunk partials summed once per image (the output workgroups then read one partial each)
  float* fin = part + (size_t)B * nchunk * PF_PART;
  hipLaunchKernelGGL(performer_reduce_kernel, dim3((PF_PART + 255) / 256, B), dim3(256), 0, s,
                     part, nchunk, fin);
  if constexpr (std::is_same<T, bf16>::value) {
    hipLaunchKernelGGL(performer_out16_kernel<PERM>, dim3((ntok + span - 1) / span, B), dim3(256),
                       PF_OUT16_LDS, s, (const bf16*)kqv, ldq, ntok, span, fin, w, (bf16*)out, ldo,
                       tstats);
    return hipGetLastError();
  }
  (void)hipFuncSetAttribute((const void*)performer_out_kernel<T>,
                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)PF_OUT_LDS);
  hipLaunchKernelGGL(performer_out_kernel<T>, dim3((ntok + span - 1) / span, B), dim3(256),
                     PF_OUT_LDS, s, (const T*)kqv, ldq, ntok, span, fin, 1, w, (T*)out, ldo);
  return hipGetLastError();
}

}  // namespace

hipError_t unfold_launch(int dtype, int in_f32, const void* in, int B, int H, int W, int C, int k,
                         int s, int p, void* out, int ldo, float* stats, int nslots,
                         hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (k <= 0 || s <= 0 || p < 0 || H + 2 * p < k || W + 2 * p < k || ldo < k * k * C)
    return hipErrorInvalidValue;
  if (dtype == DT_BF16)
    return in_f32 ? unfold_t<float, bf16>(in, B, H, W, C, k, s, p, out, ldo, stats, nslots, st)
                  : unfold_t<bf16, bf16>(in, B, H, W, C, k, s, p, out, ldo, stats, nslots, st);
  return unfold_t<float, float>(in, B, H, W, C, k, s, p, out, ldo, stats, nslots, st);
}

// token chunks of the kv pass: >= 4 workgroups per image even at 28 x 28 tokens (stage 2)
static int performer_chunks(int ntok) { return (ntok + 195) / 196; }

size_t performer_part_floats(int B, int ntok) {
  return (size_t)B * (performer_chunks(ntok) + 1) * PF_PART;  // chunk partials + per-image sums
}

hipError_t performer_launch(int dtype, const void* kqv, int64_t ldq, int B, int ntok,
                            const PerformerWeights& w, float* part, void* out, int64_t ldo,
                            hipStream_t s, float* tstats, bool kqv_perm) {
  if (B <= 0 || ntok <= 0) return hipSuccess;
  if (ldq < 3 * PF_HS || ldo < PF_HS || (ldq & 3) || (ldo & 3)) return hipErrorInvalidValue;
  if ((tstats || kqv_perm) && dtype != DT_BF16) return hipErrorInvalidValue;
  if (kqv_perm && (ldq & 7)) return hipErrorInvalidValue;  // 16-B row pieces
  const int nchunk = performer_chunks(ntok);
  const int chunk = (ntok + nchunk - 1) / nchunk;
  // tokens per output workgroup: the images' token ranges cut into about one round of
  // workgroups at 4 per CU (T2T-ViT-14 bs256: 3136 tokens -> 4 x 784, 784 -> 4 x 208: 1024
  // workgroups each; a fixed 512 gave 1792 = 1.75 rounds and 512 = half a round). A token's
  // arithmetic does not depend on its workgroup (bitwise the same for every span).
  const int per_img = max(1, (4 * device_cus() + B - 1) / B);
  const int span = max(64, ((ntok + per_img - 1) / per_img + 15) & ~15);
  if (dtype != DT_BF16)
    return performer_t<float>(kqv, ldq, B, ntok, chunk, nchunk, part, w, span, out, ldo, s, nullptr);
  return kqv_perm
             ? performer_t<bf16, true>(kqv, ldq, B, ntok, chunk, nchunk, part, w, span, out, ldo, s,
                                       tstats)
             : performer_t<bf16>(kqv, ldq, B, ntok, chunk, nchunk, part, w, span, out, ldo, s, tstats);
}

// the model's kqv weight / bias with the output columns in kqv_col order within each 64 block
__global__ void kqv_permute_kernel(const float* __restrict__ W, const float* __restrict__ bias,
                                   int K, float* __restrict__ Wp, float* __restrict__ bp) {
  const int e = blockIdx.x * 256 + threadIdx.x;  // over (K + 1) x 192
  if (e >= (K + 1) * 3 * PF_HS) return;
  const int k = e / (3 * PF_HS), n = e - k * 3 * PF_HS, blk = n / PF_HS, f = n - blk * PF_HS;
  const int dst = blk * PF_HS + kqv_col(f);
  if (k < K) Wp[(int64_t)k * 3 * PF_HS + dst] = W[(int64_t)k * 3 * PF_HS + n];
  else bp[dst] = bias[n];
}
hipError_t kqv_permute_launch(const float* W, const float* bias, int K, float* Wp, float* bp,
                              hipStream_t s) {
  const int n = (K + 1) * 3 * PF_HS;
  hipLaunchKernelGGL(kqv_permute_kernel, dim3((n + 255) / 256), dim3(256), 0, s, W, bias, K, Wp, bp);
  return hipGetLastError();
}

// Statistics of the soft split (k 3, s 2, p 1) rows from per-token statistics: row (b, y, x) of
// the OW x OW grid sums the (sum, sumsq) of its <= 9 source tokens (the zero padding adds
// nothing); slot 0, the other slots zero.
__global__ __launch_bounds__(256) void unfold_stats_kernel(const float* __restrict__ ts, int B,
                                                           int R, int OW, float* __restrict__ dst,
                                                           int nd) {
  const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (m >= (int64_t)B * OW * OW) return;
  const int b = (int)(m / (OW * OW)), r = (int)(m - (int64_t)b * OW * OW), y = r / OW, x = r - y * OW;
  float s1 = 0.f, s2 = 0.f;
  for (int kh = 0; kh < 3; ++kh) {
    const int iy = 2 * y - 1 + kh;
    if (iy < 0 || iy >= R) continue;
    for (int kw = 0; kw < 3; ++kw) {
      const int ix = 2 * x - 1 + kw;
      if (ix < 0 || ix >= R) continue;
      const f32x2 v = *(const f32x2*)(ts + 2 * (((int64_t)b * R + iy) * R + ix));
      s1 += v[0];
      s2 += v[1];
    }
  }
  float* d = dst + m * nd * 2;
  *(f32x2*)d = f32x2{s1, s2};
  for (int j = 1; j < nd; ++j) *(f32x2*)(d + 2 * j) = f32x2{0.f, 0.f};
}

hipError_t unfold_stats_launch(const float* tstats, int B, int R, float* dst, int nslots,
                               hipStream_t s) {
  if (B <= 0) return hipSuccess;
  const int OW = (R + 1) / 2;
  const int64_t rows = (int64_t)B * OW * OW;
  hipLaunchKernelGGL(unfold_stats_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s,
                     tstats, B, R, OW, dst, nslots);
  return hipGetLastError();
}

hipError_t cls_rows_launch(int dtype, void* x, int B, int ntok, int D, const float* cls,
                           const float* pos, float* stats, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  const int ns = stats_slots(D);
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(cls_rows_kernel<bf16>, dim3(B), dim3(64), 0, s, (bf16*)x, ntok, D, cls, pos,
                       stats, ns);
  else
    hipLaunchKernelGGL(cls_rows_kernel<float>, dim3(B), dim3(64), 0, s, (float*)x, ntok, D, cls,
                       pos, stats, ns);
  return hipGetLastError();
}

}  // namespace evt
