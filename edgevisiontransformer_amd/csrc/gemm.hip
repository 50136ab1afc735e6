// Token-matrix GEMM for the ViT encoder on gfx950 (MI355X, CDNA4).
//
// Replaces every tf.keras.layers.Dense on the hot path (reference `modeling/layers/attention.py:17-18`
// to_qkv / to_out, `modeling/layers/ffn.py:8-9` FC1+gelu / FC2, `modeling/models/vit.py:23,38-39`
// patch_to_embedding / mlp_head) as one templated MFMA kernel with fused epilogues.
//
// Layout. A (activations) is row-major [M][lda]; weights are packed once at model creation to
// Wp[Npad][Kpad] (K-contiguous, zero padded), so both MFMA operands are 16-byte K-contiguous
// reads. Per stage the block stages 128 bytes of K for a 128-row A tile and a 128-row W tile
// into LDS with global_load_lds (async, 16 B/lane), double buffered. The LDS image is
// row-linear; the bank-conflict swizzle (chunk ^ (row & 7)) is applied to the per-lane SOURCE
// address and to the ds_read address (glds writes lane-linear).
//
// MFMA. The product is computed transposed, C^T = W . A^T, so that each lane ends up owning 4
// consecutive output COLUMNS of one row (16x16 C layout: col = lane&15 -> token row m,
// row = 4*(lane>>4)+j -> feature n): epilogue loads/stores are 8-16 B per lane.
//   bf16: v_mfma_f32_16x16x32_bf16, one 16-B chunk (8 k) per MFMA.
//   f32 : v_mfma_f32_16x16x4_f32 (exact fp32, the parity path), one 16-B chunk = 4 MFMAs with a
//         k-permutation shared by both operands.
// 256 threads = 4 waves in 2(m) x 2(n); each wave owns a 64x64 output tile (4x4 MFMA tiles).
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

template <typename T, int FL>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(GemmParams p) {
  typedef typename std::conditional<(FL & EPI_OUT_F32) != 0, float, T>::type TO;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;

  // ---- XCD-aware bijective block remap ----
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, local = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
  const int tm = wgid / p.ntiles, tn = wgid - tm * p.ntiles;
  const int m0 = tm * GEMM_BM, n0 = tn * GEMM_BN;

  // ---- staging addresses: wave stages rows [wave*32, wave*32+32) of both tiles ----
  const int srow = lane >> 3, sslot = lane & 7;
  const int64_t lda_b = p.lda * (int64_t)sizeof(T), ldw_b = p.ldw * (int64_t)sizeof(T);
  const char* a_src[4];
  const char* w_src[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wave * 32 + i * 8 + srow;
    const int gm = min(m0 + row, p.M - 1);
    const int chunk = sslot ^ srow;  // (row & 7) == srow
    a_src[i] = (const char*)p.A + gm * lda_b + chunk * 16;
    w_src[i] = (const char*)p.W + (int64_t)(n0 + row) * ldw_b + chunk * 16;
  }
  auto stage = [&](int kt, int buf) {
    EVT_LDS char* base = (EVT_LDS char*)smem + buf * STAGE_BYTES;
    const int64_t koff = (int64_t)kt * ROWB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      glds16(a_src[i] + koff, base + (wave * 32 + i * 8) * ROWB);
      glds16(w_src[i] + koff, base + TILE_BYTES + (wave * 32 + i * 8) * ROWB);
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

  // ---- epilogue: lane owns C[m][n..n+3] ----
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int n = n0 + wn * 64 + nt * 16 + fg * 4;
    if (n >= p.N) continue;
    const bool full = p.vec_ok && (n + 4 <= p.N);
    f32x4 bias4 = f32x4{0.f, 0.f, 0.f, 0.f};
    if (FL & EPI_BIAS) {
      if (full) bias4 = load4(p.bias + n);
      else
        for (int j = 0; j < 4; ++j) bias4[j] = (n + j < p.N) ? p.bias[n + j] : 0.f;
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int m = m0 + wm * 64 + mt * 16 + frow;
      if (m >= p.M) continue;
      f32x4 v = acc[nt][mt] + bias4;
      if (FL & EPI_GELU) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = gelu_tanh(v[j]);
      }
      int64_t orow = m;
      if (FL & EPI_POS) {
        const int img = m / p.P, t = m - img * p.P;
        orow = (int64_t)img * (p.P + 1) + 1 + t;
        const float* pp = p.pos + (int64_t)(t + 1) * p.ldp + n;
        if (full) v += load4(pp);
        else
          for (int j = 0; j < 4; ++j) v[j] += (n + j < p.N) ? pp[j] : 0.f;
      }
      if (FL & EPI_RESID) {
        const T* rp = (const T*)p.resid + (int64_t)m * p.ldr + n;
        if (full) v += load4(rp);
        else
          for (int j = 0; j < 4; ++j) v[j] += (n + j < p.N) ? to_f32(rp[j]) : 0.f;
      }
      TO* cp = (TO*)p.C + orow * p.ldc + n;
      if (full) store4(cp, v);
      else
        for (int j = 0; j < 4; ++j)
          if (n + j < p.N) cp[j] = from_f32<TO>(v[j]);
    }
  }
}

template <typename T, int FL>
hipError_t launch_t(const GemmParams& p, hipStream_t s) {
  const int mtiles = (p.M + GEMM_BM - 1) / GEMM_BM;
  hipLaunchKernelGGL((gemm_nt_kernel<T, FL>), dim3(mtiles * p.ntiles), dim3(256), 0, s, p);
  return hipGetLastError();
}

template <typename T>
hipError_t dispatch(int flags, const GemmParams& p, hipStream_t s) {
  switch (flags) {
    case 0: return launch_t<T, 0>(p, s);                                        // QKV
    case EPI_BIAS | EPI_GELU: return launch_t<T, EPI_BIAS | EPI_GELU>(p, s);    // FC1, head1
    case EPI_BIAS | EPI_RESID | EPI_OUT_F32:                                    // out-proj, FC2
      return launch_t<T, EPI_BIAS | EPI_RESID | EPI_OUT_F32>(p, s);
    case EPI_BIAS | EPI_OUT_F32: return launch_t<T, EPI_BIAS | EPI_OUT_F32>(p, s);  // head2
    case EPI_BIAS | EPI_POS | EPI_OUT_F32:                                      // patch embed
      return launch_t<T, EPI_BIAS | EPI_POS | EPI_OUT_F32>(p, s);
    case EPI_BIAS: return launch_t<T, EPI_BIAS>(p, s);
    default: return hipErrorInvalidValue;
  }
}

// Wp[n][k] = W[k][n] (fp32 [K][N] in) converted to T, zero outside [N) x [K).
template <typename T>
__global__ void pack_kernel(const float* __restrict__ W, int K, int N, T* __restrict__ Wp, int Kpad,
                            int Npad) {
  __shared__ float tile[32][33];
  const int k0 = blockIdx.x * 32, n0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 8 rows per pass
  for (int r = ty; r < 32; r += 8) {
    const int k = k0 + r, n = n0 + tx;
    tile[r][tx] = (k < K && n < N) ? W[(int64_t)k * N + n] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int n = n0 + r, k = k0 + tx;
    if (n < Npad && k < Kpad) Wp[(int64_t)n * Kpad + k] = from_f32<T>(tile[tx][r]);
  }
}

}  // namespace

hipError_t gemm_launch(int dtype, int flags, const GemmParams& p, hipStream_t s) {
  if (p.M <= 0 || p.N <= 0) return hipSuccess;
  if (p.K % PAD_K != 0 || p.K <= 0) return hipErrorInvalidValue;
  if (p.ntiles * GEMM_BN < p.N) return hipErrorInvalidValue;
  return dtype == DT_BF16 ? dispatch<bf16>(flags, p, s) : dispatch<float>(flags, p, s);
}

hipError_t pack_weight(int dtype, const float* W, int K, int N, void* Wp, int Kpad, int Npad,
                       hipStream_t s) {
  dim3 grid((Kpad + 31) / 32, (Npad + 31) / 32);
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(pack_kernel<bf16>, grid, dim3(256), 0, s, W, K, N, (bf16*)Wp, Kpad, Npad);
  else
    hipLaunchKernelGGL(pack_kernel<float>, grid, dim3(256), 0, s, W, K, N, (float*)Wp, Kpad, Npad);
  return hipGetLastError();
}

}  // namespace evt
