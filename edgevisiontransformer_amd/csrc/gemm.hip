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
constexpr int BIG_BN_ = 256;

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


template <int FL>
__device__ __forceinline__ f32x4 epi_bias(const GemmParams& p, int n, bool full) {
  // full: the 4 columns are in range and 16-B aligned (always true on interior tiles)
  f32x4 b4 = f32x4{0.f, 0.f, 0.f, 0.f};
  if (FL & EPI_BIAS) {
    if (full) b4 = load4(p.bias + n);
    else
      for (int j = 0; j < 4; ++j) b4[j] = (n + j < p.N) ? p.bias[n + j] : 0.f;
  }
  return b4;
}

// v = acc + bias for C[m][n..n+3]; applies gelu / pos (+row remap) / residual and stores.
template <typename T, int FL>
__device__ __forceinline__ void epi_store(const GemmParams& p, f32x4 v, int m, int n, bool full) {
  typedef typename std::conditional<(FL & EPI_OUT_F32) != 0, float, T>::type TO;
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

// Bijective XCD-aware remap: blocks b and b+8 share an XCD (round-robin dispatch), so give each
// XCD a contiguous range of logical tiles (tile order: all N tiles of one M block consecutively,
// so an XCD's L2 keeps the A panel while it sweeps N).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, local = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
}

template <typename T, int FL>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably uniform -> SGPR math
  const int wm = wave & 1, wn = wave >> 1;

  // ---- XCD-aware bijective block remap ----
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
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
    const f32x4 bias4 = epi_bias<FL>(p, n, full);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int m = m0 + wm * 64 + mt * 16 + frow;
      if (m < p.M) epi_store<T, FL>(p, acc[nt][mt] + bias4, m, n, full);
    }
  }
}


int g_gemm_variant = 0;  // 0 auto, 1 128x128, 2 256x256 plain, 3 staggered, 4 pipelined, 5 ring

bool use_big(const GemmParams& p) {
  if ((p.ntiles * GEMM_BN) % BIG_BN_) return false;
  if (g_gemm_variant == 1) return false;
  if (g_gemm_variant >= 2) return true;
  // enough 256x256 tiles to fill the chip at least once
  return (int64_t)((p.M + 255) / 256) * (p.ntiles * GEMM_BN / 256) >= 256;
}

// ---------------------------------------------------------------------------------------------
// Large-tile bf16 kernel: 256x256 output tile, BK = 64, 512 threads = 8 waves in 2 (m) x 4 (n),
// each wave a 128 (m) x 64 (n) sub-tile = 8 x 4 MFMA tiles (128 fp32 accumulators per lane).
// 128 KiB LDS (2 buffers x {A 32 KiB, W 32 KiB}), one block per CU. The next K-tile's 8
// global_load_lds per wave are issued at the top of the current tile so a whole tile of MFMAs
// (64 per wave) covers their latency; both k32 sub-steps' fragments are read up front so the
// second step's ds_reads overlap the first step's MFMAs.
// ---------------------------------------------------------------------------------------------
constexpr int BIG_BM = 256, BIG_BN = 256;
constexpr int BIG_TILE = BIG_BM * ROWB;       // 32 KiB per operand
constexpr int BIG_STAGE = 2 * BIG_TILE;       // 64 KiB per K-tile


// LDS-staged epilogue of the 256x256 kernels. The accumulator layout gives each lane 4
// consecutive columns of one row, i.e. 8-16 B per store spread over 16 rows per instruction
// (store-issue bound: ~32 narrow stores per lane per tile). Instead, after bias/GELU the tile is
// staged through the (now idle) 128 KiB LDS in two 128-column fp32 halves (XOR-swizzled
// 512-B rows: conflict-free 16-B writes and reads), and all 8 waves then stream whole rows:
// residual loads and output stores become fully coalesced 256-512 B row segments.
template <int FL>
__device__ __forceinline__ void big_epilogue(const GemmParams& p, f32x4 (&acc)[4][8], char* smem,
                                             int m0, int n0, int wm, int wn, int lane, int wave) {
  typedef typename std::conditional<(FL & EPI_OUT_F32) != 0, float, bf16>::type TO;
  const int frow = lane & 15, fg = lane >> 4;
  const bool interior = p.vec_ok && (n0 + 256 <= p.N) && (m0 + 256 <= p.M);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __builtin_amdgcn_s_barrier();  // previous readers of the staging area are done
    if ((wn >> 1) == h) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int n = n0 + wn * 64 + nt * 16 + fg * 4;
        const f32x4 bias4 = epi_bias<FL>(p, n, interior || (p.vec_ok && n + 4 <= p.N));
        const int chunk = (wn & 1) * 16 + nt * 4 + fg;
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) {
          const int row = wm * 128 + mt * 16 + frow;
          f32x4 v = acc[nt][mt] + bias4;
          if (FL & EPI_GELU) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = gelu_tanh(v[j]);
          }
          *(EVT_LDS f32x4*)((EVT_LDS char*)smem + row * 512 + ((chunk ^ (row & 7)) * 16)) = v;
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    const int sub = lane >> 5, c = lane & 31;
    const int n = n0 + h * 128 + c * 4;
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
      const int row = wave * 32 + i * 2 + sub;
      const int m = m0 + row;
      f32x4 v = *(const EVT_LDS f32x4*)((EVT_LDS char*)smem + row * 512 + ((c ^ (row & 7)) * 16));
      if (interior) {
        int64_t orow = m;
        if (FL & EPI_POS) {
          const int img = m / p.P, t = m - img * p.P;
          orow = (int64_t)img * (p.P + 1) + 1 + t;
          v += load4(p.pos + (int64_t)(t + 1) * p.ldp + n);
        }
        if (FL & EPI_RESID) v += load4((const bf16*)p.resid + (int64_t)m * p.ldr + n);
        store4((TO*)p.C + orow * p.ldc + n, v);
      } else if (m < p.M && n < p.N) {
        const bool full = p.vec_ok && (n + 4 <= p.N);
        // bias was already added; epi_store adds pos/resid and stores (gelu off here)
        epi_store<bf16, FL & ~EPI_GELU>(p, v, m, n, full);
      }
    }
  }
}

template <int FL, int VAR>  // VAR 0: plain, 1: staggered wave groups, 2: software-pipelined
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
  // Addresses are recomputed per stage (a few VALU ops) instead of held in 16 VGPRs: the
  // staggered variant needs every register for fragments + accumulators.
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
  auto read_frags = [&](int kt, u32x4 (&a)[2][8], u32x4 (&w)[2][4]) {
    const EVT_LDS char* As = (const EVT_LDS char*)smem + (kt & 1) * BIG_STAGE;
    const EVT_LDS char* Ws = As + BIG_TILE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int coff = ((fg + 4 * ks) ^ fsw) * 16;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        w[ks][nt] = *(const EVT_LDS u32x4*)(Ws + (wn * 64 + nt * 16 + frow) * ROWB + coff);
#pragma unroll
      for (int mt = 0; mt < 8; ++mt)
        a[ks][mt] = *(const EVT_LDS u32x4*)(As + (wm * 128 + mt * 16 + frow) * ROWB + coff);
    }
  };
  auto mfma_tile = [&](const u32x4 (&a)[2][8], const u32x4 (&w)[2][4]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) Mma<bf16>::run(w[ks][nt], a[ks][mt], acc[nt][mt]);
  };
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
  if constexpr (VAR == 2) {
    // Software pipeline, one barrier per K-tile. Fragments of (tile t, k-step 0) are read during
    // the previous tile's second k-step, so every MFMA phase starts with its operands in
    // registers; the DMA for tile t+2 is issued right after the barrier that retires all reads
    // of its buffer and has 1.5 K-tiles of MFMAs to land. LDS reads and DMA issues are
    // interleaved between MFMAs with sched_group_barrier (masks: 0x8 MFMA, 0x10 VMEM,
    // 0x100 DS read).
    //   A(t): read (t, ks1) frags | 32 MFMA (t, ks0)
    //   vmcnt(0) lgkmcnt(0) barrier          -> tile t+1 visible, buffer t&1 free
    //   B(t): DMA t+2 -> buffer t&1 ; read (t+1, ks0) frags | 32 MFMA (t, ks1) ; lgkmcnt(0)
    u32x4 a0[8], w0[4], a1[8], w1[4];
    auto phase_a = [&](int kt) {
      read_step(kt, 1, a1, w1);
      mfma_step(a0, w0);
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    };
    auto sync = [&]() {
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    auto phase_b = [&](int kt, bool dma, bool next) {
      if (dma) stage(kt + 2, kt & 1);
      if (next) read_step(kt + 1, 0, a0, w0);
      mfma_step(a1, w1);
      if (dma && next) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x010, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 16, 1);
      } else if (next) {
#pragma unroll
        for (int i = 0; i < 12; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 1);
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): (t+1, ks0) frags landed (long since)
      __builtin_amdgcn_sched_barrier(0);
    };
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (nk > 1) stage(1, 1);
    read_step(0, 0, a0, w0);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    int kt = 0;
    for (; kt + 2 < nk; ++kt) {
      phase_a(kt);
      sync();
      phase_b(kt, true, true);
    }
    if (kt + 1 < nk) {  // kt == nk - 2
      phase_a(kt);
      sync();
      phase_b(kt, false, true);
      ++kt;
    }
    // kt == nk - 1: last tile, no barrier needed (no further DMA)
    read_step(kt, 1, a1, w1);
    mfma_step(a0, w0);
    mfma_step(a1, w1);
  } else if constexpr (VAR == 0) {
    for (int kt = 0; kt < nk; ++kt) {
      wait_vmcnt0();
      __builtin_amdgcn_s_barrier();
      if (kt + 1 < nk) stage(kt + 1, (kt + 1) & 1);
      u32x4 a[2][8], w[2][4];
      read_frags(kt, a, w);
      __builtin_amdgcn_s_setprio(1);
      mfma_tile(a, w);
      __builtin_amdgcn_s_setprio(0);
    }
  } else if constexpr (VAR == 6) {
    // plain structure (one barrier per K-tile, DMA for tile t+1 issued at the top of tile t),
    // with an explicit issue order: k-step-0 reads, then the 8 DMA pieces spread between the
    // first 16 MFMAs, the k-step-1 reads between the next 12, then the remaining MFMAs.
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
      __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
      if (dma) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
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
  } else if constexpr (VAR >= 10) {
    // ABLATION builds (timing only, outputs meaningless): bit0 no DMA in loop, bit1 no LDS
    // reads in loop, bit2 no MFMA, bit3 no barrier
    constexpr int ABL = VAR - 10;
    u32x4 a[2][8], w[2][4];
    read_frags(0, a, w);
    for (int kt = 0; kt < nk; ++kt) {
      wait_vmcnt0();
      if constexpr (!(ABL & 8)) __builtin_amdgcn_s_barrier();
      if constexpr (!(ABL & 1)) { if (kt + 1 < nk) stage(kt + 1, (kt + 1) & 1); }
      if constexpr (!(ABL & 2)) read_frags(kt, a, w);
      if constexpr (!(ABL & 4)) mfma_tile(a, w);
      else {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < 8; ++i) asm volatile("" ::"v"(a[ks][i]));
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(w[ks][i]));
      }
    }
  } else {
    // Two wave groups (waves 0-3 / 4-7: one of each per SIMD) run half a K-tile apart: group 1
    // executes one extra barrier up front, so while one group's wave issues its LDS reads and
    // next-tile DMA, its SIMD partner from the other group runs its 64 MFMAs. Every wave drains
    // its own DMA (vmcnt) and LDS reads (lgkmcnt) before every barrier, so a K-tile is visible to
    // all waves one barrier after its last DMA was issued, and a buffer is only re-filled one
    // barrier after its last reader passed.
    const int grp = __builtin_amdgcn_readfirstlane(tid) >> 8;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (grp) __builtin_amdgcn_s_barrier();
    for (int kt = 0; kt < nk; ++kt) {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      u32x4 a[2][8], w[2][4];
      read_frags(kt, a, w);
      if (kt + 1 < nk) stage(kt + 1, (kt + 1) & 1);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      mfma_tile(a, w);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (!grp) __builtin_amdgcn_s_barrier();
  }

  big_epilogue<FL>(p, acc, smem, m0, n0, wm, wn, lane, wave);
}


// ---------------------------------------------------------------------------------------------
// Ring kernel (bf16): 256x256 output tile, 8 waves (2 m x 4 n, 128x64 per wave), K staged in
// 32-deep slices (64 B per row) through a 5-slot LDS ring (5 x 32 KiB = all 160 KiB), so four
// slices (up to 128 KiB) of global_load_lds are in flight while one is consumed: the LDS-DMA
// latency under full load (~1-2 us) is covered by 3 slices (3 x 32 MFMAs per wave) of work.
// Per slice: issue DMA for slice s+4, counted vmcnt for slice s+1, ONE barrier, then the
// fragments of slice s+1 are read between the 32 MFMAs of slice s (register double buffer).
// 64-B rows use the swizzle chunk ^ ((row >> 1) & 3): conflict-free ds_read_b128.
// ---------------------------------------------------------------------------------------------
constexpr int RING_SLOTS = 5;
constexpr int RING_ROWB = 64;
constexpr int RING_HALF = 256 * RING_ROWB;  // 16 KiB per operand per slice
constexpr int RING_SLOT = 2 * RING_HALF;    // 32 KiB

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
}

template <int FL>
__global__ __launch_bounds__(512, 2) void gemm_ring_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[RING_SLOTS * RING_SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably uniform -> SGPR math
  const int wm = wave & 1, wn = wave >> 1;
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = wgid / p.ntiles, tn = wgid - tm * p.ntiles;
  const int m0 = tm * BIG_BM, n0 = tn * BIG_BN;

  // staging: wave w owns rows [w*32, w*32+32) of both operands: 2 glds each (16 rows x 64 B)
  const int srow = lane >> 2, sslot = lane & 3;
  const int64_t lda_b = p.lda * 2, ldw_b = p.ldw * 2;
  const int schunk = (sslot ^ ((srow >> 1) & 3)) * 16;
  const int arow0 = m0 + wave * 32 + srow;
  const char* a_base = (const char*)p.A + schunk;
  const char* w_base = (const char*)p.W + (int64_t)(n0 + wave * 32 + srow) * ldw_b + schunk;
  auto stage = [&](int sl) {
    EVT_LDS char* base = (EVT_LDS char*)smem + (sl % RING_SLOTS) * RING_SLOT;
    const int64_t koff = (int64_t)sl * RING_ROWB;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int gm = min(arow0 + i * 16, p.M - 1);
      glds16(a_base + gm * lda_b + koff, base + (wave * 32 + i * 16) * RING_ROWB);
      glds16(w_base + (i * 16) * ldw_b + koff, base + RING_HALF + (wave * 32 + i * 16) * RING_ROWB);
    }
  };

  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15, fg = lane >> 4;
  const int coff = (fg ^ ((lane >> 1) & 3)) * 16;
  auto read_slice = [&](int sl, u32x4 (&a)[8], u32x4 (&w)[4]) {
    const EVT_LDS char* As = (const EVT_LDS char*)smem + (sl % RING_SLOTS) * RING_SLOT;
    const EVT_LDS char* Ws = As + RING_HALF;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
      w[nt] = *(const EVT_LDS u32x4*)(Ws + (wn * 64 + nt * 16 + frow) * RING_ROWB + coff);
#pragma unroll
    for (int mt = 0; mt < 8; ++mt)
      a[mt] = *(const EVT_LDS u32x4*)(As + (wm * 128 + mt * 16 + frow) * RING_ROWB + coff);
  };
  auto mfma_slice = [&](const u32x4 (&a)[8], const u32x4 (&w)[4]) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) Mma<bf16>::run(w[nt], a[mt], acc[nt][mt]);
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto wait_ahead = [&](int sl, int ns) {
    const int ahead = min(sl + 4, ns - 1) - (sl + 1);  // slices issued after s+1
    if (ahead >= 3) wait_vm<12>();
    else if (ahead == 2) wait_vm<8>();
    else if (ahead == 1) wait_vm<4>();
    else wait_vm<0>();
  };
  auto interleave = [&]() {
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_sched_barrier(0);
  };

  const int ns = p.K / 32;  // even (K % 64 == 0)
  const int pre = min(4, ns);
  for (int i = 0; i < pre; ++i) stage(i);
  if (pre == 4) wait_vm<12>();
  else wait_vm<0>();
  barrier();
  u32x4 a0[8], w0[4], a1[8], w1[4];
  read_slice(0, a0, w0);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  // Each slice: DMA s+4 | counted wait for s+1 | barrier | read s+1 between the MFMAs of s.
  // Unrolled by two so the fragment double buffer keeps static register names.
  int sl = 0;
  for (; sl + 2 < ns; sl += 2) {
    if (sl + 4 < ns) stage(sl + 4);
    wait_ahead(sl, ns);
    barrier();
    read_slice(sl + 1, a1, w1);
    mfma_slice(a0, w0);
    interleave();
    if (sl + 5 < ns) stage(sl + 5);
    wait_ahead(sl + 1, ns);
    barrier();
    read_slice(sl + 2, a0, w0);
    mfma_slice(a1, w1);
    interleave();
  }
  // last two slices (sl == ns - 2): nothing further to load
  wait_vm<0>();
  barrier();
  read_slice(sl + 1, a1, w1);
  mfma_slice(a0, w0);
  interleave();
  mfma_slice(a1, w1);

  big_epilogue<FL>(p, acc, smem, m0, n0, wm, wn, lane, wave);
}

template <int FL>
hipError_t launch_big(const GemmParams& p, hipStream_t s) {
  const int mtiles = (p.M + BIG_BM - 1) / BIG_BM;
  GemmParams q = p;
  q.ntiles = (p.ntiles * GEMM_BN) / BIG_BN;
  const dim3 grid(mtiles * q.ntiles);
  if (g_gemm_variant == 2)
    hipLaunchKernelGGL((gemm_big_kernel<FL, 0>), grid, dim3(512), 0, s, q);
  else if (g_gemm_variant == 3)
    hipLaunchKernelGGL((gemm_big_kernel<FL, 1>), grid, dim3(512), 0, s, q);
  else if (g_gemm_variant == 4)
    hipLaunchKernelGGL((gemm_big_kernel<FL, 2>), grid, dim3(512), 0, s, q);
  else if (g_gemm_variant == 5)
    hipLaunchKernelGGL((gemm_ring_kernel<FL>), grid, dim3(512), 0, s, q);
  else if (g_gemm_variant >= 10 && FL == 0) {
    switch (g_gemm_variant) {
      case 11: hipLaunchKernelGGL((gemm_big_kernel<FL, 11>), grid, dim3(512), 0, s, q); break;
      case 12: hipLaunchKernelGGL((gemm_big_kernel<FL, 12>), grid, dim3(512), 0, s, q); break;
      case 13: hipLaunchKernelGGL((gemm_big_kernel<FL, 13>), grid, dim3(512), 0, s, q); break;
      case 14: hipLaunchKernelGGL((gemm_big_kernel<FL, 14>), grid, dim3(512), 0, s, q); break;
      case 15: hipLaunchKernelGGL((gemm_big_kernel<FL, 15>), grid, dim3(512), 0, s, q); break;
      case 19: hipLaunchKernelGGL((gemm_big_kernel<FL, 19>), grid, dim3(512), 0, s, q); break;
      case 17: hipLaunchKernelGGL((gemm_big_kernel<FL, 17>), grid, dim3(512), 0, s, q); break;
      default: hipLaunchKernelGGL((gemm_big_kernel<FL, 10>), grid, dim3(512), 0, s, q); break;
    }
  }
  else  // default (0) and 6
    hipLaunchKernelGGL((gemm_big_kernel<FL, 6>), grid, dim3(512), 0, s, q);
  return hipGetLastError();
}

template <typename T, int FL>
hipError_t launch_t(const GemmParams& p, hipStream_t s) {
  if (std::is_same<T, bf16>::value && use_big(p)) return launch_big<FL>(p, s);
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

void gemm_set_variant(int v) { g_gemm_variant = v; }

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
