// Host-side kernel launch interface shared by the .hip translation units and capi.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace evt {

enum Dtype : int { DT_F32 = 0, DT_BF16 = 1 };

// Epilogue flags of the token-matrix GEMM (see gemm.hip header for the LayerNorm folding).
enum : int {
  EPI_BIAS = 1,      // + bias[n]
  EPI_GELU = 2,      // tanh-GELU
  EPI_RESID = 4,     // + resid[m][n]
  EPI_POS = 8,       // patch embed: output row remap b*P+t -> b*(P+1)+1+t, + pos[t+1][n]
  EPI_OUT_F32 = 16,  // fp32 output (else activation dtype)
  EPI_LNIN = 32,     // A rows are un-normalised: v = r*acc - r*mu*colsum[n] (+ bias = c[n])
  EPI_RESLN = 64,    // residual is LN(resid): (resid - mu_r) * r_r * rgamma[n] + rbeta[n]
  EPI_STATS = 128,   // accumulate (sum, sum of squares) of each output row into stats_out
  EPI_GELU_ERF = 256,  // exact erf GELU (nn.GELU, the Swin MLP)
  EPI_OUT_MX8 = 512,   // MXFP8 output (mx8.hip GEMM only)
  EPI_GATHER = 1024,   // A rows gathered by the GEMM's loader: Swin PatchMerging (GemmParams g*)
  EPI_SPLIT = 2048,    // A rows gathered by the GEMM's loader: T2T soft split k3 s2 p1 (g*)
  EPI_HM = 4096,       // head-major QKV output [B][H][q | k | v][P][64] (P = tokens per image,
                       // N = 3 H 64): q, k, v of every (image, head) contiguous runs for the
                       // attention kernel (AttnParams sb / sh / ko / vo). Persistent kernel only
};

// C[M, N] = epilogue(A[M, K] . W[K, N]) with W pre-packed K-contiguous as Wp[Npad][Kpad].
// A, resid: activation dtype; C: fp32 when EPI_OUT_F32 else activation dtype.
struct GemmParams {
  const void* A;     int64_t lda;    // elements
  const void* W;     int64_t ldw;    // packed weights, ldw = Kpad (elements)
  void* C;           int64_t ldc;
  int M, N, K;                        // N = columns stored; K = Kpad (multiple of 64 elements)
  int ntiles;                         // Npad / GEMM_BN
  const float* bias;                  // >= N floats (zero padded) or null
  const void* resid; int64_t ldr;     // residual (activation dtype) or null
  const float* pos;  int64_t ldp;     // EPI_POS: pos[(t+1)*ldp + n], output row remap
  int P;                              // EPI_POS: patches per image
  int vec_ok;                         // 1: leading dims multiple of 4 (vector epilogue);
                                      // 2: multiple of 8 (16-B bf16 stores)
  const float* colsum;                // EPI_LNIN: column sums of the packed (gamma-folded) W
  const float* stats_in;              // EPI_LNIN: [M][nslots][2] (sum, sumsq) of the A rows
  const float* rstats;                // EPI_RESLN: [M][nslots][2] stats of the resid rows
  const float* rgamma;                // EPI_RESLN: LayerNorm gamma / beta of the residual
  const float* rbeta;
  float* stats_out;                   // EPI_STATS: [rows][nslots][2] per-slab (sum, sumsq)
  float inv_d;                        // 1 / LayerNorm width
  float eps;                          // LayerNorm epsilon (1e-5)
  int nslots;                         // stats rows are [nslots][2]: per-128-column-slab partials
  int stats_step;                     // EPI_LNIN: A row m reads stats_in row m * stats_step (0 = 1)
  int gR, gC;                         // EPI_GATHER: A row (b, y, x) of an OW x OW grid gathered
  float g_inv_rr, g_inv_r;            //   from the R x R token grid A (ld lda, C channels);
  int gmode, gOW;                     //   1/OW^2, 1/OW; gmode 1 Swin PatchMerging (OW = R/2),
  const void* gzero;                  //   2 T2T soft split k3 s2 p1 (C = 64; gzero: zero row)
  int* sk_flags;                      // stream-K hand-off flags [>= #CUs] (zero between launches)
  float* sk_part;                     // stream-K partial tiles [#CUs][256 * 256] fp32
  int ks_chunk;                       // split-K (128x128 kernel, gridDim.y splits): K per split;
  int64_t ks_stride;                  // fp32 partial C of split z at C + z * ks_stride
  int xgroups;                        // persistent 256x256 walk: XCD groups that each own
                                      // ntiles / xgroups weight panels (0 / 1: one group)
  int no_balance;                     // 1: persistent grids of 2-4 tile rounds keep one block per
                                      // CU (the launching model's lanes fill the idle CUs)
};
constexpr int GEMM_BM = 128;
constexpr int GEMM_BN = 128;
constexpr int PACK_N = 256;  // packed weight rows are padded to this (both tile shapes divide it)
constexpr int PAD_K = 64;   // K granularity (elements) of every packed operand
constexpr int PAD_N = 64;   // column granularity of activation buffers

hipError_t gemm_launch(int dtype, int flags, const GemmParams& p, hipStream_t s);
// Skinny GEMM (small M, long K: the classifier head) as S K-splits in one launch, fp32 partials
// part[S][M][ntiles*128], then a fixed-order reduction + bias (+ GELU) into C (deterministic).
// flags: EPI_BIAS and/or EPI_GELU and/or EPI_OUT_F32 only; K % (S * 64) == 0.
int device_cus();  // compute units of the current device (cached)
// whether gemm_launch(dtype, flags | EPI_HM, p) runs (the persistent 256 x 256 kernel with its
// head-major store; N = 3 H 64, M N 2 < 2^31); the caller keeps the token-major layout otherwise
bool gemm_headmajor_ok(int dtype, int flags, const GemmParams& p);
hipError_t gemm_splitk_launch(int dtype, int flags, const GemmParams& p, int S, float* part,
                              hipStream_t s);
void gemm_set_variant(int v);
// Bytes of the stream-K scratch of one GEMM stream (flags block first, zero it once after
// allocating: the kernel leaves every flag at 0); gemm_sk_bind splits it into the two arrays.
size_t gemm_sk_bytes();
void gemm_sk_bind(void* ws, GemmParams& p);
hipError_t pack_weight(int dtype, const float* W, const float* row_scale, int K, int N, void* Wp,
                       int Kpad, int Npad, hipStream_t s);
hipError_t to_bf16_launch(const float* x, void* y, int64_t n, hipStream_t s);  // y[i] = bf16(x[i])
// colsum[n] = sum_k Wp[n][k]; cvec[n] = sum_k beta[k] W[k][n] + bias[n] (bias may be null).
hipError_t ln_fold(int dtype, const void* Wp, int Kpad, const float* W, const float* beta,
                   const float* bias, int K, int N, float* colsum, float* cvec, int Npad,
                   hipStream_t s);

struct AttnParams {
  const void* qkv; int64_t ldq;   // token rows, columns (qkv h d)
  void* out;       int64_t ldo;   // token rows, columns (h d)
  int N;                          // tokens per image (<= 256)
  int H;                          // heads
  int B;                          // images
  float scale_log2;               // head_dim^-0.5 * log2(e)
  // bf16 only: when q8 is set, O is written as MX8 instead (e4m3 bytes q8[row][ldq8], scales
  // s8[ldq8/128][rows8] dwords; the MX8 model's out-proj operand) and `out` is not written
  uint8_t* q8 = nullptr;
  uint32_t* s8 = nullptr;
  int64_t ldq8 = 0;
  int rows8 = 0;
  int hd = 64;                    // head size h_k (<= 128; 64: the tuned kernels, else generic)
  // qkv addressing of the bf16 h_k = 64 kernels: (image b, head h) slice at qkv + b sb + h sh
  // (elements), its rows ldq apart, q / k / v at columns 0 / ko / vo of a row. All zero = the
  // token-major layout above (sb = N ldq, sh = 64, ko = H 64, vo = 2 H 64); the head-major layout
  // of the model's QKV GEMM (EPI_HM: [B][H][q | k | v][N][64]) sets sb = 3 H N 64, sh = 3 N 64,
  // ldq = 64, ko = N 64, vo = 2 N 64 (q, k and v of a slice each one contiguous run)
  int64_t sb = 0, sh = 0;
  int ko = 0, vo = 0;
};
hipError_t attention_launch(int dtype, const AttnParams& p, hipStream_t s);



// LayerNorm over rows of D (fp32 in) -> activation dtype out (eps 1e-5).
hipError_t layernorm_launch(int dtype, const float* x, int64_t ldx, void* y, int64_t ldy,
                            const float* gamma, const float* beta, int rows, int D, float eps,
                            hipStream_t s);

// Number of statistics slots of a LayerNorm of width D: one per 128-column slab of a 256-padded
// row (both GEMM tile shapes number their slabs n0 / 128).
__host__ __device__ inline int stats_slots(int D) { return 2 * ((D + 255) / 256); }

// NCHW fp32 images -> patch matrix [B*P, p*p*C] (p1 p2 c) in activation dtype; also writes
// the CLS token row x[b*(P+1)] = cls + pos[0] (activation dtype, row stride D) and, when stats is
// non-null, its (sum, sumsq) into slot 0 of stats[b*(P+1)] (other slots zeroed).
// channel_major: the patch vector's K axis in (c p1 p2) order instead (the model's layout; the
// patch weight then packed from patch_weight_cm's row permutation); requires ps % 8 == 0.
hipError_t patchify_launch(int dtype, const float* img, int B, int C, int HW, int ps, void* out,
                           void* x, const float* cls, const float* pos, int D, float* stats,
                           hipStream_t s, bool channel_major = false);
// Keras patch_to_embedding kernel W [(p1 p2 c), N] -> Wcm [(c p1 p2), N] (rows permuted).
hipError_t patch_weight_cm(const float* W, float* Wcm, int C, int ps, int N, hipStream_t s);

// ---- T2T stage (t2t.hip) ----
struct PerformerWeights {  // fp32 device pointers, Keras layouts
  const float* prmw;   // [32][64] random-feature matrix (already * sqrt(m))
  const float* out_w;  // [64][64] attn_output kernel [in][out]
  const float* out_b;  // [64]
  const float* ln2_g;  // [64]
  const float* ln2_b;  // [64]
  const float* fc1_w;  // [64][64]
  const float* fc1_b;  // [64]
  const float* fc2_w;  // [64][64]
  const float* fc2_b;  // [64]
};
// tf_Unfold(k, s, p, channel_last) of NHWC `in` (fp32 if in_f32 else dtype) -> rows [.., ldo].
hipError_t unfold_launch(int dtype, int in_f32, const void* in, int B, int H, int W, int C, int k,
                         int s, int p, void* out, int ldo, float* stats, int nslots,
                         hipStream_t st);
size_t performer_part_floats(int B, int ntok);
// kqv_perm (bf16): the kqv columns are in the permuted order kqv_permute_launch gives the model's
// kqv weights (t2t.hip kqv_col: 16-B row pieces per lane); false: the reference order
hipError_t performer_launch(int dtype, const void* kqv, int64_t ldq, int B, int ntok,
                            const PerformerWeights& w, float* part, void* out, int64_t ldo,
                            hipStream_t s, float* tstats = nullptr, bool kqv_perm = false);
// W [K][192] / bias [192] -> Wp / bp with the output columns of each 64-feature block permuted
hipError_t kqv_permute_launch(const float* W, const float* bias, int K, float* Wp, float* bp,
                              hipStream_t s);
// soft split (k 3, s 2, p 1) row statistics of the R x R token map from the per-token statistics
// performer_launch wrote (tstats: [B*R*R][2]) -> dst [rows][nslots][2] (t2t.hip)
hipError_t unfold_stats_launch(const float* tstats, int B, int R, float* dst, int nslots,
                               hipStream_t s);
// CLS rows x[b*ntok] = cls + pos[0] (dtype) and their LayerNorm slot statistics.
hipError_t cls_rows_launch(int dtype, void* x, int B, int ntok, int D, const float* cls,
                           const float* pos, float* stats, hipStream_t s);

// ---- Swin Transformer (swin.hip) ----
struct SwinAttnParams {
  const void* qkv; int64_t ldq;   // raster-order token rows [B*R*R], columns (qkv h d), head 32
  void* out;       int64_t ldo;   // raster-order rows, columns (h d); [C, ldo) written as 0
  const float* bias;              // [types][H][49][64] bias + shift mask, * log2(e); -inf past 49
  int B, R, nwx, C, H;            // images, resolution, windows per row (R / 7), channels, heads
  int shift;                      // cyclic shift (0: W-MSA, 3: SW-MSA with the region mask)
  float scale_log2;               // 32^-0.5 * log2(e)
};
hipError_t swin_patch_launch(int dtype, const float* img, int B, int C, int S, int ps, void* out,
                             int ldo, hipStream_t s);
hipError_t ln_rows_launch(int dtype, const void* x, int64_t ld, void* y, const float* gamma,
                          const float* beta, int rows, int D, float eps, float* stats, int nslots,
                          hipStream_t s);
hipError_t merge_launch(int dtype, const void* x, int64_t ldx, int B, int R, int C, void* out,
                        float* stats, int nslots, hipStream_t s);
// dense bias+mask tables [types][H][49][64] (types = 4 when shift > 0, else 1)
// floats of the tables rpb_dense_launch writes (dense [types][H][49][64] + compact [H][192])
size_t rpb_table_floats(int H, int w, int shift);
hipError_t rpb_dense_launch(const float* table, int H, int w, int shift, float* dense,
                            hipStream_t s);
hipError_t window_attn_launch(int dtype, const SwinAttnParams& p, hipStream_t s);
hipError_t ln_pool_launch(int dtype, const void* x, int64_t ldx, int B, int T, int D,
                          const float* stats, int nslots, const float* gamma, const float* beta,
                          void* out, int64_t ldo, hipStream_t s);

// Fused Swin MLP of a C = 96 stage (bf16): x = xm + FC2(GELU(FC1(LN2(xm)))) + row statistics.
struct SwinMlpParams {
  const void* xm;          // [M][96] block input (bf16)
  void* x;                 // [M][96] block output (bf16)
  const float* stats_in;   // [M][nslots][2] statistics of the xm rows (LN2)
  float* stats_out;        // [M][nslots][2] statistics of the x rows (slot 0 total, rest 0)
  const void* w1;          // FC1 packed [>= 384][ldw1] bf16, LN2 gamma folded
  const float* colsum;     // [384] FC1 LN-fold column sums
  const float* cvec;       // [384] FC1 beta.W + bias
  const void* w2;          // FC2 packed [>= 96][ldw2] bf16 (K = hidden)
  const float* b2;         // [96]
  int64_t ldw1, ldw2;
  int M, nslots;
  float eps;
};
hipError_t swin_mlp96_launch(const SwinMlpParams& p, hipStream_t s);

// Fused attention sublayer of a C = 96, 3-head stage (bf16): xm = x + proj(WMSA(LN1(x))) with
// the cyclic shift, QKV, window attention and proj of one window on chip; + row statistics of xm.
struct SwinAttnBlockParams {
  const void* x;           // [B*R*R][96] stage stream (bf16, raster order)
  void* xm;                // [B*R*R][96] output
  const float* stats_in;   // [rows][nslots][2] statistics of x (LN1)
  float* stats_out;        // [rows][nslots][2] statistics of xm
  const void* wqkv;        // QKV packed [>= 288][ldq] bf16, LN1 gamma folded
  const float* cqkv;       // [288] beta.W + qkv bias
  const void* wproj;       // proj packed [>= 96][ldp] bf16
  const float* bproj;      // [96]
  const float* bias;       // window bias + mask tables (rpb_dense_launch)
  int64_t ldq, ldp;
  int B, R, shift, nslots;
  float eps;
};
hipError_t swin_attn96_launch(const SwinAttnBlockParams& p, hipStream_t s);
// statistics of gathered PatchMerging rows from the source stream's slot statistics (swin.hip)
hipError_t merge_stats_launch(const float* src, int ns, int B, int R, float* dst, int nd,
                              hipStream_t s);
// fused Swin stem (swin.hip): Conv2d(3, 96, k = s = 4) + LayerNorm(96) -> bf16 stream + stats
struct SwinEmbedParams {
  const float* img;        // [B][3][S][S] fp32 NCHW
  const void* w;           // packed patch weights [>= 96][ldw] bf16, k = (c, kh, kw), zero past 48
  int64_t ldw;
  const float* bias;       // [96]
  const float* gamma;      // [96] embedding LayerNorm
  const float* beta;       // [96]
  void* x;                 // [B*(S/4)^2][96] bf16 stage-1 stream
  float* stats;            // [rows][nslots][2] statistics of x (slot 0; the rest zeroed)
  int B, S, nslots;
  float eps;
};
hipError_t swin_embed96_launch(const SwinEmbedParams& p, hipStream_t s);
int gemm_variant();  // the calling thread's evt_set_gemm_variant value (0 = automatic)
// automatic kernel selection (0; 30 / 31 only steer the 128 x 384 tiles): fused kernels allowed
inline bool gemm_auto() {
  const int v = gemm_variant();
  return v == 0 || v == 30 || v == 31;
}
bool gemm_variant_supported(int v);  // compiled into this build (lab variants: EVT_GEMM_LAB)

// ---- MXFP8 (mx8.hip): e4m3fn elements, e8m0 scale per 32 K, scales S[K/128][ld] dwords ----
struct Mx8GemmParams {
  const uint8_t* A;  int64_t lda;   // [M][K] e4m3 (bytes)
  const uint32_t* As; int64_t ldas; // [K/128][ldas] scale dwords (ldas >= M)
  const uint8_t* W;  int64_t ldw;   // packed [Npad][K] e4m3, Npad multiple of 128
  const uint32_t* Ws; int64_t ldws; // [K/128][ldws = Npad]
  void* C;           int64_t ldc;   // bf16 / fp32 / e4m3 bytes (EPI_OUT_MX8)
  uint32_t* Cs;      int64_t ldcs;  // EPI_OUT_MX8: [N/128][ldcs] output scales (N % 32 == 0)
  int M, N, K;                      // K multiple of 128, N multiple of 8
  const float* bias;                // >= N floats
  const void* resid; int64_t ldr;   // bf16
  const float* rstats;              // EPI_RESLN: [M] (mu, rstd) of the resid rows (ln_mx8_launch)
  const float* rgamma;              // EPI_RESLN: LayerNorm gamma / beta [N]
  const float* rbeta;
};
hipError_t mx8_quantize_launch(int in_dtype, const void* x, int64_t ldx, int rows, int K, int Kpad,
                               void* q, int64_t ldq, uint32_t* s, int64_t lds, hipStream_t st);
hipError_t mx8_pack_launch(const float* W, const float* row_scale, int K, int N, void* Wq, int Kpad,
                           int Npad, uint32_t* s, hipStream_t st);
hipError_t gemm_mx8_launch(int flags, const Mx8GemmParams& p, hipStream_t s);
// LayerNorm of bf16 rows [rows][D] -> MX8 q [rows][Kpad] + scales [Kpad/128][rows] and, if
// stats, (mu, rstd) per row [rows][2]; D % 8 == 0, D <= Kpad <= 1024.
hipError_t ln_mx8_launch(const void* x, int rows, int D, int Kpad, const float* gamma,
                         const float* beta, float eps, float* stats, void* q, uint32_t* s,
                         hipStream_t st);

}  // namespace evt
