// Host-side kernel launch interface shared by the .hip translation units and capi.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace evt {

enum Dtype : int { DT_F32 = 0, DT_BF16 = 1 };

// Epilogue flags of the token-matrix GEMM.
enum : int { EPI_BIAS = 1, EPI_GELU = 2, EPI_RESID = 4, EPI_POS = 8, EPI_OUT_F32 = 16 };

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
  int vec_ok;                         // all leading dims multiple of 4 -> vector epilogue
};
constexpr int GEMM_BM = 128;
constexpr int GEMM_BN = 128;
constexpr int PACK_N = 256;  // packed weight rows are padded to this (both tile shapes divide it)
constexpr int PAD_K = 64;   // K granularity (elements) of every packed operand
constexpr int PAD_N = 64;   // column granularity of activation buffers

hipError_t gemm_launch(int dtype, int flags, const GemmParams& p, hipStream_t s);
void gemm_set_variant(int v);  // 0 auto, 1 force 128x128 tiles, 2 force 256x256 (bf16)
hipError_t pack_weight(int dtype, const float* W, int K, int N, void* Wp, int Kpad, int Npad,
                       hipStream_t s);

struct AttnParams {
  const void* qkv; int64_t ldq;   // token rows, columns (qkv h d)
  void* out;       int64_t ldo;   // token rows, columns (h d)
  int N;                          // tokens per image (<= 256)
  int H;                          // heads; head_dim is fixed at 64
  int B;                          // images
  float scale_log2;               // head_dim^-0.5 * log2(e)
};
hipError_t attention_launch(int dtype, const AttnParams& p, hipStream_t s);

// LayerNorm over rows of D (fp32 in) -> activation dtype out (eps 1e-5).
hipError_t layernorm_launch(int dtype, const float* x, int64_t ldx, void* y, int64_t ldy,
                            const float* gamma, const float* beta, int rows, int D, float eps,
                            hipStream_t s);

// NCHW fp32 images -> patch matrix [B*P, p*p*C] (p1 p2 c) in activation dtype; also writes
// x[b*(P+1)] = cls + pos[0] (fp32 token stream).
hipError_t patchify_launch(int dtype, const float* img, int B, int C, int HW, int ps, void* out,
                           float* x, const float* cls, const float* pos, int D, hipStream_t s);

// Gather token-0 rows of the fp32 stream into a dense [B, D] activation-dtype matrix.
hipError_t gather_cls_launch(int dtype, const float* x, int64_t row_stride, int B, int D, void* out,
                             hipStream_t s);

}  // namespace evt
