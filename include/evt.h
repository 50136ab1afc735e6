/*
 * evt.h - C ABI of libevt_hip.so, the MI355X (gfx950) Vision-Transformer inference path.
 *
 * Drop-in boundary for the reference's `modeling.models` forward (xudoong/EdgeVisionTransformer).
 * The reference has no FFI: its "operator API" for this path is the tf.keras.Model contract
 *   construct  ViT(dim=, depth=, heads=, mlp_dim=, ...)          modeling/models/vit.py:11
 *              ViT_Pruned(..., head_size=64, prune_encoding=)     modeling/models/vit.py:60
 *              get_deit_{tiny,small,base}()                       modeling/models/vit.py:100-109
 *   call       model(img) -> logits                               modeling/models/vit.py:41-55
 * Each entry point below replaces one piece of that contract (cited per function); the Python
 * mirror `edgevisiontransformer_amd.modeling.models.vit` binds them with ctypes
 * (INTEGRATION.md shows the binding a maintainer would add on the reference side).
 *
 * Conventions
 *   - Plain C types only; no torch types cross the boundary.
 *   - All tensor pointers are DEVICE pointers (HIP, same device as evt_init); the caller owns
 *     them. The library copies/packs weights at create time and owns only its packed weights
 *     and its workspace.
 *   - Return 0 (EVT_OK) on success, a negative code on error; never throws. evt_last_error()
 *     returns a thread-local message for the last failure on the calling thread.
 *   - `stream` is a hipStream_t (NULL = default stream). Calls on one model handle must be
 *     serialised by the caller (one stream per handle); handles are independent.
 */
#ifndef EVT_H_
#define EVT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EVT_OK 0
#define EVT_EINVAL (-22) /* bad shape / argument (reference: ValueError / assert) */
#define EVT_ENOMEM (-12) /* device allocation failed */
#define EVT_EHIP (-5)    /* HIP runtime / launch error */
#define EVT_ENODEV (-19) /* no usable gfx950 device */

#define EVT_DTYPE_F32 0  /* exact fp32 path (v_mfma_f32_16x16x4_f32), logits within 1e-3 */
#define EVT_DTYPE_BF16 1 /* bf16 MFMA, fp32 accumulate / LN / softmax / GELU statistics */

/* Static shape of a ViT / ViT_Pruned (reference modeling/models/vit.py:11-75).
 * heads/head_dim/ffn are per-layer arrays of length `depth` (the pruned encoding, decoded by the
 * host mirror exactly as ViT_Pruned.decode_prune_encoding, vit.py:77-97). */
typedef struct evt_vit_desc {
  int32_t image_size;   /* 224 */
  int32_t patch_size;   /* 16; image_size % patch_size == 0 (vit.py:13) */
  int32_t in_chans;     /* 3 */
  int32_t num_classes;  /* 1000 */
  int32_t dim;          /* D: 192 / 384 / 768; multiple of 64, <= 1024 */
  int32_t depth;        /* 12 */
  int32_t mlp_dim;      /* head MLP width M (vit.py:38) */
  const int32_t* heads;    /* [depth] heads per layer (attention.py:5) */
  const int32_t* head_dim; /* [depth] h_k per layer; this build requires 64 */
  const int32_t* ffn;      /* [depth] FFN width per layer (ffn.py:5) */
  int32_t dtype;        /* EVT_DTYPE_* */
  int32_t max_batch;    /* workspace is sized for this many images */
} evt_vit_desc;

typedef struct evt_model evt_model;

/* Select and validate the device (must be gfx950). */
int evt_init(int device);

/* Thread-local description of the last error on this thread ("" if none). */
const char* evt_last_error(void);

/* Number of fp32 weight tensors evt_vit_create expects for `desc`, in order:
 *   patch_w [p*p*c, D], patch_b [D], cls [D], pos [P+1, D],
 *   per layer i: ln1_g [D], ln1_b [D], qkv_w [D, 3*h*hk], out_w [h*hk, D], out_b [D],
 *                ln2_g [D], ln2_b [D], fc1_w [D, F], fc1_b [F], fc2_w [F, D], fc2_b [D],
 *   head1_w [D, M], head1_b [M], head2_w [M, C], head2_b [C].
 * Kernels are Keras Dense layout [in, out] (y = x @ W + b). Replaces the weight creation of
 * ViT.__init__ (vit.py:18-39) + TransformerEncoderBlock(_Pruned).__init__ (transformer_encoder.py:9-36). */
int evt_vit_num_weights(const evt_vit_desc* desc);

/* Build a model: validates the shape, packs weights (fp32 device pointers, Keras layout) into the
 * kernel layout of desc->dtype, allocates the workspace for desc->max_batch images. The caller
 * may free its weight buffers once this returns (work is complete on `stream` return). */
int evt_vit_create(const evt_vit_desc* desc, const float* const* weights, int n_weights,
                   void* stream, evt_model** out);

/* Forward pass (reference ViT.call, vit.py:41-55): img fp32 NCHW [batch, C, H, W] ->
 * logits fp32 [batch, num_classes]. Asynchronous on `stream`. batch <= max_batch. */
int evt_vit_forward(evt_model* model, const float* img, int batch, float* logits, void* stream);

/* Bytes of device workspace evt_vit_create allocates for `batch` images. */
int evt_query_workspace(const evt_vit_desc* desc, int batch, size_t* bytes);

/* Release everything the handle owns. NULL is accepted. */
int evt_model_destroy(evt_model* model);

/* ---- op-level entry points (one per hot-path kernel; used by the parity tests) ---------- */

/* GEMM tile-shape policy for bf16 (process-wide tuning knob): 0 = automatic (256x256 tiles when
 * the problem fills the chip, else 128x128), 1 = always 128x128, 2 = 256x256 whenever packable. */
int evt_set_gemm_variant(int variant);

/* Pack a Keras [K, N] fp32 kernel into the GEMM operand layout Wp[Npad][Kpad] (dtype),
 * zero padded. Npad % 128 == 0, Kpad % 64 == 0. */
int evt_pack_weight(int dtype, const float* W, int K, int N, void* Wp, int Kpad, int Npad,
                    void* stream);

/* Dense layer on the token matrix: C = epi(A[M, K] . W) (reference tf.keras.layers.Dense).
 * flags: 1 bias, 2 gelu (tanh), 4 residual add (resid, activation dtype), 8 patch-embed
 * (row remap + pos add), 16 fp32 output. Supported combinations: 0, 3, 21, 17, 25, 1. */
int evt_dense(int dtype, int flags, const void* A, int64_t lda, const void* Wp, int Kpad, int Npad,
              void* C, int64_t ldc, int M, int N, const float* bias, const void* resid,
              int64_t ldr, const float* pos, int64_t ldp, int P, void* stream);

/* Multi-head attention core (attention.py:20-34): qkv [B*N, ldq] with columns (qkv h d), head
 * size 64 -> out [B*N, ldo] columns (h d). N <= 256. */
int evt_attention(int dtype, const void* qkv, int64_t ldq, void* out, int64_t ldo, int B, int N,
                  int H, float scale, void* stream);

/* LayerNormalization(epsilon) over rows of D (norm.py:6): fp32 x -> y (dtype). */
int evt_layernorm(int dtype, const float* x, int64_t ldx, void* y, int64_t ldy,
                  const float* gamma, const float* beta, int rows, int D, float eps, void* stream);

/* Rearrange 'b c (h p1) (w p2) -> b (h w) (p1 p2 c)' (vit.py:31-32) of fp32 NCHW images into
 * out [B*P, p*p*C] (dtype); also writes x[b*(P+1)*D + n] = cls[n] + pos[n] (vit.py:48-51). */
int evt_patchify(int dtype, const float* img, int B, int C, int HW, int ps, void* out, float* x,
                 const float* cls, const float* pos, int D, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* EVT_H_ */
