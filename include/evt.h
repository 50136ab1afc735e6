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
#define EVT_DTYPE_MX8 2  /* evt_vit_* with EVT_VIT_REFERENCE only: MXFP8 (OCP MX e4m3) encoder
                          * Dense layers (QKV, out-proj, FC1, FC2) on the block-scaled MFMA,
                          * LayerNorm in the quantizer, bf16 patch embed / attention / head */

/* Static shape of a ViT / ViT_Pruned (reference modeling/models/vit.py:11-75).
 * heads/head_dim/ffn are per-layer arrays of length `depth` (the pruned encoding, decoded by the
 * host mirror exactly as ViT_Pruned.decode_prune_encoding, vit.py:77-97). */
typedef struct evt_vit_desc {
  int32_t image_size;   /* 224 */
  int32_t patch_size;   /* 16; image_size % patch_size == 0 (vit.py:13) */
  int32_t in_chans;     /* 3 */
  int32_t num_classes;  /* 1000 */
  int32_t dim;          /* D: 192 / 384 / 768; multiple of 8, <= 1024 (MX8: of 64) */
  int32_t depth;        /* 12 */
  int32_t mlp_dim;      /* head MLP width M (vit.py:38) */
  const int32_t* heads;    /* [depth] heads per layer (attention.py:5) */
  const int32_t* head_dim; /* [depth] h_k per layer, in [1, 128]; heads * h_k % 8 == 0 (MX8: 64) */
  const int32_t* ffn;      /* [depth] FFN width per layer (ffn.py:5) */
  int32_t dtype;        /* EVT_DTYPE_* */
  int32_t max_batch;    /* workspace is sized for this many images */
  int32_t semantics;    /* EVT_VIT_REFERENCE (0, the reference Keras model) or EVT_VIT_STANDARD */
  float layer_norm_eps; /* LayerNorm epsilon; 0 = 1e-5 (Keras / reference norm.py:6) */
} evt_vit_desc;

/* evt_vit_desc.semantics.
 * EVT_VIT_REFERENCE: exactly modeling/models/vit.py: block returns f(LN(x)) + LN(x) (norm.py:11-12
 *   + residual.py:9), QKV without bias, tanh GELU, no final LayerNorm, mlp_head = Dense(M, gelu)
 *   -> Dense(C) on token 0.
 * EVT_VIT_STANDARD: the published DeiT / ViT (timm VisionTransformer, HF DeiTModel; what the
 *   reference loads for accuracy, utils.py:52-62): x + f(LN(x)), QKV with bias, exact (erf) GELU,
 *   final LayerNorm, one Linear head on token 0 (mlp_dim unused). Weight order in
 *   evt_vit_num_weights. */
#define EVT_VIT_REFERENCE 0
#define EVT_VIT_STANDARD 1

typedef struct evt_model evt_model;

/* Select and validate the device (must be gfx950). */
int evt_init(int device);

/* Thread-local description of the last error on this thread ("" if none). */
const char* evt_last_error(void);

/* Number of fp32 weight tensors evt_vit_create expects for `desc`, in order:
 *   patch_w [p*p*c, D], patch_b [D], cls [D], pos [P+1, D],
 *   per layer i: ln1_g [D], ln1_b [D], qkv_w [D, 3*h*hk], (STANDARD: qkv_b [3*h*hk],)
 *                out_w [h*hk, D], out_b [D],
 *                ln2_g [D], ln2_b [D], fc1_w [D, F], fc1_b [F], fc2_w [F, D], fc2_b [D],
 *   REFERENCE: head1_w [D, M], head1_b [M], head2_w [M, C], head2_b [C];
 *   STANDARD:  norm_g [D], norm_b [D], head_w [D, C], head_b [C].
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

/* HIP graph of one forward (either family): captures evt_vit_forward / evt_t2t_forward of
 * (img, batch, logits) on `stream` (must be a non-NULL stream not being captured) into a graph
 * owned by the model, replacing any previous one; evt_graph_launch replays it on `stream`
 * (same pointers, same batch: the caller refills img in place). Removes the per-kernel launch
 * cost of the ~80-launch forward at small batch. */
int evt_graph_capture(evt_model* model, const float* img, int batch, float* logits, void* stream);
int evt_graph_launch(evt_model* model, void* stream);

/* Bytes of device workspace evt_vit_create allocates for `batch` images. */
int evt_query_workspace(const evt_vit_desc* desc, int batch, size_t* bytes);

/* Release everything the handle owns, after waiting for the device (forwards still in flight on
 * any stream finish first). NULL is accepted. */
int evt_model_destroy(evt_model* model);

/* Batch lanes (any handle; the reference's tools.py times one model.call per batch,
 * tools.py:82-116): with lanes = k > 1 every later forward of batch >= k splits its images into k
 * contiguous parts of sizes differing by at most one, each run by a child of the handle (the
 * handle's weights, its own workspace for ceil(max_batch / k) images: about k + 1 workspaces in
 * all) on its own HIP stream, forked from and joined to the caller's stream by events, so the
 * kernels of the parts fill each other's idle CUs (the GEMMs at 1.5 tile rounds, the latency-bound
 * fused Swin stage-1 kernels). Logits are the same as the one-lane forward's wherever the parts
 * take the same kernels as the whole batch (bitwise at the BASELINE batch sizes, tests/
 * test_gpu_lanes.py). Forwards while profiling (evt_model_profile) run as one lane. lanes = 1
 * drops the children. Synchronises the device; call before evt_graph_capture (a capture records
 * the lanes as parallel branches). `stream` orders the workspace initialisation. EVT_EINVAL for
 * lanes outside [1, 4]. Measured: faster for T2T-ViT-14 / Swin-T bf16 and DeiT-tiny
 * fp32 at 256 images, slower for DeiT-base bf16 (512 and 64 images) and DeiT-tiny bf16. */
int evt_model_set_lanes(evt_model* model, int lanes, void* stream);
/* Run the lanes on the caller's streams (n = the lane count; they must outlive the handle or
 * the next evt_model_set_lanes) instead of the ones evt_model_set_lanes created (destroyed here):
 * for a host framework's stream pool. Each lane stream should map to its own hardware queue, apart
 * from the other lanes' (HIP gives a new stream the least-used of GPU_MAX_HW_QUEUES queues; two
 * lanes on one queue run one after the other). Synchronises the device. */
int evt_model_set_lane_streams(evt_model* model, int n, void* const* streams);
/* The handle's lane count (1 without lanes). */
int evt_model_lanes(const evt_model* model, int* lanes);

/* ---- op-level entry points (one per hot-path kernel; used by the parity tests) ---------- */



/* Per-kernel timing of real forwards (the reference times whole models and per-layer micro-models,
 * tools.py:82-116 / utils.py:322-406; this is the device-side equivalent): while enabled, every
 * launch of a forward on the model is bracketed by HIP events on its stream, and
 * evt_model_profile_read returns, per role, the summed device time (us) and launch count of the
 * LAST forward (it waits for that forward's events). Not for use inside evt_graph_capture. */
enum {
  EVT_PROF_PATCHIFY = 0,        /* einops Rearrange (+ CLS row)        vit.py:31-32,45-51 */
  EVT_PROF_PATCH_EMBED = 1,     /* patch_to_embedding Dense + pos       vit.py:23,46,51 */
  EVT_PROF_QKV = 2,             /* LN1-folded to_qkv                    attention.py:17,24 */
  EVT_PROF_ATTENTION = 3,       /* softmax(q k^T) v                     attention.py:20-34 */
  EVT_PROF_OUT_PROJ = 4,        /* to_out + LN1(x) residual             attention.py:18,35 */
  EVT_PROF_FC1 = 5,             /* LN2-folded Dense(M, gelu)            ffn.py:8 */
  EVT_PROF_FC2 = 6,             /* Dense(D) + LN2(xm) residual          ffn.py:9 */
  EVT_PROF_HEAD = 7,            /* mlp_head / classifier                vit.py:38-39,55 */
  /* 8: unused (the round-1..4 fused QKV + attention kernel, measured slower, removed) */
  EVT_PROF_T2T_UNFOLD = 9,      /* tf_Unfold soft splits 0-2            t2t_vit.py:7-40,66-81 */
  EVT_PROF_T2T_KQV = 10,        /* TokenPerformer LN1-folded kqv Dense  transformer_encoder.py:84 */
  EVT_PROF_T2T_PERFORMER = 11,  /* TokenPerformer core (prm_exp .. FFN) transformer_encoder.py:67-99 */
  EVT_PROF_MERGE = 12,          /* Swin PatchMerging gather + LN-folded reduction */
  EVT_PROF_ATTN_SUBLAYER = 13,  /* Swin stage-1 fused LN1 + QKV + W-MSA + proj + residual */
  EVT_PROF_MLP = 14,            /* Swin stage-1 fused LN2 + FC1 + GELU + FC2 + residual */
  EVT_PROF_ROLES = 15
};
/* T2T-ViT also reports its project Dense (+ CLS rows, t2t_vit.py:86,121-125) as PATCH_EMBED and
 * its LN-folded classifier as HEAD; Swin its patch im2col as PATCHIFY, patch Dense + patch norm
 * as PATCH_EMBED, W-MSA as ATTENTION, proj as OUT_PROJ, final norm + pool + head as HEAD. */
int evt_model_profile(evt_model* m, int enable);
int evt_model_profile_read(evt_model* m, float* us, int* launches);
/* Algorithmic work of the last profiled forward, per role (arrays of EVT_PROF_ROLES): gflop =
 * 2 x multiply-adds of the role's contractions (Dense: 2 M K N with the layer's real K, N;
 * attention: 4 B H N^2 d), gbytes = the bytes its kernels must move at least (every operand read
 * once, every output written once: activations, weights, residuals, row statistics). Replaces
 * the reference's FLOP counter (flops_calculation.py:216-251) per kernel; bench.py divides by the
 * role's time for the MFMA and HBM roofline fractions. */
int evt_model_profile_work(evt_model* m, double* gflop, double* gbytes);

/* Pack a Keras [K, N] fp32 kernel into the GEMM operand layout Wp[Npad][Kpad] (dtype), zero
 * padded, optionally scaling row k by row_scale[k] (a LayerNorm gamma folded into the weights;
 * NULL = no scaling). Npad % 128 == 0, Kpad % 64 == 0. */
int evt_pack_weight(int dtype, const float* W, const float* row_scale, int K, int N, void* Wp,
                    int Kpad, int Npad, void* stream);

/* LayerNorm-fold vectors of a packed weight: colsum[n] = sum_k Wp[n][k] and
 * cvec[n] = sum_k beta[k] W[k][n] + bias[n] (bias may be NULL); arrays of length Npad. */
int evt_ln_fold(int dtype, const void* Wp, int Kpad, int Npad, const float* W, const float* beta,
                const float* bias, int K, int N, float* colsum, float* cvec, void* stream);

/* Epilogue flags of evt_dense (combinable as listed under evt_dense). */
#define EVT_EPI_BIAS 1     /* + bias[n] */
#define EVT_EPI_GELU 2     /* tanh-GELU (activation.py:13-15) */
#define EVT_EPI_RESID 4    /* + resid[m][n] (residual.py:9) */
#define EVT_EPI_POS 8      /* patch embed: row b*P+t -> b*(P+1)+1+t, + pos[t+1][n] (vit.py:45-51) */
#define EVT_EPI_OUT_F32 16 /* fp32 output (else activation dtype) */
#define EVT_EPI_LNIN 32    /* A rows un-normalised: r*acc - r*mu*colsum[n] (+ bias = cvec) */
#define EVT_EPI_RESLN 64   /* residual is LN(resid) with rstats / rgamma / rbeta (norm.py:12) */
#define EVT_EPI_STATS 128  /* write per-slab (sum, sumsq) of each stored row into stats_out */
#define EVT_EPI_GELU_ERF 256 /* exact erf GELU (torch nn.GELU, the Swin MLP) */
/* LayerNorm row statistics layout: float stats[rows][S][2], S = 2 * ceil(ln_width / 256) slots
 * (one per 128-column slab); a row's (sum, sumsq) is the sum over its S slots. */

typedef struct evt_dense_args {
  int32_t flags;
  const void* A;   int64_t lda;     /* [M, Kpad] activation dtype */
  const void* Wp;  int32_t Kpad;  int32_t Npad;
  void* C;         int64_t ldc;     /* [M, N] (fp32 with EVT_EPI_OUT_F32) */
  int32_t M, N;
  const float* bias;                /* >= N floats */
  const void* resid; int64_t ldr;   /* activation dtype; with EVT_EPI_POS (bf16): optional bf16
                                       copy of pos [P+1][ldr] (the persistent-kernel path) */
  const float* pos;  int64_t ldp;  int32_t P;
  const float* colsum;              /* EVT_EPI_LNIN */
  const float* stats_in;            /* EVT_EPI_LNIN: [M][S][2] slot statistics of the A rows */
  const float* rstats;              /* EVT_EPI_RESLN: [M][S][2] slot statistics of resid rows */
  const float* rgamma; const float* rbeta;
  float* stats_out;                 /* EVT_EPI_STATS: [rows][S][2], this call's slots written */
  int32_t ln_width;                 /* LayerNorm width (D) for the stats */
  float ln_eps;                     /* LayerNorm epsilon (1e-5 in the reference) */
  int32_t stats_step;               /* EVT_EPI_LNIN: A row m uses stats_in row m * stats_step
                                       (0 or 1: consecutive; T: the CLS rows of a token stream) */
} evt_dense_args;

/* Dense layer on the token matrix: C = epi(A . W) (reference tf.keras.layers.Dense), one of the
 * flag sets 0, 1, 3, 17, 21, 25, 137 (patch embed -> stream), 33 (LN-folded QKV),
 * 35 (LN-folded FC1 + GELU), 49 (LN-folded classifier, fp32 logits), 197 (out-proj / FC2 + LN
 * residual + stats); Swin: 289 (LN-folded FC1 + erf GELU), 133 (proj / FC2 + residual + stats),
 * 161 (LN-folded patch-merge reduction + stats). */
int evt_dense(int dtype, const evt_dense_args* args, void* stream);

/* The same Dense as `splits` K-slices in one launch (the classifier head's path, M = batch: the
 * plain tile grid would leave most CUs idle): fp32 partial products into `partials`
 * ([splits][M][Npad] floats, caller-owned), then a fixed-order reduction with bias / tanh GELU
 * (flags a subset of EVT_EPI_BIAS | EVT_EPI_GELU | EVT_EPI_OUT_F32; Kpad % (splits * 64) == 0).
 * Reference: mlp_head `vit.py:38-39,55`. */
int evt_dense_splitk(int dtype, const evt_dense_args* args, int splits, float* partials,
                     void* stream);

/* Multi-head attention core (attention.py:20-34): qkv [B*N, ldq] with columns (qkv h d), head
 * size 64 -> out [B*N, ldo] columns (h d). N <= 256. */
int evt_attention(int dtype, const void* qkv, int64_t ldq, void* out, int64_t ldo, int B, int N,
                  int H, float scale, void* stream);

/* evt_attention for any head size h_k = head_dim in [1, 128] (attention.py:6-12: h_k = dim //
 * heads): qkv [B*N, ldq >= 3*H*h_k] columns (qkv h d), out [B*N, ldo >= H*h_k] columns (h d).
 * h_k == 64 runs the tuned kernels, other sizes generic ones (features zero-padded to 32 / 64). */
int evt_attention_hd(int dtype, const void* qkv, int64_t ldq, void* out, int64_t ldo, int B, int N,
                     int H, int head_dim, float scale, void* stream);

/* LayerNormalization(epsilon) over rows of D (norm.py:6): fp32 x -> y (dtype). */
int evt_layernorm(int dtype, const float* x, int64_t ldx, void* y, int64_t ldy,
                  const float* gamma, const float* beta, int rows, int D, float eps, void* stream);

/* Rearrange 'b c (h p1) (w p2) -> b (h w) (p1 p2 c)' (vit.py:31-32) of fp32 NCHW images into
 * out [B*P, p*p*C] (dtype); also writes the CLS row x[b*(P+1)*D + n] = cls[n] + pos[n] (dtype,
 * vit.py:48-51) and, if stats != NULL, its (sum, sumsq) into slot 0 of stats[b*(P+1)] (the
 * other S-1 slots of that row zeroed; S from the LayerNorm width D as above). */
int evt_patchify(int dtype, const float* img, int B, int C, int HW, int ps, void* out, void* x,
                 const float* cls, const float* pos, int D, float* stats, void* stream);

/* evt_patchify with the patch vector's K axis in channel-major (c p1 p2) order - the layout the
 * model uses: each vector is C*ps runs of ps contiguous pixels (a streaming gather), and the
 * model packs its patch-embedding weight rows in the same permuted order, so the product is the
 * reference Dense of the (p1 p2 c) vector. ps % 8 == 0. */
int evt_patchify_cm(int dtype, const float* img, int B, int C, int HW, int ps, void* out, void* x,
                    const float* cls, const float* pos, int D, float* stats, void* stream);

/* ---- T2T-ViT (reference modeling/models/t2t_vit.py) ------------------------------------ */

/* Static shape of a T2T_ViT (t2t_vit.py:91-114; factories get_t2t_vit_{7,10,12,14} :138-148).
 * tokens_type 'performer' only (:49-59). Soft splits k7s4p2, k3s2p1, k3s2p1 give S/4, S/8 and
 * S/16 token grids; image_size must be a multiple of 16 with (S/16)^2 + 1 <= 256 tokens. */
typedef struct evt_t2t_desc {
  int32_t image_size;   /* S = 224 */
  int32_t in_chans;     /* 3 */
  int32_t num_classes;  /* 1000 */
  int32_t dim;          /* hidden_size: multiple of 8, <= 1024 */
  int32_t depth;        /* encoder layers */
  int32_t heads;        /* num_heads; h_k = dim / heads <= 128 (attention.py:6-12) */
  int32_t mlp_dim;      /* int(mlp_ratio * hidden_size) */
  int32_t token_size;   /* TokenPerformer head size; this build requires 64 (m = 32) */
  int32_t dtype;        /* EVT_DTYPE_* */
  int32_t max_batch;
} evt_t2t_desc;

/* Number of fp32 weight tensors evt_t2t_create expects, in order:
 *   for performer p1 (Din = 49*in_chans) then p2 (Din = 9*token_size):
 *     ln1_g [Din], ln1_b [Din], kqv_w [Din, 3*hs], kqv_b [3*hs], w [m, hs] (Orthogonal*sqrt(m),
 *     transformer_encoder.py:60-65), out_w [hs, hs], out_b [hs], ln2_g [hs], ln2_b [hs],
 *     fc1_w [hs, hs], fc1_b [hs], fc2_w [hs, hs], fc2_b [hs]
 *   project_w [9*hs, D], project_b [D], cls [D], pos [P+1, D] (the sinusoid table),
 *   per layer i: the 11 ViT encoder tensors (see evt_vit_num_weights),
 *   norm_g [D], norm_b [D], head_w [D, C], head_b [C]. */
int evt_t2t_num_weights(const evt_t2t_desc* desc);

/* Build a T2T-ViT (same ownership rules as evt_vit_create). */
int evt_t2t_create(const evt_t2t_desc* desc, const float* const* weights, int n_weights,
                   void* stream, evt_model** out);

/* Forward (T2T_ViT.call, t2t_vit.py:120-135): img fp32 NHWC [batch, S, S, in_chans] ->
 * logits fp32 [batch, num_classes]. Asynchronous on `stream`. */
int evt_t2t_forward(evt_model* model, const float* img, int batch, float* logits, void* stream);

/* Bytes of device workspace evt_t2t_create allocates for `batch` images. */
int evt_t2t_query_workspace(const evt_t2t_desc* desc, int batch, size_t* bytes);

/* tf_Unfold(k, stride, pad, channel_last=True) (t2t_vit.py:7-40): NHWC in [B, H, W, C]
 * (fp32 when in_f32, else `dtype`) -> out [B*OH*OW, ldo] (dtype), vector order (kh, kw, c) of
 * tf.image.extract_patches, columns [k*k*C, ldo) zeroed (ldo <= 256; <= 512 when ldo is even;
 * <= 1024 when C % 4 == 0 and ldo % 4 == 0). If stats != NULL, each row's
 * (sum, sumsq) goes to slot 0 of stats[row][nslots][2] (other slots zeroed). */
int evt_unfold(int dtype, int in_f32, const void* in, int B, int H, int W, int C, int k,
               int stride, int pad, void* out, int ldo, float* stats, int nslots, void* stream);

/* TokenPerformer core after its kqv Dense (transformer_encoder.py:83-99): kqv [B*T, ldq]
 * (columns k | q | v, 64 each) -> out [B*T, ldo] = y + FFN(LN2(y)), y = v + attn_output(
 * qp kptv^T / (D + 1e-8)). Weights fp32 Keras layouts: w [32, 64], out_w/fc1_w/fc2_w [64, 64],
 * out_b/ln2_g/ln2_b/fc1_b/fc2_b [64]. `part` is scratch of evt_performer_scratch floats. */
int evt_performer(int dtype, const void* kqv, int64_t ldq, int B, int T, const float* w,
                  const float* out_w, const float* out_b, const float* ln2_g, const float* ln2_b,
                  const float* fc1_w, const float* fc1_b, const float* fc2_w, const float* fc2_b,
                  float* part, void* out, int64_t ldo, void* stream);

/* fp32 scratch elements evt_performer needs for B images of T tokens: per image, a (kptv, ksum)
 * partial of 64*32 + 32 floats per 196-token chunk and their sum. */
int64_t evt_performer_scratch(int B, int T);

/* ---- Swin Transformer (reference utils.py:14-47 get_swin -> microsoft SwinTransformer) ---- */

#define EVT_SWIN_MAX_STAGES 8

/* Static shape of a SwinTransformer(img_size, patch_size, in_chans, num_classes, embed_dim, depths,
 * num_heads, window_size, mlp_ratio, qkv_bias=True, ape=False, patch_norm=True) as get_swin builds
 * it (utils.py:28-43; swin_tiny_patch4_window7_224 = embed 96, depths (2,2,6,2), heads
 * (3,6,12,24)). This build: window 7, head size 32 (stage width / heads), every stage resolution
 * a multiple of 7 (no padding), stage width <= 1024. */
typedef struct evt_swin_desc {
  int32_t image_size;   /* 224 */
  int32_t patch_size;   /* 4 */
  int32_t in_chans;     /* 3 */
  int32_t num_classes;  /* 1000 */
  int32_t embed_dim;    /* 96; stage i has embed_dim << i channels */
  int32_t num_stages;   /* len(depths), <= EVT_SWIN_MAX_STAGES */
  int32_t depths[EVT_SWIN_MAX_STAGES];
  int32_t num_heads[EVT_SWIN_MAX_STAGES];
  int32_t window_size;  /* 7 */
  float mlp_ratio;      /* 4.0: MLP width int(C * mlp_ratio) */
  int32_t dtype;        /* EVT_DTYPE_* */
  int32_t max_batch;
} evt_swin_desc;

/* Number of fp32 weight tensors evt_swin_create expects, in order:
 *   patch_w [in_chans*p*p, E] (Conv2d kernel, rows (c, kh, kw)), patch_b [E], pnorm_g [E], pnorm_b [E],
 *   per stage i (width C): if i > 0: merge_g [2C], merge_b [2C], merge_w [2C, C] (LayerNorm(4C') +
 *     reduction Linear(4C', 2C', bias=False) of PatchMerging, C' = C / 2);
 *     per block: ln1_g [C], ln1_b [C], qkv_w [C, 3C] (columns (qkv h d)), qkv_b [3C],
 *       rpb [169, heads] (relative_position_bias_table), proj_w [C, C], proj_b [C], ln2_g [C],
 *       ln2_b [C], fc1_w [C, M], fc1_b [M], fc2_w [M, C], fc2_b [C]   (M = int(C * mlp_ratio))
 *   norm_g [F], norm_b [F], head_w [F, classes], head_b [classes]   (F = last stage width).
 * Dense kernels are [in, out] (the transpose of a torch Linear weight). */
int evt_swin_num_weights(const evt_swin_desc* desc);

/* Build a Swin model (same ownership rules as evt_vit_create). */
int evt_swin_create(const evt_swin_desc* desc, const float* const* weights, int n_weights,
                    void* stream, evt_model** out);

/* Forward (SwinTransformer.forward): img fp32 NCHW [batch, in_chans, S, S] -> logits fp32
 * [batch, num_classes]. Asynchronous on `stream`. */
int evt_swin_forward(evt_model* model, const float* img, int batch, float* logits, void* stream);

/* Bytes of device workspace evt_swin_create allocates for `batch` images. */
int evt_swin_query_workspace(const evt_swin_desc* desc, int batch, size_t* bytes);

/* (Shifted-)window multi-head self-attention core of one Swin block (WindowAttention + the
 * cyclic shift / window partition / reverse around it): qkv [B*R*R, ldq] raster-order token rows
 * with columns (qkv h d) (the qkv Linear output incl. bias), head size 32, window 7, cyclic shift
 * `shift` (0 = W-MSA; else SW-MSA with the -100 region mask) -> out [B*R*R, ldo] raster rows,
 * columns (h d), columns [C, ldo) set to 0. rpb = relative_position_bias_table [169, H]. */
int evt_window_attention(int dtype, const void* qkv, int64_t ldq, void* out, int64_t ldo,
                         const float* rpb, int B, int R, int C, int H, int shift, void* stream);

/* PatchMerging gather: x [B, R, R, ldx] (C used) -> out [B*(R/2)^2, 4C] in the order
 * x[0::2,0::2] | x[1::2,0::2] | x[0::2,1::2] | x[1::2,1::2]; each row's (sum, sumsq) goes to slot
 * 0 of stats[row][nslots][2] (other slots zeroed). */
int evt_patch_merge(int dtype, const void* x, int64_t ldx, int B, int R, int C, void* out,
                    float* stats, int nslots, void* stream);

/* ---- MXFP8: the reduced-precision axis (reference utils.py:242-294 tf2tflite quantization
 * 'float16' / 'dynamic' / 'int8', tools.py:458-498) on the MI355X's block-scaled matrix cores.
 * An MX8 matrix [rows][K] is e4m3fn bytes q[rows][ldq] plus e8m0 scales, one per 32 consecutive K
 * of a row, stored k-step-major as dwords scales[K/128][ld_s] (ld_s >= rows; byte j of
 * scales[ks][r] is block 4*ks + j of row r): value = e4m3(q) * 2^(scale - 127). Quantization is
 * the OCP MX v1.0 rule (shared exponent floor(log2 amax) - 8, RNE, saturate to +-448). */
#define EVT_EPI_OUT_MX8 512 /* evt_dense_mx8: MX8 output (C bytes + c_scales), N % 32 == 0 */

/* rows x K activations (in_dtype EVT_DTYPE_F32 / _BF16, K % 8 == 0) -> MX8 [rows][Kpad]
 * (Kpad % 128 == 0, columns past K quantized as zeros). */
int evt_mx8_quantize(int in_dtype, const void* x, int64_t ldx, int rows, int K, int Kpad, void* q,
                     int64_t ldq, uint32_t* scales, int64_t ld_s, void* stream);

/* Keras Dense kernel W[K][N] fp32 (optionally row-scaled by row_scale[K]) -> packed MX8 weights
 * Wq[Npad][Kpad] (row n = output column n, K-contiguous) + scales[Kpad/128][Npad];
 * Kpad % 128 == 0, Npad % 128 == 0, padding quantized as zeros. */
int evt_mx8_pack_weight(const float* W, const float* row_scale, int K, int N, void* Wq, int Kpad,
                        int Npad, uint32_t* scales, void* stream);

typedef struct evt_dense_mx8_args {
  int32_t flags;                     /* EVT_EPI_BIAS | GELU | GELU_ERF | RESID | OUT_F32 | OUT_MX8 */
  const void* A; int64_t lda;        /* MX8 [M][Kpad] */
  const uint32_t* a_scales; int64_t ld_as;
  const void* Wq; int32_t Kpad; int32_t Npad;
  const uint32_t* w_scales;          /* [Kpad/128][Npad] */
  void* C; int64_t ldc;              /* bf16 (default) / fp32 / MX8 bytes */
  uint32_t* c_scales; int64_t ld_cs; /* EVT_EPI_OUT_MX8 */
  int32_t M, N;                      /* N % 8 == 0 */
  const float* bias;
  const void* resid; int64_t ldr;    /* bf16 */
  const float* rstats;               /* EVT_EPI_RESLN: [M][2] (mu, rstd) of the resid rows, as
                                        evt_mx8_layernorm writes them */
  const float* rgamma; const float* rbeta; /* EVT_EPI_RESLN: LayerNorm gamma / beta [N] */
} evt_dense_mx8_args;

/* Dense layer on MX8 operands (tf.keras.layers.Dense on the quantized model):
 * C = epi(dequant(A) . dequant(W)), fp32 accumulation; flag sets 0, 1, 3, 257, 5, 16, 17, 19,
 * 273, 512, 513, 515, 769, and 69 (bias + residual LN(resid) re-formed from rstats: the MX8
 * model's out-proj / FC2, reference norm.py:11-12 + residual.py:9). */
int evt_dense_mx8(const evt_dense_mx8_args* args, void* stream);

/* LayerNormalization(epsilon) of bf16 rows x [rows][D] (reference norm.py:6, population variance)
 * quantized straight to MX8: q [rows][Kpad] e4m3 (columns [D, Kpad) quantized as zeros), scales
 * [Kpad/128][rows] dwords, and, if stats != NULL, (mu, rstd) per row [rows][2] for a consumer's
 * EVT_EPI_RESLN. D % 8 == 0, D <= Kpad <= 1024, Kpad % 128 == 0. The MX8 model's LN1 / LN2. */
int evt_mx8_layernorm(const void* x, int rows, int D, int Kpad, const float* gamma,
                      const float* beta, float eps, float* stats, void* q, uint32_t* scales,
                      void* stream);

/* evt_attention (bf16 qkv, head size 64) with the output O written as MX8 instead of bf16:
 * q8 [B*N][ldq8] e4m3 (columns (h d)), scales s8[ldq8/128][ld_s8] dwords (ld_s8 >= B*N): the
 * MX8 model's out-proj operand (attention.py:20-35). ldq8 % 128 == 0, ldq8 >= 64*H. */
int evt_attention_mx8(const void* qkv, int64_t ldq, void* q8, int64_t ldq8, uint32_t* s8,
                      int64_t ld_s8, int B, int N, int H, float scale, void* stream);

/* ---- diagnostics (not part of the model contract) ---------------------------------------- */

/* GEMM kernel selection for bf16 Dense launches made FROM THE CALLING THREAD (thread-local: other
 * threads and their handles are unaffected), for parity tests and A/B measurements only:
 * 0 = automatic (the persistent 256x256 kernel unless its tile rounds cost more than the 128x128
 * kernel's, else 128x128), 1 = always 128x128, 2 / 6 / 8 = non-persistent 256x256 tiles with the
 * plain / interleaved / 8-phase ping-pong main loop whenever the packed width allows, 9 =
 * tile-persistent, 16 = stream-K persistent where it applies, 30 = the 128 x 384 persistent tiles
 * wherever the width allows (multiple of 384), 31 = automatic without them, 36 = automatic with the
 * persistent grids at one block per CU (no balancing of 2-4-round launches to fewer blocks: the
 * same tiles and arithmetic, bitwise the same outputs). Builds with
 * EVT_LAB=1 (-DEVT_GEMM_LAB) also accept the ablation / timeline variants 10, 11, 13, 15, 17-25,
 * 106, 108; other values return EVT_EINVAL. */
int evt_set_gemm_variant(int variant);

/* Number of encoder layers whose QKV GEMM stored its output head-major ([B][H][q | k | v][T][64],
 * the persistent kernel's EPI_HM store) in the handle's last forward; 0 when every layer kept the
 * token-major (qkv h d) columns of attention.py:20 (EVT_QKV_LAYOUT=token, f32, head size != 64 or
 * a problem the persistent kernel does not take). Lets the layout-equality tests assert which
 * path ran. */
int evt_model_qkv_layout(const evt_model* m, int* headmajor_layers);

#ifdef __cplusplus
}
#endif
#endif /* EVT_H_ */
