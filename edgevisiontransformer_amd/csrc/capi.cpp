// C ABI of libevt_hip.so (declared in include/evt.h): model plumbing around the HIP kernels.
//
// The model handle owns the packed weights (kernel operand layout, zero padded, LayerNorm gamma
// folded in) and one workspace sized for max_batch; evt_vit_forward enqueues the whole ViT
// forward of reference `modeling/models/vit.py:41-55` on the caller's stream with no host
// synchronisation. Per encoder layer (transformer_encoder.py:13-18):
//
//   QKV GEMM   A = x (raw stream), epilogue applies LN1 per row        (attention.py:24 + norm.py:12)
//   attention  fused softmax(q k^T * 64^-0.5) v                        (attention.py:20-34)
//   out GEMM   + bias + LN1(x) residual -> xm, row stats of xm         (attention.py:35, residual.py:9)
//   FC1 GEMM   A = xm, epilogue applies LN2 per row, + bias, GELU      (ffn.py:8)
//   FC2 GEMM   + bias + LN2(xm) residual -> x, row stats of x          (ffn.py:9, residual.py:9)
//
// Row statistics (sum, sum of squares) are written by the producing GEMM's epilogue as one partial
// per 128-column slab (stats slot) with plain stores; consumers sum the slots in a fixed order, so
// the forward is bitwise reproducible and needs no memsets.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/evt.h"
#include "evt_internal.h"

using namespace evt;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(EVT_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define EVT_HIP(call, what)                            \
  do {                                                 \
    hipError_t e__ = (call);                           \
    if (e__ != hipSuccess) return hip_fail(e__, what); \
  } while (0)

#define EVT_RC(x)          \
  do {                     \
    int rc__ = (x);        \
    if (rc__) return rc__; \
  } while (0)

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
inline size_t elem_size(int dtype) { return dtype == DT_BF16 ? 2 : 4; }

struct DenseW {  // packed Dense layer
  void* w = nullptr;        // [npad][kpad] activation dtype
  float* b = nullptr;       // [npad] fp32, zero padded (bias, or the LN-fold vector c)
  float* colsum = nullptr;  // [npad] LN fold: column sums of the packed weights (or null)
  int K = 0, N = 0, kpad = 0, npad = 0;
};

struct Mx8W {  // MXFP8-packed Dense layer (mx8.hip): Wq [npad][kpad] e4m3, scales [kpad/128][npad]
  void* w = nullptr;
  uint32_t* s = nullptr;
  float* b = nullptr;       // [npad] fp32 bias, zero padded (zeros for the bias-less QKV)
  int K = 0, N = 0, kpad = 0, npad = 0;
};

struct Layer {
  int heads = 0, hd = 64, inner = 0, ffn = 0, ffn_st = 0;
  float *ln1_g = nullptr, *ln1_b = nullptr, *ln2_g = nullptr, *ln2_b = nullptr;
  DenseW qkv, out, fc1, fc2;
  Mx8W mqkv, mout, mfc1, mfc2;  // EVT_DTYPE_MX8 models
};

struct Shape {
  int P = 0, T = 0, pd = 0, D = 0, max_inner = 0, max_ffn_st = 0, head_st = 0;
};

}  // namespace

struct Performer {  // one TokenPerformer (transformer_encoder.py:39-101)
  int din = 0, dpad = 0;     // unfolded input width, padded to PAD_K
  DenseW kqv;                // LN1-folded Dense(3*64) + bias
  PerformerWeights w{};      // fp32 device copies (Keras layouts)
};

struct SwinBlock {  // one Swin block (microsoft SwinTransformerBlock)
  int shift = 0;
  float* bias = nullptr;     // [H][49][64] dense relative position bias (* log2 e)
  DenseW qkv, proj, fc1, fc2;
};

struct SwinStage {
  int C = 0, Cst = 0, H = 0, R = 0, mlp = 0, mst = 0;
  DenseW merge;              // LN(4C)-folded reduction Linear(4C, 2C, bias=False) (stage > 0)
  std::vector<SwinBlock> blocks;
};

// EVT_QKV_LAYOUT=token (read when a model is created): keep the token-major qkv layout
static bool qkv_headmajor_default() {
  const char* e = std::getenv("EVT_QKV_LAYOUT");
  return !(e && std::strcmp(e, "token") == 0);
}

struct evt_model {
  int family = 0;            // 0: ViT / ViT_Pruned, 1: T2T-ViT, 2: Swin
  bool standard = false;     // ViT with EVT_VIT_STANDARD semantics
  bool mx8 = false;          // EVT_DTYPE_MX8: MXFP8 encoder Dense layers (dtype is then bf16)
  // QKV output head-major where the GEMM supports it (run_encoder); EVT_QKV_LAYOUT=token at model
  // creation keeps the token-major layout (the A/B and bitwise-equality tests)
  bool headmajor = qkv_headmajor_default();
  int hm_layers = 0;         // encoder layers whose QKV stored head-major in the last forward
  bool patch_cm = false;     // ViT: channel-major patch vectors / patch weight rows
  void* qa = nullptr;        // MX8: [rows][max(Dpad, innerpad)] e4m3 A operand (LN out / attn out)
  uint32_t* sa = nullptr;    // MX8: its scales [pad/128][rows]
  void* qh = nullptr;        // MX8: [rows][ffnpad] FC1 output (e4m3, zero-initialised)
  uint32_t* shd = nullptr;   // MX8: its scales
  float* lnst = nullptr;     // MX8: [rows][2] (mu, rstd) of the last LayerNorm'd rows
  int qa_ld = 0, qh_ld = 0;
  float eps = 1e-5f;         // LayerNorm epsilon of every folded LayerNorm
  int dtype = 0, D = 0, max_batch = 0, num_classes = 0;
  evt_vit_desc desc{};       // ViT only
  evt_t2t_desc tdesc{};      // T2T only
  std::vector<int32_t> heads, head_dim, ffn;
  Shape sh;
  DenseW patch, head1, head2;
  float *cls = nullptr, *pos = nullptr;
  void* pos_h = nullptr;     // bf16 copy of pos (the persistent patch-embedding GEMM's EPI_POS)
  std::vector<Layer> layers;
  std::vector<void*> allocs;
  // T2T stage
  Performer perf[2];
  DenseW project, head;      // head: LN-folded classifier (final LayerNorm, t2t_vit.py:129,134)
  int grid[3] = {0, 0, 0};   // token grids S/4, S/8, S/16
  void* u = nullptr;         // unfold output (GEMM A operand)
  float* su = nullptr;       // unfold row statistics
  void* kqvb = nullptr;      // [B*T1, 192]
  void* pout = nullptr;      // [B*T1, 64] performer output (NHWC for the next unfold)
  float* tstats = nullptr;   // [B*T1, 2] per-token (sum, sumsq) of pout (gathered soft split)
  void* zrow = nullptr;      // 256 zero bytes: the soft split's padding rows (gathered loader)
  float* part = nullptr;     // performer partial sums
  // workspace (activation dtype unless noted)
  void* apatch = nullptr;    // [B*P, pd] patch matrix (aliases hbuf)
  void* x = nullptr;         // [B*T, D] token stream at layer input / output
  void* xm = nullptr;        // [B*T, D] token stream between the two sublayers
  float* sx = nullptr;       // [B*T, nslots, 2] fp32 per-slab (sum, sumsq) of x rows
  float* sm = nullptr;       // [B*T, nslots, 2] fp32 per-slab (sum, sumsq) of xm rows
  void* qkv = nullptr;       // [B*T, 3*inner]
  void* o = nullptr;         // [B*T, inner]
  void* hbuf = nullptr;      // [B*T, ffn_st]
  size_t hbuf_bytes = 0;
  void* hh = nullptr;        // [B, head_st]
  void* sk = nullptr;        // stream-K scratch of the model's GEMMs (gemm_sk_bytes)
  // Swin (family 2)
  evt_swin_desc sdesc{};
  std::vector<SwinStage> stages;
  float *pnorm_g = nullptr, *pnorm_b = nullptr, *norm_g = nullptr, *norm_b = nullptr;
  void* pooled = nullptr;    // [B, Cst_last] LayerNorm + token mean (head A operand)
  size_t ws_bytes = 0;
  hipGraph_t graph = nullptr;        // evt_graph_capture
  hipGraphExec_t graph_exec = nullptr;
  // evt_model_profile: HIP events around every launch of the last forward, by role
  bool prof = false;
  std::vector<hipEvent_t> prof_ev;   // pool (pairs)
  std::vector<int> prof_role;        // role of pair i of the last forward
  // algorithmic work of pair i (evt_model_profile_work): GFLOP and GB its kernels must do / move
  mutable std::vector<double> prof_gflop, prof_gbytes;
  // evt_model_set_lanes: the batch split over k lanes, each a child model with its own workspace
  // (the weights are this model's) on its own HIP stream, forked from / joined to the caller's
  // stream by events; the kernels of the lanes then fill each other's idle CUs
  std::vector<evt_model*> lanes;
  std::vector<hipStream_t> lane_s;
  std::vector<char> lane_own;        // lane_s[i] created (and destroyed) by the library
  std::vector<hipEvent_t> lane_ev;   // [0]: fork, [1 + i]: lane i done
  bool is_lane = false;              // a child: weights and lanes belong to the parent
  // T2T-ViT lanes: their persistent GEMMs keep one block per CU at 2-4 tile rounds (the other
  // lane fills the CUs a balanced grid leaves idle; measured +2.9 % on T2T-ViT-14 bs256, while
  // Swin lanes measured -1.3 % without the balancing: DESIGN.md, batch lanes)
  int no_balance = 0;
};

namespace {


// evt_model_profile: a pair of events around each launch of a forward (profiling forwards only)
struct ProfScope {
  evt_model* m;
  hipStream_t s;
  int pair = -1;
  ProfScope(evt_model* m_, int role, hipStream_t s_) : m(m_), s(s_) {
    if (!m->prof) return;
    pair = (int)m->prof_role.size();
    while ((int)m->prof_ev.size() < 2 * (pair + 1)) {
      hipEvent_t e = nullptr;
      if (hipEventCreate(&e) != hipSuccess) {
        pair = -1;
        return;
      }
      m->prof_ev.push_back(e);
    }
    m->prof_role.push_back(role);
    m->prof_gflop.push_back(0.0);
    m->prof_gbytes.push_back(0.0);
    (void)hipEventRecord(m->prof_ev[2 * pair], s);
  }
  ~ProfScope() {
    if (pair >= 0) (void)hipEventRecord(m->prof_ev[2 * pair + 1], s);
  }
};
void prof_reset(evt_model* m) {
  if (!m->prof) return;
  m->prof_role.clear();
  m->prof_gflop.clear();
  m->prof_gbytes.clear();
}
// add algorithmic work (flops, bytes) to the innermost open ProfScope of a profiled forward
void prof_work(const evt_model* m, double flops, double bytes) {
  if (!m->prof || m->prof_gflop.empty()) return;
  m->prof_gflop.back() += flops * 1e-9;
  m->prof_gbytes.back() += bytes * 1e-9;
}

int dev_alloc(evt_model* m, void** p, size_t bytes) {
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess)
    return fail(EVT_ENOMEM, std::string("hipMalloc failed: ") + hipGetErrorString(e));
  m->allocs.push_back(*p);
  return EVT_OK;
}

int validate(const evt_vit_desc* d, Shape* sh) {
  if (!d) return fail(EVT_EINVAL, "desc is NULL");
  if (d->dtype != EVT_DTYPE_F32 && d->dtype != EVT_DTYPE_BF16 && d->dtype != EVT_DTYPE_MX8)
    return fail(EVT_EINVAL, "dtype must be EVT_DTYPE_F32, EVT_DTYPE_BF16 or EVT_DTYPE_MX8");
  if (d->dtype == EVT_DTYPE_MX8 && d->semantics != EVT_VIT_REFERENCE)
    return fail(EVT_EINVAL, "EVT_DTYPE_MX8 supports EVT_VIT_REFERENCE semantics only");
  if (d->patch_size <= 0 || d->image_size <= 0 || d->image_size % d->patch_size != 0)
    return fail(EVT_EINVAL, "image dimensions must be divisible by the patch size");
  if (d->in_chans <= 0 || d->num_classes <= 0 || d->depth < 0 || d->mlp_dim <= 0)
    return fail(EVT_EINVAL, "in_chans, num_classes, mlp_dim must be positive, depth >= 0");
  if (d->dim <= 0 || d->dim % 8 != 0 || d->dim > 1024)
    return fail(EVT_EINVAL, "dim must be a positive multiple of 8 and <= 1024");
  if (d->dtype == EVT_DTYPE_MX8 && d->dim % 64 != 0)
    return fail(EVT_EINVAL, "EVT_DTYPE_MX8 needs dim % 64 == 0");
  if (d->max_batch <= 0) return fail(EVT_EINVAL, "max_batch must be positive");
  if (d->semantics != EVT_VIT_REFERENCE && d->semantics != EVT_VIT_STANDARD)
    return fail(EVT_EINVAL, "semantics must be EVT_VIT_REFERENCE or EVT_VIT_STANDARD");
  if (d->layer_norm_eps < 0.f) return fail(EVT_EINVAL, "layer_norm_eps must be >= 0");
  if (d->depth > 0 && (!d->heads || !d->head_dim || !d->ffn))
    return fail(EVT_EINVAL, "heads/head_dim/ffn arrays are required");
  const int np = d->image_size / d->patch_size;
  sh->P = np * np;
  sh->T = sh->P + 1;
  if (sh->T > 256) return fail(EVT_EINVAL, "at most 255 patches per image are supported");
  sh->pd = d->patch_size * d->patch_size * d->in_chans;
  if (sh->pd % PAD_K) return fail(EVT_EINVAL, "patch_size^2 * in_chans must be a multiple of 64");
  if (d->patch_size * d->image_size % 4)
    return fail(EVT_EINVAL, "patch_size * image_size must be a multiple of 4");
  if ((size_t)d->in_chans * d->patch_size * d->image_size * 4 > 160 * 1024)
    return fail(EVT_EINVAL, "image strip exceeds LDS");
  sh->D = d->dim;
  sh->max_inner = 0;
  sh->max_ffn_st = 0;
  for (int i = 0; i < d->depth; ++i) {
    if (d->heads[i] <= 0) return fail(EVT_EINVAL, "heads per layer must be positive");
    // any h_k (attention.py:6-12) up to 128; 64 runs the tuned kernels, others the generic ones
    if (d->head_dim[i] <= 0 || d->head_dim[i] > 128)
      return fail(EVT_EINVAL, "head size must be in [1, 128]");
    if (d->heads[i] * d->head_dim[i] % 8)
      return fail(EVT_EINVAL, "heads * head size must be a multiple of 8 (16-B token rows)");
    if (d->dtype == EVT_DTYPE_MX8 && d->head_dim[i] != 64)
      return fail(EVT_EINVAL, "EVT_DTYPE_MX8 supports head size 64 only");
    if (d->ffn[i] <= 0) return fail(EVT_EINVAL, "ffn width per layer must be positive");
    sh->max_inner = std::max(sh->max_inner, d->heads[i] * d->head_dim[i]);
    sh->max_ffn_st = std::max<int>(sh->max_ffn_st, (int)round_up(d->ffn[i], PAD_N));
  }
  sh->head_st = (int)round_up(d->mlp_dim, PAD_N);
  return EVT_OK;
}

// Pack a Keras [K, N] Dense kernel. With ln_g/ln_b (the LayerNorm in front of it), gamma is folded
// into the weight rows and b becomes c = beta . W + bias, with the column sums of the packed
// weights alongside (gemm.hip, "LayerNorm folding").
int make_dense(evt_model* m, DenseW* dw, const float* W, const float* bias, int K, int N,
               hipStream_t s, const float* ln_g = nullptr, const float* ln_b = nullptr) {
  const int dt = m->dtype;
  dw->K = K;
  dw->N = N;
  dw->kpad = (int)round_up(K, PAD_K);
  dw->npad = (int)round_up(N, PACK_N);
  EVT_RC(dev_alloc(m, &dw->w, (size_t)dw->kpad * dw->npad * elem_size(dt)));
  EVT_HIP(pack_weight(dt, W, ln_g, K, N, dw->w, dw->kpad, dw->npad, s), "pack_weight");
  if (ln_g) {
    EVT_RC(dev_alloc(m, (void**)&dw->b, (size_t)dw->npad * sizeof(float)));
    EVT_RC(dev_alloc(m, (void**)&dw->colsum, (size_t)dw->npad * sizeof(float)));
    EVT_HIP(ln_fold(dt, dw->w, dw->kpad, W, ln_b, bias, K, N, dw->colsum, dw->b, dw->npad, s),
            "ln_fold");
  } else if (bias) {
    EVT_RC(dev_alloc(m, (void**)&dw->b, (size_t)dw->npad * sizeof(float)));
    EVT_HIP(hipMemsetAsync(dw->b, 0, (size_t)dw->npad * sizeof(float), s), "memset bias");
    EVT_HIP(hipMemcpyAsync(dw->b, bias, (size_t)N * sizeof(float), hipMemcpyDeviceToDevice, s),
            "copy bias");
  }
  return EVT_OK;
}

int copy_vec(evt_model* m, float** dst, const float* src, size_t n, hipStream_t s) {
  EVT_RC(dev_alloc(m, (void**)dst, n * sizeof(float)));
  EVT_HIP(hipMemcpyAsync(*dst, src, n * sizeof(float), hipMemcpyDeviceToDevice, s), "copy vec");
  return EVT_OK;
}

// Pack a Keras [K, N] Dense kernel to MXFP8 (no LayerNorm folding: the MX8 model normalises in
// the quantizer). N is padded to 32 columns of zeros so an MX8 output covers whole blocks.
int make_mx8(evt_model* m, Mx8W* dw, const float* W, const float* bias, int K, int N,
             hipStream_t s) {
  dw->K = K;
  dw->N = (int)round_up(N, 32);
  dw->kpad = (int)round_up(K, 128);
  dw->npad = (int)round_up(N, 128);
  EVT_RC(dev_alloc(m, &dw->w, (size_t)dw->kpad * dw->npad));
  EVT_RC(dev_alloc(m, (void**)&dw->s, (size_t)dw->kpad / 128 * dw->npad * 4));
  EVT_HIP(mx8_pack_launch(W, nullptr, K, N, dw->w, dw->kpad, dw->npad, dw->s, s), "mx8_pack");
  EVT_RC(dev_alloc(m, (void**)&dw->b, (size_t)dw->npad * sizeof(float)));
  EVT_HIP(hipMemsetAsync(dw->b, 0, (size_t)dw->npad * sizeof(float), s), "memset bias");
  if (bias)
    EVT_HIP(hipMemcpyAsync(dw->b, bias, (size_t)N * sizeof(float), hipMemcpyDeviceToDevice, s),
            "copy bias");
  return EVT_OK;
}

int dense_mx8(const Mx8W& w, int flags, const void* A, int64_t lda, const uint32_t* as, void* C,
              int64_t ldc, uint32_t* cs, int M, const void* resid, int64_t ldr, hipStream_t s,
              const float* rstats = nullptr, const float* rgamma = nullptr,
              const float* rbeta = nullptr) {
  Mx8GemmParams p{};
  p.A = (const uint8_t*)A; p.lda = lda; p.As = as; p.ldas = M;
  p.W = (const uint8_t*)w.w; p.ldw = w.kpad; p.Ws = w.s; p.ldws = w.npad;
  p.C = C; p.ldc = ldc; p.Cs = cs; p.ldcs = M;
  p.M = M; p.N = w.N; p.K = w.kpad;
  p.bias = w.b; p.resid = resid; p.ldr = ldr;
  p.rstats = rstats; p.rgamma = rgamma; p.rbeta = rbeta;
  EVT_HIP(gemm_mx8_launch(flags, p, s), "dense_mx8");
  return EVT_OK;
}

size_t workspace_bytes(const evt_vit_desc* d, const Shape& sh, int B) {
  const bool mx8 = d->dtype == EVT_DTYPE_MX8;
  const size_t es = elem_size(mx8 ? DT_BF16 : d->dtype);
  const size_t rows = (size_t)B * sh.T;
  const size_t hb = std::max(rows * sh.max_ffn_st, (size_t)B * sh.P * sh.pd) * es;
  size_t extra = 0;
  if (mx8) {  // qa + sa, qh + its scales, LayerNorm row statistics (run_encoder_mx8)
    const size_t qa = std::max(round_up(sh.D, 128), round_up(sh.max_inner, 128));
    int maxffn = 0;
    for (int i = 0; i < d->depth; ++i) maxffn = std::max(maxffn, (int)d->ffn[i]);
    const size_t qh = round_up(maxffn, 128);
    extra = rows * (qa + qa / 32 + qh + qh / 32 + 2 * sizeof(float)) + 5 * 256;
  }
  return 2 * rows * sh.D * es + 2 * rows * stats_slots(sh.D) * 2 * sizeof(float) +
         rows * 3 * sh.max_inner * es +
         rows * sh.max_inner * es + hb + (size_t)B * sh.head_st * es + 9 * 256 + extra;
}

struct DenseCall {
  int flags = 0;
  const void* A = nullptr;
  int64_t lda = 0;
  void* C = nullptr;
  int64_t ldc = 0;
  int M = 0, N = 0;
  const void* resid = nullptr;
  int64_t ldr = 0;
  const float* pos = nullptr;
  int64_t ldp = 0;
  int P = 0;
  const float* stats_in = nullptr;
  const float* rstats = nullptr;
  const float* rgamma = nullptr;
  const float* rbeta = nullptr;
  float* stats_out = nullptr;
  int ln_width = 0;    // LayerNorm width of stats_in / rstats / stats_out (0: the model width D)
  int stats_step = 1;  // EPI_LNIN: A row m reads stats_in row m * stats_step
  int slot_width = 0;  // width whose stats_slots() numbers the slots (0: ln_width)
};

// Algorithmic work of one Dense launch: 2 M K N with the layer's real K and N; bytes = A and W
// read once, C written once, plus the residual, the row statistics read / written and the small
// bias / position vectors (what the kernel cannot avoid moving).
void dense_work(const evt_model* m, const DenseW& w, const DenseCall& c) {
  if (!m->prof) return;
  const double es = (double)elem_size(m->dtype);
  const double M = c.M, K = w.K, N = std::min(c.N, w.N);
  const int width = c.ln_width ? c.ln_width : m->D;
  const double slot_row = (double)stats_slots(c.slot_width ? c.slot_width : width) * 8.0;
  double bytes = M * K * es + K * N * es + M * N * ((c.flags & EPI_OUT_F32) ? 4.0 : es) + 8.0 * N;
  if (c.flags & EPI_RESID) bytes += M * N * es;
  if (c.flags & EPI_LNIN) bytes += M * slot_row;
  if (c.flags & EPI_RESLN) bytes += M * slot_row + 8.0 * N;
  if (c.flags & EPI_STATS) bytes += M * slot_row;
  if (c.flags & EPI_POS) bytes += (double)(c.P + 1) * N * 4.0;
  prof_work(m, 2.0 * M * K * N, bytes);
}

GemmParams dense_params(const evt_model* m, const DenseW& w, const DenseCall& c) {
  GemmParams p{};
  p.A = c.A;
  p.lda = c.lda;
  p.W = w.w;
  p.ldw = w.kpad;
  p.C = c.C;
  p.ldc = c.ldc;
  p.M = c.M;
  p.N = c.N;
  p.K = w.kpad;
  p.ntiles = w.npad / GEMM_BN;
  p.bias = w.b;
  p.resid = c.resid;
  p.ldr = c.ldr;
  p.pos = c.pos;
  p.ldp = c.ldp;
  p.P = c.P;
  p.vec_ok = (c.ldc % 4 == 0) && (c.ldr % 4 == 0) && (c.ldp % 4 == 0);
  if (p.vec_ok && c.ldc % 8 == 0 && c.ldr % 8 == 0 && c.ldp % 8 == 0 &&
      (((uintptr_t)c.C | (uintptr_t)c.resid) & 15) == 0)
    p.vec_ok = 2;
  p.colsum = w.colsum;
  p.no_balance = m->no_balance;
  p.stats_in = c.stats_in;
  p.rstats = c.rstats;
  p.rgamma = c.rgamma;
  p.rbeta = c.rbeta;
  p.stats_out = c.stats_out;
  const int width = c.ln_width ? c.ln_width : m->D;
  p.inv_d = 1.0f / (float)width;
  p.eps = m->eps;  // Keras LayerNormalization(epsilon=1e-5), reference norm.py:6
  p.nslots = stats_slots(c.slot_width ? c.slot_width : width);
  p.stats_step = c.stats_step;
  gemm_sk_bind(m->sk, p);
  return p;
}

int dense(const evt_model* m, const DenseW& w, const DenseCall& c, hipStream_t s) {
  dense_work(m, w, c);
  const GemmParams p = dense_params(m, w, c);
  EVT_HIP(gemm_launch(m->dtype, c.flags, p, s), "dense");
  return EVT_OK;
}

// Encoder weights (11 tensors per layer, 12 with the STANDARD qkv bias; evt_vit_num_weights
// order) for m->heads / m->ffn.
int build_encoder(evt_model* m, const float* const* w, hipStream_t s) {
  const int D = m->D;
  const int depth = (int)m->heads.size();
  const int qb = m->standard ? 1 : 0;  // qkv bias present
  m->layers.resize(depth);
  int k = 0;
  for (int i = 0; i < depth; ++i) {
    Layer& L = m->layers[i];
    L.heads = m->heads[i];
    L.hd = m->head_dim[i];
    L.inner = L.heads * L.hd;
    L.ffn = m->ffn[i];
    L.ffn_st = (int)round_up(L.ffn, PAD_N);
    EVT_RC(copy_vec(m, &L.ln1_g, w[k + 0], D, s));
    EVT_RC(copy_vec(m, &L.ln1_b, w[k + 1], D, s));
    if (m->mx8) {  // reference semantics only (validate): no qkv bias
      EVT_RC(copy_vec(m, &L.ln2_g, w[k + 5], D, s));
      EVT_RC(copy_vec(m, &L.ln2_b, w[k + 6], D, s));
      EVT_RC(make_mx8(m, &L.mqkv, w[k + 2], nullptr, D, 3 * L.inner, s));
      EVT_RC(make_mx8(m, &L.mout, w[k + 3], w[k + 4], L.inner, D, s));
      EVT_RC(make_mx8(m, &L.mfc1, w[k + 7], w[k + 8], D, L.ffn, s));
      EVT_RC(make_mx8(m, &L.mfc2, w[k + 9], w[k + 10], L.ffn, D, s));
      k += 11;
      continue;
    }
    EVT_RC(make_dense(m, &L.qkv, w[k + 2], qb ? w[k + 3] : nullptr, D, 3 * L.inner, s, w[k + 0],
                      w[k + 1]));
    k += qb;
    EVT_RC(make_dense(m, &L.out, w[k + 3], w[k + 4], L.inner, D, s));
    EVT_RC(copy_vec(m, &L.ln2_g, w[k + 5], D, s));
    EVT_RC(copy_vec(m, &L.ln2_b, w[k + 6], D, s));
    EVT_RC(make_dense(m, &L.fc1, w[k + 7], w[k + 8], D, L.ffn, s, w[k + 5], w[k + 6]));
    EVT_RC(make_dense(m, &L.fc2, w[k + 9], w[k + 10], L.ffn, D, s));
    k += 11;
  }
  return EVT_OK;
}

// Token-stream workspace of the encoder for B images (hbuf_bytes: the FFN hidden buffer), and the
// stream-K scratch of the model's GEMMs (its flag block zeroed once; kernels leave it zeroed).
int alloc_encoder_ws(evt_model* m, int B, size_t hbuf_bytes, hipStream_t s) {
  const size_t es = elem_size(m->dtype);
  if (m->dtype == DT_BF16) {
    EVT_RC(dev_alloc(m, &m->sk, gemm_sk_bytes()));
    EVT_HIP(hipMemsetAsync(m->sk, 0, 4096, s), "memset stream-K flags");
  }
  const size_t rows = (size_t)B * m->sh.T;
  // x, xm (width D) and o (width heads * h_k) are GEMM A operands read in 64-column K-tiles: with
  // a width that is not a multiple of 64 a row's last K-tile runs into the next row (cancelled by
  // the zero-padded weight rows) and the last row into PAD_K zeroed slack elements; every byte is
  // zeroed once here (finite everywhere)
  const size_t xb = (rows * m->D + PAD_K) * es, ob = (rows * m->sh.max_inner + PAD_K) * es;
  EVT_RC(dev_alloc(m, &m->x, xb));
  EVT_RC(dev_alloc(m, &m->xm, xb));
  const size_t stats_bytes = rows * stats_slots(m->D) * 2 * sizeof(float);
  EVT_RC(dev_alloc(m, (void**)&m->sx, stats_bytes));
  EVT_RC(dev_alloc(m, (void**)&m->sm, stats_bytes));
  EVT_RC(dev_alloc(m, &m->qkv, rows * 3 * m->sh.max_inner * es));
  EVT_RC(dev_alloc(m, &m->o, ob));
  EVT_HIP(hipMemsetAsync(m->x, 0, xb, s), "memset x");
  EVT_HIP(hipMemsetAsync(m->xm, 0, xb, s), "memset xm");
  EVT_HIP(hipMemsetAsync(m->o, 0, ob, s), "memset o");
  EVT_RC(dev_alloc(m, &m->hbuf, hbuf_bytes));
  m->hbuf_bytes = hbuf_bytes;
  return EVT_OK;
}

// Small-M, long-K Dense layers (the classifier head: M = batch) as K splits in one launch when the
// plain tile grid would leave most CUs idle; fp32 partials in the (then idle) hidden buffer.
int dense_head(const evt_model* m, const DenseW& w, const DenseCall& c, hipStream_t s) {
  const int tiles = ((c.M + GEMM_BM - 1) / GEMM_BM) * (w.npad / GEMM_BN);
  int S = 1;
  while (S < 8 && tiles * S * 2 <= device_cus() && w.kpad % (S * 2 * PAD_K) == 0) S *= 2;
  const size_t part = (size_t)S * c.M * w.npad * sizeof(float);
  if (S < 2 || !m->hbuf || part > m->hbuf_bytes ||
      (c.flags & ~(EPI_BIAS | EPI_GELU | EPI_OUT_F32)))
    return dense(m, w, c, s);
  dense_work(m, w, c);
  GemmParams p{};
  p.A = c.A; p.lda = c.lda; p.W = w.w; p.ldw = w.kpad; p.C = c.C; p.ldc = c.ldc;
  p.M = c.M; p.N = c.N; p.K = w.kpad; p.ntiles = w.npad / GEMM_BN; p.bias = w.b;
  EVT_HIP(gemm_splitk_launch(m->dtype, c.flags, p, S, (float*)m->hbuf, s), "dense (split-K)");
  return EVT_OK;
}

// Encoder layers (transformer_encoder.py:13-18 / :26-34) on the token stream m->x (+ stats sx).
int run_encoder(evt_model* m, int B, hipStream_t s) {
  const int D = m->D, T = m->sh.T, rows = B * T;
  const float log2e = 1.4426950408889634f;
  m->hm_layers = 0;
  for (const Layer& L : m->layers) {
    const float scale_log2 = log2e / std::sqrt((float)L.hd);  // h_k^-0.5 (attention.py:13)
    // qkv head-major ([B][heads][q | k | v][T][64], EPI_HM) where the QKV GEMM takes the
    // persistent kernel (h_k = 64, bf16): an (image, head)'s q, k and v are three contiguous 25 KB
    // runs instead of T 128-B pieces at a 3 D-element stride each; token-major otherwise
    bool hm = false;
    {  // LN1-folded QKV (attention.py:24)
      ProfScope ps(m, EVT_PROF_QKV, s);
      DenseCall c;
      c.flags = EPI_LNIN | EPI_BIAS;
      c.A = m->x; c.lda = D; c.C = m->qkv; c.ldc = 3 * L.inner; c.M = rows; c.N = 3 * L.inner;
      c.stats_in = m->sx;
      if (L.hd == 64 && m->headmajor) {
        DenseCall h = c;
        h.flags |= EPI_HM;
        h.ldc = 64;
        h.P = T;
        if (gemm_headmajor_ok(m->dtype, h.flags, dense_params(m, L.qkv, h))) {
          c = h;
          hm = true;
          ++m->hm_layers;
        }
      }
      EVT_RC(dense(m, L.qkv, c, s));
    }
    {
      ProfScope ps(m, EVT_PROF_ATTENTION, s);
      prof_work(m, 4.0 * B * L.heads * (double)T * T * L.hd,
                (double)rows * 4 * L.inner * elem_size(m->dtype));  // qkv read + O written
      AttnParams ap{m->qkv, 3 * L.inner, m->o, L.inner, T, L.heads, B, scale_log2};
      ap.hd = L.hd;
      if (hm) {
        ap.ldq = 64;
        ap.sb = (int64_t)L.heads * 3 * T * 64;
        ap.sh = (int64_t)3 * T * 64;
        ap.ko = T * 64;
        ap.vo = 2 * T * 64;
      }
      EVT_HIP(attention_launch(m->dtype, ap, s), "attention");
    }
    // out-proj + bias + LN1(x) residual -> xm (+ stats); STANDARD: + x
    DenseCall co;
    co.flags = m->standard ? (EPI_BIAS | EPI_RESID | EPI_STATS)
                           : (EPI_BIAS | EPI_RESID | EPI_RESLN | EPI_STATS);
    co.A = m->o; co.lda = L.inner; co.C = m->xm; co.ldc = D; co.M = rows; co.N = D;
    co.resid = m->x; co.ldr = D; co.rstats = m->sx; co.rgamma = L.ln1_g; co.rbeta = L.ln1_b;
    co.stats_out = m->sm;
    // LN2-folded FC1 + GELU (ffn.py:8; STANDARD: exact erf GELU)
    DenseCall c1;
    c1.flags = EPI_LNIN | EPI_BIAS | (m->standard ? EPI_GELU_ERF : EPI_GELU);
    c1.A = m->xm; c1.lda = D; c1.C = m->hbuf; c1.ldc = L.ffn_st; c1.M = rows; c1.N = L.ffn_st;
    c1.stats_in = m->sm;
    {
      ProfScope ps(m, EVT_PROF_OUT_PROJ, s);
      EVT_RC(dense(m, L.out, co, s));
    }
    {
      ProfScope ps(m, EVT_PROF_FC1, s);
      EVT_RC(dense(m, L.fc1, c1, s));
    }
    {  // FC2 + bias + LN2(xm) residual -> x (+ stats); STANDARD: + xm
      ProfScope ps(m, EVT_PROF_FC2, s);
      DenseCall c;
      c.flags = m->standard ? (EPI_BIAS | EPI_RESID | EPI_STATS)
                            : (EPI_BIAS | EPI_RESID | EPI_RESLN | EPI_STATS);
      c.A = m->hbuf; c.lda = L.ffn_st; c.C = m->x; c.ldc = D; c.M = rows; c.N = D;
      c.resid = m->xm; c.ldr = D; c.rstats = m->sm; c.rgamma = L.ln2_g; c.rbeta = L.ln2_b;
      c.stats_out = m->sx;
      EVT_RC(dense(m, L.fc2, c, s));
    }
  }
  return EVT_OK;
}

// MX8 encoder (reference semantics, transformer_encoder.py:13-18): per sublayer the LayerNorm
// runs in the quantizer (which keeps each row's (mu, rstd)), the Dense layers on the block-scaled
// MFMA, the residual LN(x) (norm.py:11-12 + residual.py:9) re-formed in the out-proj / FC2
// epilogues from x and those statistics; the attention and FC1 (GELU) outputs are quantized in
// their producing kernels' epilogues.
int run_encoder_mx8(evt_model* m, int B, hipStream_t s) {
  const int D = m->D, T = m->sh.T, rows = B * T;
  const float log2e = 1.4426950408889634f;
  const int dpad = (int)round_up(D, 128);
  for (const Layer& L : m->layers) {
    EVT_HIP(ln_mx8_launch(m->x, rows, D, dpad, L.ln1_g, L.ln1_b, m->eps, m->lnst, m->qa, m->sa, s),
            "ln1 mx8");
    EVT_RC(dense_mx8(L.mqkv, EPI_BIAS, m->qa, dpad, m->sa, m->qkv, 3 * L.inner, nullptr, rows,
                     nullptr, 0, s));
    // attention writes O straight as the MX8 operand of the out-proj (columns [inner, ipad) of
    // qa keep finite stale values, cancelled by the zero rows of the packed weights)
    const int ipad = L.mout.kpad;
    AttnParams ap{m->qkv, 3 * L.inner, m->o, L.inner, T, L.heads, B, 0.125f * log2e};
    ap.q8 = (uint8_t*)m->qa;
    ap.s8 = m->sa;
    ap.ldq8 = ipad;
    ap.rows8 = rows;
    EVT_HIP(attention_launch(DT_BF16, ap, s), "attention");
    EVT_RC(dense_mx8(L.mout, EPI_BIAS | EPI_RESID | EPI_RESLN, m->qa, ipad, m->sa, m->xm, D,
                     nullptr, rows, m->x, D, s, m->lnst, L.ln1_g, L.ln1_b));
    EVT_HIP(ln_mx8_launch(m->xm, rows, D, dpad, L.ln2_g, L.ln2_b, m->eps, m->lnst, m->qa, m->sa,
                          s),
            "ln2 mx8");
    EVT_RC(dense_mx8(L.mfc1, EPI_BIAS | EPI_GELU | EPI_OUT_MX8, m->qa, dpad, m->sa, m->qh,
                     m->qh_ld, m->shd, rows, nullptr, 0, s));
    EVT_RC(dense_mx8(L.mfc2, EPI_BIAS | EPI_RESID | EPI_RESLN, m->qh, m->qh_ld, m->shd, m->x, D,
                     nullptr, rows, m->xm, D, s, m->lnst, L.ln2_g, L.ln2_b));
  }
  return EVT_OK;
}

int finish_create(evt_model* m, int rc, evt_model** out) {
  if (rc) {
    std::string keep = g_err;
    evt_model_destroy(m);
    g_err = keep;
    return rc;
  }
  *out = m;
  return EVT_OK;
}

struct T2TShape {
  Shape enc;             // encoder geometry (P = (S/16)^2 patches, T = P + 1)
  int grid[3] = {0, 0, 0};
  int din[2] = {0, 0};   // unfolded widths feeding performer 1 / 2
};

int validate_t2t(const evt_t2t_desc* d, T2TShape* ts) {
  if (!d) return fail(EVT_EINVAL, "desc is NULL");
  if (d->dtype != EVT_DTYPE_F32 && d->dtype != EVT_DTYPE_BF16)
    return fail(EVT_EINVAL, "dtype must be EVT_DTYPE_F32 or EVT_DTYPE_BF16");
  if (d->image_size <= 0 || d->image_size % 16)
    return fail(EVT_EINVAL, "image_size must be a positive multiple of 16");
  if (d->in_chans <= 0 || d->num_classes <= 0 || d->depth < 0 || d->mlp_dim <= 0)
    return fail(EVT_EINVAL, "in_chans, num_classes, mlp_dim must be positive, depth >= 0");
  if (d->dim <= 0 || d->dim % 8 != 0 || d->dim > 1024)
    return fail(EVT_EINVAL, "dim must be a positive multiple of 8 and <= 1024");
  if (d->heads <= 0 || d->dim % d->heads != 0)  // Attention raises ValueError (attention.py:8-9)
    return fail(EVT_EINVAL, "hidden_size must be a multiple of num_heads");
  if (d->dim / d->heads > 128) return fail(EVT_EINVAL, "head size (dim / heads) must be <= 128");
  if (d->token_size != 64) return fail(EVT_EINVAL, "token_size must be 64 in this build");
  if (d->max_batch <= 0) return fail(EVT_EINVAL, "max_batch must be positive");
  const int S = d->image_size;
  ts->grid[0] = S / 4;
  ts->grid[1] = S / 8;
  ts->grid[2] = S / 16;
  ts->din[0] = 49 * d->in_chans;
  ts->din[1] = 9 * 64;
  Shape& sh = ts->enc;
  sh.P = ts->grid[2] * ts->grid[2];
  sh.T = sh.P + 1;
  if (sh.T > 256) return fail(EVT_EINVAL, "at most 255 patches per image are supported");
  sh.D = d->dim;
  sh.pd = 9 * 64;
  sh.max_inner = d->dim;  // heads * (dim / heads)
  sh.max_ffn_st = (int)round_up(d->mlp_dim, PAD_N);
  sh.head_st = 0;
  return EVT_OK;
}

size_t t2t_unfold_elems(const T2TShape& ts, int B) {
  const size_t t1 = (size_t)ts.grid[0] * ts.grid[0], t2 = (size_t)ts.grid[1] * ts.grid[1];
  const size_t t3 = (size_t)ts.grid[2] * ts.grid[2];
  return (size_t)B * std::max({t1 * round_up(ts.din[0], PAD_K), t2 * ts.din[1], t3 * ts.din[1]});
}

size_t t2t_unfold_stat_floats(const T2TShape& ts, int B) {
  const size_t t1 = (size_t)ts.grid[0] * ts.grid[0], t2 = (size_t)ts.grid[1] * ts.grid[1];
  return (size_t)B * std::max(t1 * stats_slots(ts.din[0]), t2 * stats_slots(ts.din[1])) * 2;
}

size_t t2t_workspace_bytes(const evt_t2t_desc* d, const T2TShape& ts, int B) {
  const size_t es = elem_size(d->dtype);
  const size_t rows = (size_t)B * ts.enc.T, t1 = (size_t)B * ts.grid[0] * ts.grid[0];
  return t2t_unfold_elems(ts, B) * es + t2t_unfold_stat_floats(ts, B) * 4 + t1 * 4 * 64 * es +
         performer_part_floats(B, ts.grid[0] * ts.grid[0]) * 4 + 2 * rows * d->dim * es +
         2 * rows * stats_slots(d->dim) * 2 * 4 + rows * 4 * ts.enc.max_inner * es +
         rows * ts.enc.max_ffn_st * es + t1 * 2 * 4 + 256;
}


// ---- Swin geometry ------------------------------------------------------------------------
struct SwinGeo {
  int ns = 0;
  int C[EVT_SWIN_MAX_STAGES], Cst[EVT_SWIN_MAX_STAGES], R[EVT_SWIN_MAX_STAGES];
  int mlp[EVT_SWIN_MAX_STAGES], mst[EVT_SWIN_MAX_STAGES];
  int pd = 0, pdst = 0;  // patch vector width (c, kh, kw) and its K padding
};

int validate_swin(const evt_swin_desc* d, SwinGeo* g) {
  if (!d) return fail(EVT_EINVAL, "desc is NULL");
  if (d->dtype != EVT_DTYPE_F32 && d->dtype != EVT_DTYPE_BF16)
    return fail(EVT_EINVAL, "dtype must be EVT_DTYPE_F32 or EVT_DTYPE_BF16");
  if (d->num_stages < 1 || d->num_stages > EVT_SWIN_MAX_STAGES)
    return fail(EVT_EINVAL, "num_stages must be in [1, 8]");
  if (d->patch_size <= 0 || d->image_size <= 0 || d->image_size % d->patch_size)
    return fail(EVT_EINVAL, "image_size must be a multiple of patch_size");
  if (d->in_chans <= 0 || d->num_classes <= 0 || d->max_batch <= 0 || !(d->mlp_ratio > 0.f))
    return fail(EVT_EINVAL, "in_chans, num_classes, max_batch, mlp_ratio must be positive");
  if (d->window_size != 7) return fail(EVT_EINVAL, "window_size must be 7 in this build");
  if (d->embed_dim <= 0 || d->embed_dim % 32)
    return fail(EVT_EINVAL, "embed_dim must be a positive multiple of 32");
  g->ns = d->num_stages;
  g->pd = d->in_chans * d->patch_size * d->patch_size;
  g->pdst = (int)round_up(g->pd, PAD_K);
  int R = d->image_size / d->patch_size;
  for (int i = 0; i < g->ns; ++i) {
    if (i > 0) {
      if (R % 2) return fail(EVT_EINVAL, "patch merging needs an even resolution");
      R /= 2;
    }
    if (R % 7) return fail(EVT_EINVAL, "every stage resolution must be a multiple of the window (7)");
    const int C = d->embed_dim << i;
    if (C > 1024) return fail(EVT_EINVAL, "stage width must be <= 1024");
    if (d->depths[i] < 0) return fail(EVT_EINVAL, "depths must be >= 0");
    if (d->num_heads[i] <= 0 || C % d->num_heads[i] || C / d->num_heads[i] != 32)
      return fail(EVT_EINVAL, "head size (stage width / num_heads) must be 32 in this build");
    g->C[i] = C;
    // Row stride = C (a multiple of 32): no stream padding. The GEMMs that consume these rows
    // read K rounded up to 64 columns; the columns past C belong to the next row (finite values,
    // multiplied by the zero-padded weight rows) and the last row's overrun lands in the zeroed
    // slack SWIN_SLACK at the end of each such buffer.
    g->Cst[i] = C;
    g->R[i] = R;
    g->mlp[i] = (int)(C * d->mlp_ratio);
    if (g->mlp[i] <= 0) return fail(EVT_EINVAL, "mlp width must be positive");
    g->mst[i] = (int)round_up(g->mlp[i], PAD_N);
  }
  return EVT_OK;
}

constexpr size_t SWIN_SLACK = 64;  // zeroed elements after x / xm / o (K-padding overrun)

struct SwinWs {  // element / float counts of the Swin workspace for B images
  size_t stream = 0, stats = 0, qkv = 0, o = 0, hbuf = 0, pooled = 0;
};

SwinWs swin_ws(const SwinGeo& g, int B) {
  SwinWs w;
  for (int i = 0; i < g.ns; ++i) {
    const size_t rows = (size_t)B * g.R[i] * g.R[i];
    w.stream = std::max(w.stream, rows * g.Cst[i]);
    w.stats = std::max(w.stats, rows * stats_slots(g.C[i]) * 2);
    w.qkv = std::max(w.qkv, rows * 3 * g.C[i]);
    w.o = std::max(w.o, rows * g.Cst[i]);
    w.hbuf = std::max(w.hbuf, rows * g.mst[i]);
    if (i > 0) w.hbuf = std::max(w.hbuf, rows * 4 * g.C[i - 1]);
  }
  w.hbuf = std::max(w.hbuf, (size_t)B * g.R[0] * g.R[0] * g.pdst);
  w.pooled = (size_t)B * g.Cst[g.ns - 1];
  return w;
}

size_t swin_workspace_bytes(const evt_swin_desc* d, const SwinGeo& g, int B) {
  const SwinWs w = swin_ws(g, B);
  const size_t es = elem_size(d->dtype);
  return (2 * w.stream + w.qkv + w.o + w.hbuf + w.pooled + 3 * SWIN_SLACK) * es +
         2 * w.stats * sizeof(float);
}

}  // namespace

extern "C" {

int evt_init(int device) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) return fail(EVT_ENODEV, "no HIP device visible");
  if (device < 0 || device >= n) return fail(EVT_ENODEV, "device index out of range");
  hipDeviceProp_t prop;
  EVT_HIP(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(EVT_ENODEV, std::string("device is ") + prop.gcnArchName + ", this build is gfx950");
  EVT_HIP(hipSetDevice(device), "hipSetDevice");
  return EVT_OK;
}

const char* evt_last_error(void) { return g_err.c_str(); }

int evt_vit_num_weights(const evt_vit_desc* desc) {
  if (!desc || desc->depth < 0) return fail(EVT_EINVAL, "bad desc");
  return 4 + (desc->semantics == EVT_VIT_STANDARD ? 12 : 11) * desc->depth + 4;
}

int evt_query_workspace(const evt_vit_desc* desc, int batch, size_t* bytes) {
  Shape sh;
  EVT_RC(validate(desc, &sh));
  if (!bytes || batch <= 0) return fail(EVT_EINVAL, "bytes must be non-null and batch positive");
  *bytes = workspace_bytes(desc, sh, batch);
  return EVT_OK;
}

// evt_model_set_lanes: the children (their workspaces), streams and events of a model
static void release_lanes(evt_model* m) {
  for (evt_model* c : m->lanes) evt_model_destroy(c);
  for (size_t i = 0; i < m->lane_s.size(); ++i)
    if (m->lane_own[i]) (void)hipStreamDestroy(m->lane_s[i]);
  for (hipEvent_t e : m->lane_ev) (void)hipEventDestroy(e);
  m->lanes.clear();
  m->lane_s.clear();
  m->lane_own.clear();
  m->lane_ev.clear();
}

int evt_model_destroy(evt_model* m) {
  if (!m) return EVT_OK;
  // forwards enqueued on any stream may still read the workspace / weights: wait for the device
  // before freeing (hipFree would also synchronise, but only implicitly)
  (void)hipDeviceSynchronize();
  release_lanes(m);
  if (m->graph_exec) (void)hipGraphExecDestroy(m->graph_exec);
  if (m->graph) (void)hipGraphDestroy(m->graph);
  for (hipEvent_t e : m->prof_ev) (void)hipEventDestroy(e);
  for (void* p : m->allocs) (void)hipFree(p);
  delete m;
  return EVT_OK;
}

static int swin_alloc_ws(evt_model* m, int B, hipStream_t s);  // (the Swin section)

// A forward of B images over the model's lanes (evt_model_set_lanes): lane i takes images
// [B i / k, B (i + 1) / k) on its own stream, forked from and joined to s by events (a HIP graph
// capture on s records the lanes as parallel branches)
typedef int (*ForwardFn)(evt_model*, const float*, int, float*, void*);
static int lanes_forward(evt_model* m, ForwardFn fwd, const float* img, size_t img_elems, int B,
                         float* logits, hipStream_t s) {
  // the joins go onto s after every lane's work: a lane stream that shares s's hardware queue
  // would otherwise queue its kernels behind s's wait for the previous lane (measured: lanes
  // serialised in part)
  const int k = (int)m->lanes.size();
  EVT_HIP(hipEventRecord(m->lane_ev[0], s), "lanes fork");
  for (int i = 0; i < k; ++i)
    EVT_HIP(hipStreamWaitEvent(m->lane_s[i], m->lane_ev[0], 0), "lane fork wait");
  for (int i = 0; i < k; ++i) {
    const int b0 = (int)((int64_t)B * i / k), b1 = (int)((int64_t)B * (i + 1) / k);
    if (b1 > b0)
      EVT_RC(fwd(m->lanes[i], img + (size_t)b0 * img_elems, b1 - b0,
                 logits + (size_t)b0 * m->num_classes, m->lane_s[i]));
    EVT_HIP(hipEventRecord(m->lane_ev[1 + i], m->lane_s[i]), "lane done");
  }
  for (int i = 0; i < k; ++i)
    EVT_HIP(hipStreamWaitEvent(s, m->lane_ev[1 + i], 0), "lanes join");
  m->hm_layers = m->lanes[0]->hm_layers;
  return EVT_OK;
}

// The ViT workspace for B images (activation buffers only; lanes allocate their own)
static int vit_alloc_ws(evt_model* m, int B, hipStream_t s) {
  const Shape& sh = m->sh;
  const int D = m->D;
  const size_t es = elem_size(m->dtype);
  EVT_RC(alloc_encoder_ws(m, B, std::max((size_t)B * sh.T * sh.max_ffn_st,
                                         (size_t)B * sh.P * sh.pd) * es, s));
  m->apatch = m->hbuf;
  EVT_RC(dev_alloc(m, &m->hh, (size_t)B * sh.head_st * es));
  if (m->mx8) {
    const size_t rows = (size_t)B * sh.T;
    m->qa_ld = (int)std::max(round_up(D, 128), round_up(sh.max_inner, 128));
    int maxffn = 0;
    for (int f : m->ffn) maxffn = std::max(maxffn, f);
    m->qh_ld = (int)round_up(maxffn, 128);
    EVT_RC(dev_alloc(m, &m->qa, rows * m->qa_ld));
    EVT_RC(dev_alloc(m, (void**)&m->sa, rows * (m->qa_ld / 128) * 4));
    EVT_RC(dev_alloc(m, &m->qh, rows * m->qh_ld));
    EVT_RC(dev_alloc(m, (void**)&m->shd, rows * (m->qh_ld / 128) * 4));
    EVT_RC(dev_alloc(m, (void**)&m->lnst, rows * 2 * sizeof(float)));
    // every byte of the MX8 operands is written finite before it is read (NaN-free padding)
    EVT_HIP(hipMemsetAsync(m->qa, 0, rows * m->qa_ld, s), "memset qa");
    EVT_HIP(hipMemsetAsync(m->sa, 0, rows * (m->qa_ld / 128) * 4, s), "memset qa scales");
    // FC1 writes columns < roundup(ffn, 32) only: the rest of the FC2 operand stays zero
    EVT_HIP(hipMemsetAsync(m->qh, 0, rows * m->qh_ld, s), "memset qh");
    EVT_HIP(hipMemsetAsync(m->shd, 0, rows * (m->qh_ld / 128) * 4, s), "memset qh scales");
  }
  m->ws_bytes = workspace_bytes(&m->desc, sh, B);
  return EVT_OK;
}

int evt_vit_create(const evt_vit_desc* desc, const float* const* w, int n_weights, void* stream,
                   evt_model** out) {
  if (!out) return fail(EVT_EINVAL, "out is NULL");
  *out = nullptr;
  Shape sh;
  EVT_RC(validate(desc, &sh));
  if (n_weights != evt_vit_num_weights(desc) || !w)
    return fail(EVT_EINVAL, "expected " + std::to_string(evt_vit_num_weights(desc)) + " weights");
  for (int i = 0; i < n_weights; ++i)
    if (!w[i]) return fail(EVT_EINVAL, "weight pointer " + std::to_string(i) + " is NULL");
  hipStream_t s = (hipStream_t)stream;
  evt_model* m = new evt_model();
  m->family = 0;
  m->mx8 = desc->dtype == EVT_DTYPE_MX8;
  m->dtype = m->mx8 ? DT_BF16 : desc->dtype;  // MX8 models keep bf16 for everything else
  m->D = desc->dim;
  m->max_batch = desc->max_batch;
  m->num_classes = desc->num_classes;
  m->desc = *desc;
  m->standard = desc->semantics == EVT_VIT_STANDARD;
  if (desc->layer_norm_eps > 0.f) m->eps = desc->layer_norm_eps;
  m->heads.assign(desc->heads, desc->heads + desc->depth);
  m->head_dim.assign(desc->head_dim, desc->head_dim + desc->depth);
  m->ffn.assign(desc->ffn, desc->ffn + desc->depth);
  m->desc.heads = m->heads.data();
  m->desc.head_dim = m->head_dim.data();
  m->desc.ffn = m->ffn.data();
  m->sh = sh;
  const int D = desc->dim;
  auto run = [&]() -> int {
    if (desc->patch_size % 8 == 0) {  // channel-major patch vectors (patchify_cm_kernel)
      float* wcm = nullptr;
      EVT_RC(dev_alloc(m, (void**)&wcm, (size_t)sh.pd * D * sizeof(float)));
      EVT_HIP(patch_weight_cm(w[0], wcm, desc->in_chans, desc->patch_size, D, s), "patch weight");
      EVT_RC(make_dense(m, &m->patch, wcm, w[1], sh.pd, D, s));
      m->patch_cm = true;
    } else {
      EVT_RC(make_dense(m, &m->patch, w[0], w[1], sh.pd, D, s));
    }
    EVT_RC(copy_vec(m, &m->cls, w[2], D, s));
    EVT_RC(copy_vec(m, &m->pos, w[3], (size_t)sh.T * D, s));
    if (m->dtype == DT_BF16) {
      EVT_RC(dev_alloc(m, &m->pos_h, (size_t)sh.T * D * 2));
      EVT_HIP(to_bf16_launch(m->pos, m->pos_h, (int64_t)sh.T * D, s), "pos -> bf16");
    }
    EVT_RC(build_encoder(m, w + 4, s));
    const int k = 4 + (m->standard ? 12 : 11) * desc->depth;
    if (m->standard) {  // final LayerNorm folded into the classifier (CLS rows)
      EVT_RC(make_dense(m, &m->head, w[k + 2], w[k + 3], D, desc->num_classes, s, w[k + 0],
                        w[k + 1]));
    } else {
      EVT_RC(make_dense(m, &m->head1, w[k + 0], w[k + 1], D, desc->mlp_dim, s));
      EVT_RC(make_dense(m, &m->head2, w[k + 2], w[k + 3], desc->mlp_dim, desc->num_classes, s));
    }
    EVT_RC(vit_alloc_ws(m, desc->max_batch, s));
    EVT_HIP(hipStreamSynchronize(s), "create sync");
    return EVT_OK;
  };
  return finish_create(m, run(), out);
}

int evt_vit_forward(evt_model* m, const float* img, int B, float* logits, void* stream) {
  if (!m || !img || !logits) return fail(EVT_EINVAL, "model, img and logits must be non-null");
  if (m->family != 0) return fail(EVT_EINVAL, "model is not a ViT (use evt_t2t_forward)");
  if (B <= 0 || B > m->max_batch)
    return fail(EVT_EINVAL, "batch must be in [1, max_batch=" + std::to_string(m->max_batch) + "]");
  hipStream_t s = (hipStream_t)stream;
  if (!m->lanes.empty() && !m->prof && B >= (int)m->lanes.size())  // profiling: one lane
    return lanes_forward(m, evt_vit_forward, img,
                         (size_t)m->desc.in_chans * m->desc.image_size * m->desc.image_size, B,
                         logits, s);
  const evt_vit_desc& d = m->desc;
  const Shape& sh = m->sh;
  const int D = d.dim, T = sh.T, dt = m->dtype;
  prof_reset(m);
  // patch embedding (vit.py:45-51): rearrange -> Dense(D) + pos, CLS row = cls + pos[0]
  {
    ProfScope ps(m, EVT_PROF_PATCHIFY, s);
    prof_work(m, 0.0, (double)B * d.in_chans * d.image_size * d.image_size * 4 +
                          (double)B * (sh.P * sh.pd + D) * elem_size(dt) +
                          (double)B * stats_slots(D) * 8);  // image read, patch rows + CLS rows
    EVT_HIP(patchify_launch(dt, img, B, d.in_chans, d.image_size, d.patch_size, m->apatch, m->x,
                            m->cls, m->pos, D, m->sx, s, m->patch_cm),
            "patchify");
  }
  {
    ProfScope ps(m, EVT_PROF_PATCH_EMBED, s);
    DenseCall c;
    c.flags = EPI_BIAS | EPI_POS | EPI_STATS;
    c.A = m->apatch; c.lda = sh.pd; c.C = m->x; c.ldc = D; c.M = B * sh.P; c.N = D;
    c.pos = m->pos; c.ldp = D; c.P = sh.P; c.stats_out = m->sx;
    c.resid = m->pos_h; c.ldr = m->pos_h ? D : 0;  // bf16 table for the persistent kernel
    EVT_RC(dense(m, m->patch, c, s));
  }
  EVT_RC(m->mx8 ? run_encoder_mx8(m, B, s) : run_encoder(m, B, s));
  ProfScope ps_head(m, EVT_PROF_HEAD, s);
  if (m->standard) {  // final LayerNorm of the CLS rows folded into the Linear head
    DenseCall c;
    c.flags = EPI_LNIN | EPI_BIAS | EPI_OUT_F32;
    c.A = m->x; c.lda = (int64_t)T * D; c.C = logits; c.ldc = d.num_classes; c.M = B;
    c.N = d.num_classes; c.stats_in = m->sx; c.stats_step = T;
    EVT_RC(dense(m, m->head, c, s));
    return EVT_OK;
  }
  // head on token 0 (vit.py:54-55; no final LayerNorm): rows b*T of the stream, stride T*D
  {
    DenseCall c;
    c.flags = EPI_BIAS | EPI_GELU;
    c.A = m->x; c.lda = (int64_t)T * D; c.C = m->hh; c.ldc = sh.head_st; c.M = B; c.N = sh.head_st;
    EVT_RC(dense_head(m, m->head1, c, s));
  }
  {
    DenseCall c;
    c.flags = EPI_BIAS | EPI_OUT_F32;
    c.A = m->hh; c.lda = sh.head_st; c.C = logits; c.ldc = d.num_classes; c.M = B;
    c.N = d.num_classes;
    EVT_RC(dense_head(m, m->head2, c, s));
  }
  return EVT_OK;
}

// ---- T2T-ViT ----------------------------------------------------------------------------

int evt_t2t_num_weights(const evt_t2t_desc* desc) {
  if (!desc || desc->depth < 0) return fail(EVT_EINVAL, "bad desc");
  return 2 * 13 + 4 + 11 * desc->depth + 4;
}

int evt_t2t_query_workspace(const evt_t2t_desc* desc, int batch, size_t* bytes) {
  T2TShape ts;
  EVT_RC(validate_t2t(desc, &ts));
  if (!bytes || batch <= 0) return fail(EVT_EINVAL, "bytes must be non-null and batch positive");
  *bytes = t2t_workspace_bytes(desc, ts, batch);
  return EVT_OK;
}

// The T2T-ViT workspace for B images (activation buffers only; lanes allocate their own)
static int t2t_alloc_ws(evt_model* m, int B, hipStream_t s) {
  T2TShape ts;
  EVT_RC(validate_t2t(&m->tdesc, &ts));
  const size_t es = elem_size(m->dtype);
  const size_t t1 = (size_t)B * ts.grid[0] * ts.grid[0];
  EVT_RC(dev_alloc(m, &m->u, t2t_unfold_elems(ts, B) * es));
  EVT_RC(dev_alloc(m, (void**)&m->su, t2t_unfold_stat_floats(ts, B) * sizeof(float)));
  EVT_RC(dev_alloc(m, &m->kqvb, t1 * 3 * 64 * es));
  EVT_RC(dev_alloc(m, &m->pout, t1 * 64 * es));
  EVT_RC(dev_alloc(m, (void**)&m->tstats, t1 * 2 * sizeof(float)));
  EVT_RC(dev_alloc(m, &m->zrow, 256));
  EVT_HIP(hipMemsetAsync(m->zrow, 0, 256, s), "memset zero row");
  EVT_RC(dev_alloc(m, (void**)&m->part, performer_part_floats(B, ts.grid[0] * ts.grid[0]) *
                                            sizeof(float)));
  EVT_RC(alloc_encoder_ws(m, B, (size_t)B * ts.enc.T * ts.enc.max_ffn_st * es, s));
  m->ws_bytes = t2t_workspace_bytes(&m->tdesc, ts, B);
  return EVT_OK;
}

int evt_t2t_create(const evt_t2t_desc* desc, const float* const* w, int n_weights, void* stream,
                   evt_model** out) {
  if (!out) return fail(EVT_EINVAL, "out is NULL");
  *out = nullptr;
  T2TShape ts;
  EVT_RC(validate_t2t(desc, &ts));
  if (n_weights != evt_t2t_num_weights(desc) || !w)
    return fail(EVT_EINVAL, "expected " + std::to_string(evt_t2t_num_weights(desc)) + " weights");
  for (int i = 0; i < n_weights; ++i)
    if (!w[i]) return fail(EVT_EINVAL, "weight pointer " + std::to_string(i) + " is NULL");
  hipStream_t s = (hipStream_t)stream;
  evt_model* m = new evt_model();
  m->family = 1;
  m->dtype = desc->dtype;
  m->D = desc->dim;
  m->max_batch = desc->max_batch;
  m->num_classes = desc->num_classes;
  m->tdesc = *desc;
  m->heads.assign(desc->depth, desc->heads);
  m->head_dim.assign(desc->depth, desc->dim / desc->heads);  // h_k = dim // heads
  m->ffn.assign(desc->depth, desc->mlp_dim);
  m->sh = ts.enc;
  for (int i = 0; i < 3; ++i) m->grid[i] = ts.grid[i];
  const int D = desc->dim;
  auto run = [&]() -> int {
    int k = 0;
    for (int pi = 0; pi < 2; ++pi) {  // transformer_encoder.py:43-65
      Performer& P = m->perf[pi];
      P.din = ts.din[pi];
      P.dpad = (int)round_up(P.din, PAD_K);
      if (m->dtype == DT_BF16) {  // output columns permuted for the performers' 16-B loads
        float *wp = nullptr, *bp = nullptr;
        EVT_RC(dev_alloc(m, (void**)&wp, (size_t)P.din * 3 * 64 * sizeof(float)));
        EVT_RC(dev_alloc(m, (void**)&bp, 3 * 64 * sizeof(float)));
        EVT_HIP(kqv_permute_launch(w[k + 2], w[k + 3], P.din, wp, bp, s), "kqv permute");
        EVT_RC(make_dense(m, &P.kqv, wp, bp, P.din, 3 * 64, s, w[k + 0], w[k + 1]));
      } else {
        EVT_RC(make_dense(m, &P.kqv, w[k + 2], w[k + 3], P.din, 3 * 64, s, w[k + 0], w[k + 1]));
      }
      const float* src[9] = {w[k + 4], w[k + 5], w[k + 6], w[k + 7], w[k + 8],
                             w[k + 9], w[k + 10], w[k + 11], w[k + 12]};
      const size_t len[9] = {32 * 64, 64 * 64, 64, 64, 64, 64 * 64, 64, 64 * 64, 64};
      float* dst[9];
      for (int j = 0; j < 9; ++j) EVT_RC(copy_vec(m, &dst[j], src[j], len[j], s));
      P.w = PerformerWeights{dst[0], dst[1], dst[2], dst[3], dst[4], dst[5], dst[6], dst[7], dst[8]};
      k += 13;
    }
    EVT_RC(make_dense(m, &m->project, w[k + 0], w[k + 1], 9 * 64, D, s));  // t2t_vit.py:56,86
    EVT_RC(copy_vec(m, &m->cls, w[k + 2], D, s));
    EVT_RC(copy_vec(m, &m->pos, w[k + 3], (size_t)ts.enc.T * D, s));
    if (desc->dtype == DT_BF16) {  // bf16 table for the persistent project GEMM (EPI_POS)
      EVT_RC(dev_alloc(m, &m->pos_h, (size_t)ts.enc.T * D * 2));
      EVT_HIP(to_bf16_launch(m->pos, m->pos_h, (int64_t)ts.enc.T * D, s), "pos -> bf16");
    }
    k += 4;
    EVT_RC(build_encoder(m, w + k, s));
    k += 11 * desc->depth;
    // final LayerNorm (t2t_vit.py:111,129) folded into the classifier (:114,134)
    EVT_RC(make_dense(m, &m->head, w[k + 2], w[k + 3], D, desc->num_classes, s, w[k + 0], w[k + 1]));
    EVT_RC(t2t_alloc_ws(m, desc->max_batch, s));
    EVT_HIP(hipStreamSynchronize(s), "create sync");
    return EVT_OK;
  };
  return finish_create(m, run(), out);
}

int evt_t2t_forward(evt_model* m, const float* img, int B, float* logits, void* stream) {
  if (!m || !img || !logits) return fail(EVT_EINVAL, "model, img and logits must be non-null");
  if (m->family != 1) return fail(EVT_EINVAL, "model is not a T2T-ViT (use evt_vit_forward)");
  if (B <= 0 || B > m->max_batch)
    return fail(EVT_EINVAL, "batch must be in [1, max_batch=" + std::to_string(m->max_batch) + "]");
  hipStream_t s = (hipStream_t)stream;
  if (!m->lanes.empty() && !m->prof && B >= (int)m->lanes.size())  // profiling: one lane
    return lanes_forward(m, evt_t2t_forward, img,
                         (size_t)m->tdesc.image_size * m->tdesc.image_size * m->tdesc.in_chans, B,
                         logits, s);
  prof_reset(m);
  const evt_t2t_desc& d = m->tdesc;
  const int dt = d.dtype, D = d.dim, T = m->sh.T, P = m->sh.P, S = d.image_size;
  const int g1 = m->grid[0], g2 = m->grid[1];
  const int t1 = g1 * g1, t2 = g2 * g2;
  // iteration 1: soft_split0 (k7 s4 p2) of the NHWC image -> TokenPerformer    (t2t_vit.py:66-68)
  const double es = (double)elem_size(dt);
  // performer core per token (transformer_encoder.py:67-99): prm_exp of k and q (2 x 64x32),
  // D (32), kptv (32x64), y (32x64), attn_output Dense (64x64), FFN (2 x 64x64)
  const double perf_flops = 2.0 * (2 * 64 * 32 + 32 + 32 * 64 + 32 * 64 + 3 * 64 * 64);
  const Performer& P1 = m->perf[0];
  {
    ProfScope ps(m, EVT_PROF_T2T_UNFOLD, s);
    prof_work(m, 0.0, (double)B * S * S * d.in_chans * 4 + (double)B * t1 * P1.din * es +
                          (double)B * t1 * stats_slots(P1.din) * 8);
    EVT_HIP(unfold_launch(dt, 1, img, B, S, S, d.in_chans, 7, 4, 2, m->u, P1.dpad, m->su,
                          stats_slots(P1.din), s),
            "soft_split0");
  }
  {
    ProfScope ps(m, EVT_PROF_T2T_KQV, s);
    DenseCall c;
    c.flags = EPI_LNIN | EPI_BIAS;
    c.A = m->u; c.lda = P1.dpad; c.C = m->kqvb; c.ldc = 3 * 64; c.M = B * t1; c.N = 3 * 64;
    c.stats_in = m->su; c.ln_width = P1.din;
    EVT_RC(dense(m, P1.kqv, c, s));
  }
  // soft_split1 gathered inside the kqv GEMM's A loader where it can (bf16, persistent GEMM): the
  // performer then also writes per-token statistics, from which the split rows' are summed
  const Performer& P2 = m->perf[1];
  const bool gather1 = dt == DT_BF16 && P2.dpad == 9 * 64 && g2 == (g1 + 1) / 2 && m->zrow;
  {
    ProfScope ps(m, EVT_PROF_T2T_PERFORMER, s);
    prof_work(m, perf_flops * B * t1, (double)B * t1 * (3 * 64 + 64) * es);
    EVT_HIP(performer_launch(dt, m->kqvb, 3 * 64, B, t1, P1.w, m->part, m->pout, 64, s,
                             gather1 ? m->tstats : nullptr, dt == DT_BF16),
            "performer1");
  }
  // iteration 2: soft_split1 (k3 s2 p1) of the [B, S/4, S/4, 64] map -> TokenPerformer (:72-77)
  bool fused1 = false;
  if (gather1) {
    ProfScope ps(m, EVT_PROF_T2T_KQV, s);
    DenseCall c;
    c.flags = EPI_LNIN | EPI_BIAS | EPI_SPLIT;
    c.A = m->pout; c.lda = 64; c.C = m->kqvb; c.ldc = 3 * 64; c.M = B * t2; c.N = 3 * 64;
    c.stats_in = m->su; c.ln_width = P2.din;
    GemmParams p = dense_params(m, P2.kqv, c);
    p.gmode = 2; p.gR = g1; p.gC = 64; p.gOW = g2; p.gzero = m->zrow;
    p.g_inv_rr = 1.0f / (float)(g2 * g2); p.g_inv_r = 1.0f / (float)g2;
    EVT_HIP(unfold_stats_launch(m->tstats, B, g1, m->su, stats_slots(P2.din), s),
            "soft_split1 statistics");
    const hipError_t e = gemm_launch(dt, c.flags, p, s);
    if (e == hipSuccess) {
      c.flags &= ~EPI_SPLIT;
      dense_work(m, P2.kqv, c);
      fused1 = true;
    } else if (e != hipErrorNotSupported) {
      EVT_HIP(e, "soft_split1 + kqv (gathered)");
    }
  }
  if (!fused1) {
    {
      ProfScope ps(m, EVT_PROF_T2T_UNFOLD, s);
      prof_work(m, 0.0, (double)B * t1 * 64 * es + (double)B * t2 * P2.din * es +
                            (double)B * t2 * stats_slots(P2.din) * 8);
      EVT_HIP(unfold_launch(dt, 0, m->pout, B, g1, g1, 64, 3, 2, 1, m->u, P2.dpad, m->su,
                            stats_slots(P2.din), s),
              "soft_split1");
    }
    ProfScope ps(m, EVT_PROF_T2T_KQV, s);
    DenseCall c;
    c.flags = EPI_LNIN | EPI_BIAS;
    c.A = m->u; c.lda = P2.dpad; c.C = m->kqvb; c.ldc = 3 * 64; c.M = B * t2; c.N = 3 * 64;
    c.stats_in = m->su; c.ln_width = P2.din;
    EVT_RC(dense(m, P2.kqv, c, s));
  }
  {
    ProfScope ps(m, EVT_PROF_T2T_PERFORMER, s);
    prof_work(m, perf_flops * B * t2, (double)B * t2 * (3 * 64 + 64) * es);
    EVT_HIP(performer_launch(dt, m->kqvb, 3 * 64, B, t2, P2.w, m->part, m->pout, 64, s, nullptr,
                             dt == DT_BF16),
            "performer2");
  }
  // soft_split2 -> project Dense(D) into token rows 1..P, + CLS row, + sinusoid pos (:81-86,121-125)
  // (the split gathered inside the project GEMM's A loader where it can, as soft_split1)
  const int g3 = m->grid[2];
  bool fused2 = false;
  if (dt == DT_BF16 && g3 == (g2 + 1) / 2 && m->zrow && m->pos_h) {
    ProfScope ps(m, EVT_PROF_PATCH_EMBED, s);
    prof_work(m, 0.0, (double)B * D * es + (double)B * stats_slots(D) * 8);
    EVT_HIP(cls_rows_launch(dt, m->x, B, T, D, m->cls, m->pos, m->sx, s), "cls rows");
    DenseCall c;
    c.flags = EPI_BIAS | EPI_POS | EPI_STATS | EPI_SPLIT;
    c.A = m->pout; c.lda = 64; c.C = m->x; c.ldc = D; c.M = B * P; c.N = D;
    c.pos = m->pos; c.ldp = D; c.P = P; c.stats_out = m->sx;
    c.resid = m->pos_h; c.ldr = D;
    GemmParams p = dense_params(m, m->project, c);
    p.gmode = 2; p.gR = g2; p.gC = 64; p.gOW = g3; p.gzero = m->zrow;
    p.g_inv_rr = 1.0f / (float)(g3 * g3); p.g_inv_r = 1.0f / (float)g3;
    const hipError_t e = gemm_launch(dt, c.flags, p, s);
    if (e == hipSuccess) {
      c.flags &= ~EPI_SPLIT;
      dense_work(m, m->project, c);
      fused2 = true;
    } else if (e != hipErrorNotSupported) {
      EVT_HIP(e, "soft_split2 + project (gathered)");
    }
  }
  if (!fused2) {
    {
      ProfScope ps(m, EVT_PROF_T2T_UNFOLD, s);
      prof_work(m, 0.0, (double)B * t2 * 64 * es + (double)B * P * 9 * 64 * es);
      EVT_HIP(unfold_launch(dt, 0, m->pout, B, g2, g2, 64, 3, 2, 1, m->u, 9 * 64, nullptr, 0, s),
              "soft_split2");
    }
    ProfScope ps(m, EVT_PROF_PATCH_EMBED, s);
    prof_work(m, 0.0, (double)B * D * es + (double)B * stats_slots(D) * 8);
    EVT_HIP(cls_rows_launch(dt, m->x, B, T, D, m->cls, m->pos, m->sx, s), "cls rows");
    DenseCall c;
    c.flags = EPI_BIAS | EPI_POS | EPI_STATS;
    c.A = m->u; c.lda = 9 * 64; c.C = m->x; c.ldc = D; c.M = B * P; c.N = D;
    c.pos = m->pos; c.ldp = D; c.P = P; c.stats_out = m->sx;
    EVT_RC(dense(m, m->project, c, s));
  }
  EVT_RC(run_encoder(m, B, s));  // :127
  {  // LayerNorm of the CLS rows folded into the classifier (:129-134)
    ProfScope ps(m, EVT_PROF_HEAD, s);
    DenseCall c;
    c.flags = EPI_LNIN | EPI_BIAS | EPI_OUT_F32;
    c.A = m->x; c.lda = (int64_t)T * D; c.C = logits; c.ldc = d.num_classes; c.M = B;
    c.N = d.num_classes; c.stats_in = m->sx; c.stats_step = T;
    EVT_RC(dense(m, m->head, c, s));
  }
  return EVT_OK;
}

int evt_model_profile(evt_model* m, int enable) {
  if (!m) return fail(EVT_EINVAL, "model is NULL");
  if (m->graph && enable) return fail(EVT_EINVAL, "profiling a model with a captured graph");
  m->prof = enable != 0;
  m->prof_role.clear();
  m->prof_gflop.clear();
  m->prof_gbytes.clear();
  return EVT_OK;
}

int evt_model_profile_read(evt_model* m, float* us, int* launches) {
  if (!m || !us || !launches) return fail(EVT_EINVAL, "null argument");
  for (int r = 0; r < EVT_PROF_ROLES; ++r) {
    us[r] = 0.f;
    launches[r] = 0;
  }
  for (size_t i = 0; i < m->prof_role.size(); ++i) {
    EVT_HIP(hipEventSynchronize(m->prof_ev[2 * i + 1]), "profile sync");
    float ms = 0.f;
    EVT_HIP(hipEventElapsedTime(&ms, m->prof_ev[2 * i], m->prof_ev[2 * i + 1]), "profile read");
    us[m->prof_role[i]] += 1000.f * ms;
    launches[m->prof_role[i]] += 1;
  }
  return EVT_OK;
}

int evt_model_qkv_layout(const evt_model* m, int* headmajor_layers) {
  if (!m || !headmajor_layers) return fail(EVT_EINVAL, "null argument");
  *headmajor_layers = m->hm_layers;
  return EVT_OK;
}

int evt_model_set_lanes(evt_model* m, int lanes, void* stream) {
  if (!m) return fail(EVT_EINVAL, "model is NULL");
  if (m->is_lane) return fail(EVT_EINVAL, "the model is a lane of another model");
  if (lanes < 1 || lanes > 4) return fail(EVT_EINVAL, "lanes must be in [1, 4]");
  if (m->graph) return fail(EVT_EINVAL, "set the lanes before evt_graph_capture");
  (void)hipDeviceSynchronize();  // forwards of the current lanes may still be running
  release_lanes(m);
  if (lanes == 1) return EVT_OK;
  hipStream_t s = (hipStream_t)stream;
  const int per = (m->max_batch + lanes - 1) / lanes;
  auto run = [&]() -> int {
    for (int i = 0; i < lanes; ++i) {
      // the copy shares the parent's weights (its allocations stay the parent's); everything
      // per-model is reset and the workspace allocated anew for `per` images
      evt_model* c = new evt_model(*m);
      c->allocs.clear();
      c->lanes.clear();
      c->lane_s.clear();
      c->lane_own.clear();
      c->lane_ev.clear();
      c->graph = nullptr;
      c->graph_exec = nullptr;
      c->prof = false;
      c->prof_ev.clear();
      c->prof_role.clear();
      c->prof_gflop.clear();
      c->prof_gbytes.clear();
      c->is_lane = true;
      c->max_batch = per;
      c->no_balance = m->family == 1 ? 1 : 0;
      c->u = c->kqvb = c->pout = c->zrow = c->x = c->xm = c->qkv = c->o = c->hbuf = nullptr;
      c->hh = c->sk = c->pooled = c->apatch = c->qa = c->qh = nullptr;
      c->su = c->tstats = c->part = c->sx = c->sm = c->lnst = nullptr;
      c->sa = c->shd = nullptr;
      m->lanes.push_back(c);
      EVT_RC(m->family == 0   ? vit_alloc_ws(c, per, s)
             : m->family == 1 ? t2t_alloc_ws(c, per, s)
                              : swin_alloc_ws(c, per, s));
      hipStream_t st = nullptr;
      EVT_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "lane stream");
      m->lane_s.push_back(st);
      m->lane_own.push_back(1);
    }
    for (int i = 0; i <= lanes; ++i) {
      hipEvent_t e = nullptr;
      EVT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming), "lane event");
      m->lane_ev.push_back(e);
    }
    EVT_HIP(hipStreamSynchronize(s), "lanes sync");
    return EVT_OK;
  };
  const int rc = run();
  if (rc) {
    const std::string keep = g_err;
    (void)hipDeviceSynchronize();
    release_lanes(m);
    g_err = keep;
  }
  return rc;
}

int evt_model_set_lane_streams(evt_model* m, int n, void* const* streams) {
  if (!m || !streams) return fail(EVT_EINVAL, "null argument");
  if (m->lanes.empty() || n != (int)m->lanes.size())
    return fail(EVT_EINVAL, "n must equal the lane count (evt_model_set_lanes first)");
  for (int i = 0; i < n; ++i)
    if (!streams[i]) return fail(EVT_EINVAL, "lane streams must be non-NULL");
  if (m->graph) return fail(EVT_EINVAL, "set the lane streams before evt_graph_capture");
  (void)hipDeviceSynchronize();
  for (int i = 0; i < n; ++i) {
    if (m->lane_own[i]) (void)hipStreamDestroy(m->lane_s[i]);
    m->lane_s[i] = (hipStream_t)streams[i];
    m->lane_own[i] = 0;
  }
  return EVT_OK;
}

int evt_model_lanes(const evt_model* m, int* lanes) {
  if (!m || !lanes) return fail(EVT_EINVAL, "null argument");
  *lanes = m->lanes.empty() ? 1 : (int)m->lanes.size();
  return EVT_OK;
}

int evt_model_profile_work(evt_model* m, double* gflop, double* gbytes) {
  if (!m || !gflop || !gbytes) return fail(EVT_EINVAL, "null argument");
  for (int r = 0; r < EVT_PROF_ROLES; ++r) gflop[r] = gbytes[r] = 0.0;
  for (size_t i = 0; i < m->prof_role.size(); ++i) {
    gflop[m->prof_role[i]] += m->prof_gflop[i];
    gbytes[m->prof_role[i]] += m->prof_gbytes[i];
  }
  return EVT_OK;
}

int evt_graph_capture(evt_model* m, const float* img, int batch, float* logits, void* stream) {
  if (!m || !stream) return fail(EVT_EINVAL, "graph capture needs a model and a non-NULL stream");
  if (m->prof)  // the events would be captured into the graph, never recorded on the stream
    return fail(EVT_EINVAL, "graph capture while profiling is enabled (evt_model_profile(m, 0) first)");
  hipStream_t s = (hipStream_t)stream;
  if (m->graph_exec) {
    (void)hipGraphExecDestroy(m->graph_exec);
    m->graph_exec = nullptr;
  }
  if (m->graph) {
    (void)hipGraphDestroy(m->graph);
    m->graph = nullptr;
  }
  EVT_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal), "begin capture");
  const int rc = m->family == 0   ? evt_vit_forward(m, img, batch, logits, stream)
                 : m->family == 1 ? evt_t2t_forward(m, img, batch, logits, stream)
                                  : evt_swin_forward(m, img, batch, logits, stream);
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(s, &g);
  if (rc) {
    if (g) (void)hipGraphDestroy(g);
    return rc;
  }
  if (e != hipSuccess) return hip_fail(e, "end capture");
  hipGraphExec_t ge = nullptr;
  const hipError_t ei = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  if (ei != hipSuccess) {
    (void)hipGraphDestroy(g);
    return hip_fail(ei, "graph instantiate");
  }
  m->graph = g;
  m->graph_exec = ge;
  return EVT_OK;
}

int evt_graph_launch(evt_model* m, void* stream) {
  if (!m || !m->graph_exec) return fail(EVT_EINVAL, "no captured graph (call evt_graph_capture)");
  EVT_HIP(hipGraphLaunch(m->graph_exec, (hipStream_t)stream), "graph launch");
  return EVT_OK;
}

// ---- Swin Transformer -------------------------------------------------------------------

int evt_swin_num_weights(const evt_swin_desc* desc) {
  if (!desc || desc->num_stages < 1 || desc->num_stages > EVT_SWIN_MAX_STAGES)
    return fail(EVT_EINVAL, "bad desc");
  int n = 4 + 4;
  for (int i = 0; i < desc->num_stages; ++i) n += (i > 0 ? 3 : 0) + 13 * desc->depths[i];
  return n;
}

int evt_swin_query_workspace(const evt_swin_desc* desc, int batch, size_t* bytes) {
  SwinGeo g;
  EVT_RC(validate_swin(desc, &g));
  if (!bytes || batch <= 0) return fail(EVT_EINVAL, "bytes must be non-null and batch positive");
  *bytes = swin_workspace_bytes(desc, g, batch);
  return EVT_OK;
}

// The Swin workspace for B images (activation buffers only; lanes allocate their own)
static int swin_alloc_ws(evt_model* m, int B, hipStream_t s) {
  SwinGeo g;
  EVT_RC(validate_swin(&m->sdesc, &g));
  const SwinWs ws = swin_ws(g, B);
  const size_t es = elem_size(m->dtype);
  EVT_RC(dev_alloc(m, &m->x, (ws.stream + SWIN_SLACK) * es));
  EVT_RC(dev_alloc(m, &m->xm, (ws.stream + SWIN_SLACK) * es));
  EVT_HIP(hipMemsetAsync(m->x, 0, (ws.stream + SWIN_SLACK) * es, s), "memset x");
  EVT_HIP(hipMemsetAsync(m->xm, 0, (ws.stream + SWIN_SLACK) * es, s), "memset xm");
  EVT_RC(dev_alloc(m, (void**)&m->sx, ws.stats * sizeof(float)));
  EVT_RC(dev_alloc(m, (void**)&m->sm, ws.stats * sizeof(float)));
  EVT_RC(dev_alloc(m, &m->qkv, ws.qkv * es));
  EVT_RC(dev_alloc(m, &m->o, (ws.o + SWIN_SLACK) * es));
  EVT_HIP(hipMemsetAsync(m->o, 0, (ws.o + SWIN_SLACK) * es, s), "memset o");
  EVT_RC(dev_alloc(m, &m->hbuf, ws.hbuf * es));
  EVT_RC(dev_alloc(m, &m->pooled, ws.pooled * es));
  if (m->dtype == DT_BF16) {
    EVT_RC(dev_alloc(m, &m->sk, gemm_sk_bytes()));
    EVT_HIP(hipMemsetAsync(m->sk, 0, 4096, s), "memset stream-K flags");
  }
  m->ws_bytes = swin_workspace_bytes(&m->sdesc, g, B);
  return EVT_OK;
}

int evt_swin_create(const evt_swin_desc* desc, const float* const* w, int n_weights, void* stream,
                    evt_model** out) {
  if (!out) return fail(EVT_EINVAL, "out is NULL");
  *out = nullptr;
  SwinGeo g;
  EVT_RC(validate_swin(desc, &g));
  if (n_weights != evt_swin_num_weights(desc) || !w)
    return fail(EVT_EINVAL, "expected " + std::to_string(evt_swin_num_weights(desc)) + " weights");
  for (int i = 0; i < n_weights; ++i)
    if (!w[i]) return fail(EVT_EINVAL, "weight pointer " + std::to_string(i) + " is NULL");
  hipStream_t s = (hipStream_t)stream;
  evt_model* m = new evt_model();
  m->family = 2;
  m->dtype = desc->dtype;
  m->D = desc->embed_dim;
  m->max_batch = desc->max_batch;
  m->num_classes = desc->num_classes;
  m->sdesc = *desc;
  auto run = [&]() -> int {
    const int E = desc->embed_dim;
    int k = 0;
    EVT_RC(make_dense(m, &m->patch, w[0], w[1], g.pd, E, s));  // Conv2d(k = s = patch)
    EVT_RC(copy_vec(m, &m->pnorm_g, w[2], E, s));
    EVT_RC(copy_vec(m, &m->pnorm_b, w[3], E, s));
    k = 4;
    m->stages.resize(g.ns);
    for (int i = 0; i < g.ns; ++i) {
      SwinStage& st = m->stages[i];
      st.C = g.C[i];
      st.Cst = g.Cst[i];
      st.H = desc->num_heads[i];
      st.R = g.R[i];
      st.mlp = g.mlp[i];
      st.mst = g.mst[i];
      if (i > 0) {  // PatchMerging: LayerNorm(4C) folded into reduction Linear(4C, 2C, bias=False)
        EVT_RC(make_dense(m, &st.merge, w[k + 2], nullptr, 4 * g.C[i - 1], st.C, s, w[k], w[k + 1]));
        k += 3;
      }
      st.blocks.resize(desc->depths[i]);
      for (int j = 0; j < desc->depths[i]; ++j) {
        SwinBlock& bl = st.blocks[j];
        bl.shift = (j % 2 == 1 && st.R > 7) ? 3 : 0;  // SW-MSA on odd blocks; none at R == window
        const int C = st.C;
        EVT_RC(make_dense(m, &bl.qkv, w[k + 2], w[k + 3], C, 3 * C, s, w[k + 0], w[k + 1]));
        EVT_RC(dev_alloc(m, (void**)&bl.bias, rpb_table_floats(st.H, 7, bl.shift) * sizeof(float)));
        EVT_HIP(rpb_dense_launch(w[k + 4], st.H, 7, bl.shift, bl.bias, s), "relative position bias");
        EVT_RC(make_dense(m, &bl.proj, w[k + 5], w[k + 6], C, C, s));
        EVT_RC(make_dense(m, &bl.fc1, w[k + 9], w[k + 10], C, st.mlp, s, w[k + 7], w[k + 8]));
        EVT_RC(make_dense(m, &bl.fc2, w[k + 11], w[k + 12], st.mlp, C, s));
        k += 13;
      }
    }
    const int nf = g.C[g.ns - 1];
    EVT_RC(copy_vec(m, &m->norm_g, w[k + 0], nf, s));
    EVT_RC(copy_vec(m, &m->norm_b, w[k + 1], nf, s));
    EVT_RC(make_dense(m, &m->head, w[k + 2], w[k + 3], nf, desc->num_classes, s));
    EVT_RC(swin_alloc_ws(m, desc->max_batch, s));
    EVT_HIP(hipStreamSynchronize(s), "create sync");
    return EVT_OK;
  };
  return finish_create(m, run(), out);
}

int evt_swin_forward(evt_model* m, const float* img, int B, float* logits, void* stream) {
  if (!m || !img || !logits) return fail(EVT_EINVAL, "model, img and logits must be non-null");
  if (m->family != 2) return fail(EVT_EINVAL, "model is not a Swin Transformer");
  if (B <= 0 || B > m->max_batch)
    return fail(EVT_EINVAL, "batch must be in [1, max_batch=" + std::to_string(m->max_batch) + "]");
  hipStream_t s = (hipStream_t)stream;
  if (!m->lanes.empty() && !m->prof && B >= (int)m->lanes.size())  // profiling: one lane
    return lanes_forward(m, evt_swin_forward, img,
                         (size_t)m->sdesc.in_chans * m->sdesc.image_size * m->sdesc.image_size, B,
                         logits, s);
  prof_reset(m);
  const evt_swin_desc& d = m->sdesc;
  const int dt = d.dtype;
  const SwinStage& s0 = m->stages[0];
  const int pdst = (int)round_up(d.in_chans * d.patch_size * d.patch_size, PAD_K);
  const float scale_log2 = 0.17677669529663687f * 1.4426950408889634f;  // 32^-0.5 * log2(e)
  // patch embed: Conv2d(k = s = patch) as im2col + Dense, then its LayerNorm -> stream x + stats
  int rows = B * s0.R * s0.R;
  const double es = (double)elem_size(dt);
  const bool stem96 = dt == DT_BF16 && d.in_chans == 3 && d.patch_size == 4 && s0.C == 96 &&
                      s0.Cst == 96 && m->patch.kpad == 64 && d.image_size % 16 == 0 &&
                      d.image_size <= 256;
  if (stem96) {  // Conv2d + embedding LayerNorm in one kernel (swin.hip, swin_embed96_kernel)
    ProfScope ps(m, EVT_PROF_PATCH_EMBED, s);
    prof_work(m, 2.0 * rows * 96 * 48,
              (double)B * 3 * d.image_size * d.image_size * 4 + (double)rows * 96 * es +
                  (double)rows * stats_slots(96) * 8);
    SwinEmbedParams ep;
    ep.img = img; ep.w = m->patch.w; ep.ldw = m->patch.kpad; ep.bias = m->patch.b;
    ep.gamma = m->pnorm_g; ep.beta = m->pnorm_b; ep.x = m->x; ep.stats = m->sx;
    ep.B = B; ep.S = d.image_size; ep.nslots = stats_slots(96); ep.eps = 1e-5f;
    EVT_HIP(swin_embed96_launch(ep, s), "fused patch embedding");
  } else {
  {
    ProfScope ps(m, EVT_PROF_PATCHIFY, s);
    prof_work(m, 0.0, (double)B * d.in_chans * d.image_size * d.image_size * 4 +
                          (double)rows * d.in_chans * d.patch_size * d.patch_size * es);
    EVT_HIP(swin_patch_launch(dt, img, B, d.in_chans, d.image_size, d.patch_size, m->hbuf, pdst, s),
            "patch im2col");
  }
  {
    ProfScope ps(m, EVT_PROF_PATCH_EMBED, s);
    DenseCall c;
    c.flags = EPI_BIAS;
    c.A = m->hbuf; c.lda = pdst; c.C = m->xm; c.ldc = s0.Cst; c.M = rows; c.N = s0.Cst;
    EVT_RC(dense(m, m->patch, c, s));
    prof_work(m, 0.0, 2.0 * rows * s0.C * es + (double)rows * stats_slots(s0.C) * 8);
    EVT_HIP(ln_rows_launch(dt, m->xm, s0.Cst, m->x, m->pnorm_g, m->pnorm_b, rows, s0.C, 1e-5f,
                           m->sx, stats_slots(s0.C), s),
            "patch norm");
  }
  }
  for (size_t i = 0; i < m->stages.size(); ++i) {
    const SwinStage& st = m->stages[i];
    const int C = st.C, Cst = st.Cst;
    rows = B * st.R * st.R;
    if (i > 0) {  // PatchMerging: gather -> LN(4C)-folded reduction -> stream x (+ stats)
      const SwinStage& pv = m->stages[i - 1];
      ProfScope ps(m, EVT_PROF_MERGE, s);
      DenseCall c;
      c.flags = EPI_LNIN | EPI_BIAS | EPI_STATS;
      c.C = m->x; c.ldc = Cst; c.M = rows; c.N = Cst;
      c.stats_in = m->sm; c.stats_out = m->sx; c.ln_width = 4 * pv.C; c.slot_width = C;
      bool fused = false;
      if (dt == DT_BF16 && pv.Cst == pv.C && pv.R % 2 == 0) {
        // the gather inside the reduction GEMM's A loader (gemm.hip, EPI_GATHER): A = the old
        // stream, read in place, so the new stream goes to xm and the two buffers swap roles
        DenseCall g = c;
        g.flags |= EPI_GATHER;
        g.A = m->x; g.lda = pv.Cst; g.C = m->xm;
        GemmParams p = dense_params(m, st.merge, g);
        const int R2 = pv.R / 2;
        p.gmode = 1; p.gR = pv.R; p.gC = pv.C; p.gOW = R2;
        p.g_inv_rr = 1.0f / (float)(R2 * R2); p.g_inv_r = 1.0f / (float)R2;
        EVT_HIP(merge_stats_launch(m->sx, stats_slots(pv.C), B, pv.R, m->sm, stats_slots(C), s),
                "merge statistics");
        const hipError_t e = gemm_launch(dt, g.flags, p, s);
        if (e == hipSuccess) {
          c.A = m->x; c.lda = 4 * pv.C;  // (work accounting: the same A bytes, gathered)
          dense_work(m, st.merge, c);
          std::swap(m->x, m->xm);
          fused = true;
        } else if (e != hipErrorNotSupported) {
          EVT_HIP(e, "patch merge (gathered)");
        }
      }
      if (!fused) {
        prof_work(m, 0.0, 2.0 * rows * 4 * pv.C * es + (double)rows * stats_slots(C) * 8);
        EVT_HIP(merge_launch(dt, m->x, pv.Cst, B, pv.R, pv.C, m->hbuf, m->sm, stats_slots(C), s),
                "patch merge");
        c.A = m->hbuf; c.lda = 4 * pv.C;
        EVT_RC(dense(m, st.merge, c, s));
      }
    }
    for (const SwinBlock& bl : st.blocks) {
      const bool fuse96 = dt == DT_BF16 && C == 96 && st.H == 3 && gemm_auto();
      const double slot_rows = (double)rows * stats_slots(C) * 8;
      if (fuse96) {  // stage-1 attention sublayer fused (swin.hip, swin_attn96_kernel)
        ProfScope ps(m, EVT_PROF_ATTN_SUBLAYER, s);
        prof_work(m, 2.0 * rows * C * 4 * C + 4.0 * rows * 49 * C,
                  2.0 * rows * C * es + 2 * slot_rows + 4.0 * C * C * es);
        SwinAttnBlockParams ab{m->x, m->xm, m->sx, m->sm, bl.qkv.w, bl.qkv.b, bl.proj.w,
                               bl.proj.b, bl.bias, bl.qkv.kpad, bl.proj.kpad, B, st.R, bl.shift,
                               stats_slots(C), m->eps};
        EVT_HIP(swin_attn96_launch(ab, s), "fused window attention sublayer");
      }
      if (!fuse96) {  // LN1-folded QKV (+ bias)
        {
          ProfScope ps(m, EVT_PROF_QKV, s);
          DenseCall c;
          c.flags = EPI_LNIN | EPI_BIAS;
          c.A = m->x; c.lda = Cst; c.C = m->qkv; c.ldc = 3 * C; c.M = rows; c.N = 3 * C;
          c.stats_in = m->sx; c.ln_width = C;
          EVT_RC(dense(m, bl.qkv, c, s));
        }
        {
          ProfScope ps(m, EVT_PROF_ATTENTION, s);
          prof_work(m, 4.0 * rows * 49 * C, 4.0 * rows * C * es);  // 49 keys per query
          SwinAttnParams ap{m->qkv, 3 * C, m->o, Cst, bl.bias, B, st.R, st.R / 7, C, st.H,
                            bl.shift, scale_log2};
          EVT_HIP(window_attn_launch(dt, ap, s), "window attention");
        }
        ProfScope ps(m, EVT_PROF_OUT_PROJ, s);
        DenseCall pc;  // proj + bias + residual x -> xm (+ stats)
        pc.flags = EPI_BIAS | EPI_RESID | EPI_STATS;
        pc.A = m->o; pc.lda = Cst; pc.C = m->xm; pc.ldc = Cst; pc.M = rows; pc.N = Cst;
        pc.resid = m->x; pc.ldr = Cst; pc.stats_out = m->sm; pc.ln_width = C;
        EVT_RC(dense(m, bl.proj, pc, s));
      }
      if (dt == DT_BF16 && C == 96 && st.mlp == 384 && gemm_auto()) {
        // stage-1 MLP (C = 96) fused: hidden kept on chip (swin.hip, swin_mlp96_kernel)
        ProfScope ps(m, EVT_PROF_MLP, s);
        prof_work(m, 4.0 * rows * C * st.mlp, 2.0 * rows * C * es + 2 * slot_rows +
                                                   2.0 * C * st.mlp * es);
        SwinMlpParams mp{m->xm, m->x, m->sm, m->sx, bl.fc1.w, bl.fc1.colsum, bl.fc1.b,
                         bl.fc2.w, bl.fc2.b, bl.fc1.kpad, bl.fc2.kpad, rows, stats_slots(C),
                         m->eps};
        EVT_HIP(swin_mlp96_launch(mp, s), "fused MLP");
        continue;
      }
      {  // LN2-folded FC1 + erf GELU
        ProfScope ps(m, EVT_PROF_FC1, s);
        DenseCall c;
        c.flags = EPI_LNIN | EPI_BIAS | EPI_GELU_ERF;
        c.A = m->xm; c.lda = Cst; c.C = m->hbuf; c.ldc = st.mst; c.M = rows; c.N = st.mst;
        c.stats_in = m->sm; c.ln_width = C;
        EVT_RC(dense(m, bl.fc1, c, s));
      }
      {  // FC2 + bias + residual xm -> x (+ stats)
        ProfScope ps(m, EVT_PROF_FC2, s);
        DenseCall c;
        c.flags = EPI_BIAS | EPI_RESID | EPI_STATS;
        c.A = m->hbuf; c.lda = st.mst; c.C = m->x; c.ldc = Cst; c.M = rows; c.N = Cst;
        c.resid = m->xm; c.ldr = Cst; c.stats_out = m->sx; c.ln_width = C;
        EVT_RC(dense(m, bl.fc2, c, s));
      }
    }
  }
  // final LayerNorm + mean over tokens -> head Dense (fp32 logits)
  const SwinStage& sl = m->stages.back();
  ProfScope ps_head(m, EVT_PROF_HEAD, s);
  prof_work(m, 0.0, (double)B * sl.R * sl.R * sl.C * es + (double)B * sl.R * sl.R * stats_slots(sl.C) * 8 +
                        (double)B * sl.C * es);
  EVT_HIP(ln_pool_launch(dt, m->x, sl.Cst, B, sl.R * sl.R, sl.C, m->sx, stats_slots(sl.C),
                         m->norm_g, m->norm_b, m->pooled, sl.Cst, s),
          "norm + avgpool");
  {
    DenseCall c;
    c.flags = EPI_BIAS | EPI_OUT_F32;
    c.A = m->pooled; c.lda = sl.Cst; c.C = logits; c.ldc = d.num_classes; c.M = B;
    c.N = d.num_classes;
    EVT_RC(dense(m, m->head, c, s));
  }
  return EVT_OK;
}

int evt_window_attention(int dtype, const void* qkv, int64_t ldq, void* out, int64_t ldo,
                         const float* rpb, int B, int R, int C, int H, int shift, void* stream) {
  if (!qkv || !out || !rpb) return fail(EVT_EINVAL, "null pointer");
  if (dtype != EVT_DTYPE_F32 && dtype != EVT_DTYPE_BF16) return fail(EVT_EINVAL, "bad dtype");
  if (B < 0 || R <= 0 || R % 7 || H <= 0 || C != 32 * H || ldo < C || ldq < 3 * C || shift < 0 ||
      shift >= 7 || ldq % 8 || ldo % 4)
    return fail(EVT_EINVAL, "bad window-attention shape (R % 7 == 0, head size 32, 0 <= shift < 7)");
  hipStream_t s = (hipStream_t)stream;
  float* dense_bias = nullptr;
  EVT_HIP(hipMallocAsync((void**)&dense_bias, rpb_table_floats(H, 7, shift) * sizeof(float), s),
          "malloc bias");
  EVT_HIP(rpb_dense_launch(rpb, H, 7, shift, dense_bias, s), "relative position bias");
  SwinAttnParams ap{qkv, ldq, out, ldo, dense_bias, B, R, R / 7, C, H, shift,
                    0.17677669529663687f * 1.4426950408889634f};
  const hipError_t e = window_attn_launch(dtype, ap, s);
  (void)hipFreeAsync(dense_bias, s);
  EVT_HIP(e, "window attention");
  return EVT_OK;
}

int evt_patch_merge(int dtype, const void* x, int64_t ldx, int B, int R, int C, void* out,
                    float* stats, int nslots, void* stream) {
  if (!x || !out || !stats) return fail(EVT_EINVAL, "null pointer");
  if (dtype != EVT_DTYPE_F32 && dtype != EVT_DTYPE_BF16) return fail(EVT_EINVAL, "bad dtype");
  if (B < 0 || R <= 0 || R % 2 || C <= 0 || ldx < C || nslots <= 0 || nslots > 64)
    return fail(EVT_EINVAL, "bad patch-merge shape");
  EVT_HIP(merge_launch(dtype, x, ldx, B, R, C, out, stats, nslots, (hipStream_t)stream), "merge");
  return EVT_OK;
}

// ---- op-level entry points --------------------------------------------------------------

int evt_set_gemm_variant(int variant) {
  if (!gemm_variant_supported(variant))
    return fail(EVT_EINVAL, "variant must be 0, 1, 2, 6, 8, 9, 16, 30, 31 or 36 (lab builds: also "
                            "10, 11, 13, 15, 17-25, 106, 108)");
  gemm_set_variant(variant);
  return EVT_OK;
}

int evt_pack_weight(int dtype, const float* W, const float* row_scale, int K, int N, void* Wp,
                    int Kpad, int Npad, void* stream) {
  if (!W || !Wp || K <= 0 || N <= 0 || Kpad < K || Npad < N || Kpad % PAD_K || Npad % GEMM_BN)
    return fail(EVT_EINVAL, "pack: bad shape (Npad % 128, Kpad % 64, Kpad >= K, Npad >= N)");
  EVT_HIP(pack_weight(dtype, W, row_scale, K, N, Wp, Kpad, Npad, (hipStream_t)stream),
          "pack_weight");
  return EVT_OK;
}

int evt_mx8_quantize(int in_dtype, const void* x, int64_t ldx, int rows, int K, int Kpad, void* q,
                     int64_t ldq, uint32_t* scales, int64_t ld_s, void* stream) {
  if (!x || !q || !scales || rows < 0 || K <= 0 || K % 8 || Kpad < K || Kpad % 128 ||
      ldx < K || ldq < Kpad || ld_s < rows || ldq % 8 ||
      (in_dtype != EVT_DTYPE_F32 && in_dtype != EVT_DTYPE_BF16) ||
      ldx % (in_dtype == EVT_DTYPE_F32 ? 4 : 8))
    return fail(EVT_EINVAL, "mx8_quantize: bad shape (K % 8, Kpad % 128, aligned rows)");
  EVT_HIP(mx8_quantize_launch(in_dtype, x, ldx, rows, K, Kpad, q, ldq, scales, ld_s,
                              (hipStream_t)stream),
          "mx8_quantize");
  return EVT_OK;
}

int evt_mx8_pack_weight(const float* W, const float* row_scale, int K, int N, void* Wq, int Kpad,
                        int Npad, uint32_t* scales, void* stream) {
  if (!W || !Wq || !scales || K <= 0 || N <= 0 || Kpad < K || Npad < N || Kpad % 128 ||
      Npad % 128)
    return fail(EVT_EINVAL, "mx8_pack: bad shape (Kpad % 128, Npad % 128)");
  EVT_HIP(mx8_pack_launch(W, row_scale, K, N, Wq, Kpad, Npad, scales, (hipStream_t)stream),
          "mx8_pack");
  return EVT_OK;
}

int evt_dense_mx8(const evt_dense_mx8_args* a, void* stream) {
  if (!a || !a->A || !a->a_scales || !a->Wq || !a->w_scales || !a->C || a->M < 0 || a->N <= 0 ||
      a->N % 8 || a->N > a->Npad || a->Kpad <= 0 || a->Kpad % 128 || a->Npad % 128 ||
      a->lda < a->Kpad || a->lda % 16 || a->ld_as < a->M || a->ldc < a->N || a->ldc % 8)
    return fail(EVT_EINVAL, "dense_mx8: bad shape (N % 8, Kpad % 128, Npad % 128, lda % 16)");
  const int f = a->flags;
  if ((f & EPI_BIAS) && !a->bias) return fail(EVT_EINVAL, "dense_mx8: bias flag without bias");
  if ((f & EPI_RESID) && (!a->resid || a->ldr < a->N || a->ldr % 8))
    return fail(EVT_EINVAL, "dense_mx8: bad resid");
  if ((f & EPI_RESLN) && (!(f & EPI_RESID) || !a->rstats || !a->rgamma || !a->rbeta))
    return fail(EVT_EINVAL, "dense_mx8: LN residual needs resid, rstats, rgamma, rbeta");
  if (f & (EPI_LNIN | EPI_STATS | EPI_POS))
    return fail(EVT_EINVAL, "dense_mx8: unsupported flags");
  if ((f & EPI_OUT_MX8) && (!a->c_scales || a->N % 32 || a->ld_cs < a->M))
    return fail(EVT_EINVAL, "dense_mx8: MX8 output needs c_scales, N % 32, ld_cs >= M");
  Mx8GemmParams p{};
  p.A = (const uint8_t*)a->A; p.lda = a->lda; p.As = a->a_scales; p.ldas = a->ld_as;
  p.W = (const uint8_t*)a->Wq; p.ldw = a->Kpad; p.Ws = a->w_scales; p.ldws = a->Npad;
  p.C = a->C; p.ldc = a->ldc; p.Cs = a->c_scales; p.ldcs = a->ld_cs;
  p.M = a->M; p.N = a->N; p.K = a->Kpad;
  p.bias = a->bias; p.resid = a->resid; p.ldr = a->ldr;
  p.rstats = a->rstats; p.rgamma = a->rgamma; p.rbeta = a->rbeta;
  hipError_t e = gemm_mx8_launch(f, p, (hipStream_t)stream);
  if (e == hipErrorInvalidValue) return fail(EVT_EINVAL, "dense_mx8: unsupported flags");
  EVT_HIP(e, "dense_mx8");
  return EVT_OK;
}

int evt_mx8_layernorm(const void* x, int rows, int D, int Kpad, const float* gamma,
                      const float* beta, float eps, float* stats, void* q, uint32_t* scales,
                      void* stream) {
  if (!x || !gamma || !beta || !q || !scales || rows < 0 || D <= 0 || D % 8 || D > Kpad ||
      Kpad % 128 || Kpad > 1024 || !(eps > 0.f))
    return fail(EVT_EINVAL, "mx8_layernorm: bad shape (D % 8, D <= Kpad <= 1024, Kpad % 128)");
  if ((((uintptr_t)x | (uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)q) & 15) ||
      (((uintptr_t)scales | (uintptr_t)stats) & 7))
    return fail(EVT_EINVAL, "mx8_layernorm: misaligned pointer");
  EVT_HIP(ln_mx8_launch(x, rows, D, Kpad, gamma, beta, eps, stats, q, scales,
                        (hipStream_t)stream),
          "mx8_layernorm");
  return EVT_OK;
}

int evt_attention_mx8(const void* qkv, int64_t ldq, void* q8, int64_t ldq8, uint32_t* s8,
                      int64_t ld_s8, int B, int N, int H, float scale, void* stream) {
  if (!qkv || !q8 || !s8 || B < 0 || N <= 0 || N > 256 || H <= 0 || ldq < 3 * H * 64 ||
      ldq % 8 || ldq8 < H * 64 || ldq8 % 128 || ld_s8 < (int64_t)B * N || ld_s8 > INT32_MAX)
    return fail(EVT_EINVAL, "attention_mx8: bad shape (N <= 256, head size 64, ldq8 % 128)");
  AttnParams p{qkv, ldq, nullptr, 0, N, H, B, scale * 1.4426950408889634f};
  p.q8 = (uint8_t*)q8;
  p.s8 = s8;
  p.ldq8 = ldq8;
  p.rows8 = (int)ld_s8;
  EVT_HIP(attention_launch(DT_BF16, p, (hipStream_t)stream), "attention_mx8");
  return EVT_OK;
}

int evt_ln_fold(int dtype, const void* Wp, int Kpad, int Npad, const float* W, const float* beta,
                const float* bias, int K, int N, float* colsum, float* cvec, void* stream) {
  if (!Wp || !W || !beta || !colsum || !cvec || K <= 0 || N <= 0 || Kpad < K || Npad < N)
    return fail(EVT_EINVAL, "ln_fold: bad shape");
  EVT_HIP(ln_fold(dtype, Wp, Kpad, W, beta, bias, K, N, colsum, cvec, Npad, (hipStream_t)stream),
          "ln_fold");
  return EVT_OK;
}

int evt_dense(int dtype, const evt_dense_args* a, void* stream) {
  if (!a || !a->A || !a->Wp || !a->C || a->M < 0 || a->N <= 0 || a->N > a->Npad ||
      a->Kpad % PAD_K || a->Npad % GEMM_BN || a->lda < a->Kpad || a->ldc < a->N)
    return fail(EVT_EINVAL, "dense: bad shape");
  const int f = a->flags;
  if ((f & EPI_BIAS) && !a->bias) return fail(EVT_EINVAL, "dense: bias flag without bias");
  if ((f & EPI_RESID) && (!a->resid || a->ldr < a->N)) return fail(EVT_EINVAL, "dense: bad resid");
  if ((f & EPI_POS) && (!a->pos || a->P <= 0 || a->ldp < a->N || (a->resid && a->ldr < a->N)))
    return fail(EVT_EINVAL, "dense: bad pos");
  if ((f & EPI_LNIN) && (!a->colsum || !a->stats_in || a->ln_width <= 0))
    return fail(EVT_EINVAL, "dense: LN-in needs colsum, stats_in, ln_width");
  if ((f & EPI_RESLN) && (!a->rstats || !a->rgamma || !a->rbeta || a->ln_width <= 0))
    return fail(EVT_EINVAL, "dense: LN residual needs rstats, rgamma, rbeta, ln_width");
  if ((f & EPI_STATS) && !a->stats_out)
    return fail(EVT_EINVAL, "dense: stats flag without stats_out");
  GemmParams p{};
  p.A = a->A; p.lda = a->lda; p.W = a->Wp; p.ldw = a->Kpad; p.C = a->C; p.ldc = a->ldc;
  p.M = a->M; p.N = a->N; p.K = a->Kpad; p.ntiles = a->Npad / GEMM_BN;
  p.bias = a->bias; p.resid = a->resid; p.ldr = a->ldr; p.pos = a->pos; p.ldp = a->ldp; p.P = a->P;
  p.vec_ok = (a->ldc % 4 == 0) && (a->ldr % 4 == 0) && (a->ldp % 4 == 0);
  if (p.vec_ok && a->ldc % 8 == 0 && a->ldr % 8 == 0 && a->ldp % 8 == 0 &&
      (((uintptr_t)a->C | (uintptr_t)a->resid) & 15) == 0)
    p.vec_ok = 2;
  p.colsum = a->colsum; p.stats_in = a->stats_in; p.rstats = a->rstats;
  p.rgamma = a->rgamma; p.rbeta = a->rbeta; p.stats_out = a->stats_out;
  p.inv_d = a->ln_width > 0 ? 1.0f / (float)a->ln_width : 0.f;
  p.eps = a->ln_eps;
  p.nslots = a->ln_width > 0 ? stats_slots(a->ln_width) : 1;
  p.stats_step = a->stats_step;
  if (dtype == EVT_DTYPE_BF16) {  // op-level calls share one stream-K scratch (one stream at a time)
    static void* sk = nullptr;
    if (!sk) {
      EVT_HIP(hipMalloc(&sk, gemm_sk_bytes()), "hipMalloc stream-K scratch");
      EVT_HIP(hipMemset(sk, 0, 4096), "memset stream-K flags");
    }
    gemm_sk_bind(sk, p);
  }
  hipError_t e = gemm_launch(dtype, f, p, (hipStream_t)stream);
  if (e == hipErrorInvalidValue) return fail(EVT_EINVAL, "dense: unsupported flags/shape");
  EVT_HIP(e, "dense");
  return EVT_OK;
}

int evt_dense_splitk(int dtype, const evt_dense_args* a, int splits, float* partials,
                     void* stream) {
  if (!a || !a->A || !a->Wp || !a->C || !partials || a->M < 0 || a->N <= 0 || a->N > a->Npad ||
      a->Kpad % PAD_K || a->Npad % GEMM_BN || a->lda < a->Kpad || a->ldc < a->N)
    return fail(EVT_EINVAL, "dense_splitk: bad shape");
  if (a->flags & ~(EPI_BIAS | EPI_GELU | EPI_OUT_F32))
    return fail(EVT_EINVAL, "dense_splitk: flags must be a subset of BIAS | GELU | OUT_F32");
  if ((a->flags & EPI_BIAS) && !a->bias) return fail(EVT_EINVAL, "dense_splitk: bias flag without bias");
  if (splits < 1 || splits > 64 || a->Kpad % (splits * PAD_K))
    return fail(EVT_EINVAL, "dense_splitk: Kpad must be a multiple of splits * 64");
  GemmParams p{};
  p.A = a->A; p.lda = a->lda; p.W = a->Wp; p.ldw = a->Kpad; p.C = a->C; p.ldc = a->ldc;
  p.M = a->M; p.N = a->N; p.K = a->Kpad; p.ntiles = a->Npad / GEMM_BN; p.bias = a->bias;
  hipError_t e = gemm_splitk_launch(dtype, a->flags, p, splits, partials, (hipStream_t)stream);
  if (e == hipErrorInvalidValue) return fail(EVT_EINVAL, "dense_splitk: unsupported flags/shape");
  EVT_HIP(e, "dense_splitk");
  return EVT_OK;
}

int evt_attention_hd(int dtype, const void* qkv, int64_t ldq, void* out, int64_t ldo, int B,
                     int N, int H, int head_dim, float scale, void* stream) {
  if (!qkv || !out || B < 0 || N <= 0 || N > 256 || H <= 0 || head_dim <= 0 || head_dim > 128 ||
      ldq < 3 * (int64_t)H * head_dim || ldo < (int64_t)H * head_dim)
    return fail(EVT_EINVAL, "attention: bad shape (N <= 256, head size in [1, 128])");
  // vector accesses: 16-B loads of q / k / v rows when h_k is a multiple of 16 B, 4-element stores
  // of O when h_k % 4 == 0 (head size 64: the tuned kernels' 16-B loads and stores)
  const int64_t vec = dtype == DT_BF16 ? 8 : 4;
  const bool vload = head_dim % vec == 0, vstore = head_dim % 4 == 0;
  if (vload && (ldq % vec || ((uintptr_t)qkv & 15)))
    return fail(EVT_EINVAL, "attention: qkv rows must be 16-B aligned for this head size");
  if ((vstore || head_dim == 64) && (ldo % (head_dim == 64 ? vec : 4) || ((uintptr_t)out & 15)))
    return fail(EVT_EINVAL, "attention: out rows must be 16-B aligned for this head size");
  AttnParams p{qkv, ldq, out, ldo, N, H, B, scale * 1.4426950408889634f};
  p.hd = head_dim;
  EVT_HIP(attention_launch(dtype, p, (hipStream_t)stream), "attention");
  return EVT_OK;
}

int evt_attention(int dtype, const void* qkv, int64_t ldq, void* out, int64_t ldo, int B, int N,
                  int H, float scale, void* stream) {
  // 16-B Q / O accesses: row pitches of 16 bytes multiple, 16-B aligned bases
  const int64_t vec = dtype == DT_BF16 ? 8 : 4;
  if (!qkv || !out || B < 0 || N <= 0 || N > 256 || H <= 0 || ldq < 3 * H * 64 || ldo < H * 64 ||
      ldq % vec || ldo % vec || (((uintptr_t)qkv | (uintptr_t)out) & 15))
    return fail(EVT_EINVAL, "attention: bad shape (N <= 256, head size 64, 16-B aligned rows)");
  AttnParams p{qkv, ldq, out, ldo, N, H, B, scale * 1.4426950408889634f};
  EVT_HIP(attention_launch(dtype, p, (hipStream_t)stream), "attention");
  return EVT_OK;
}

int evt_layernorm(int dtype, const float* x, int64_t ldx, void* y, int64_t ldy,
                  const float* gamma, const float* beta, int rows, int D, float eps,
                  void* stream) {
  if (!x || !y || !gamma || !beta || rows < 0 || D <= 0 || D > 1024 || D % 4 || ldx < D || ldy < D)
    return fail(EVT_EINVAL, "layernorm: bad shape (D % 4 == 0, D <= 1024)");
  EVT_HIP(layernorm_launch(dtype, x, ldx, y, ldy, gamma, beta, rows, D, eps, (hipStream_t)stream),
          "layernorm");
  return EVT_OK;
}

int evt_patchify(int dtype, const float* img, int B, int C, int HW, int ps, void* out, void* x,
                 const float* cls, const float* pos, int D, float* stats, void* stream) {
  if (!img || !out || !x || !cls || !pos || B < 0 || C <= 0 || ps <= 0 || HW % ps)
    return fail(EVT_EINVAL, "patchify: bad shape");
  EVT_HIP(patchify_launch(dtype, img, B, C, HW, ps, out, x, cls, pos, D, stats,
                          (hipStream_t)stream),
          "patchify");
  return EVT_OK;
}

int evt_patchify_cm(int dtype, const float* img, int B, int C, int HW, int ps, void* out, void* x,
                    const float* cls, const float* pos, int D, float* stats, void* stream) {
  if (!img || !out || !x || !cls || !pos || B < 0 || C <= 0 || ps <= 0 || HW % ps || ps % 8)
    return fail(EVT_EINVAL, "patchify_cm: bad shape (ps % 8 == 0)");
  EVT_HIP(patchify_launch(dtype, img, B, C, HW, ps, out, x, cls, pos, D, stats,
                          (hipStream_t)stream, true),
          "patchify_cm");
  return EVT_OK;
}

int evt_unfold(int dtype, int in_f32, const void* in, int B, int H, int W, int C, int k,
               int stride, int pad, void* out, int ldo, float* stats, int nslots, void* stream) {
  if (!in || !out || B < 0 || H <= 0 || W <= 0 || C <= 0 || k <= 0 || stride <= 0 || pad < 0 ||
      H + 2 * pad < k || W + 2 * pad < k || ldo < k * k * C || (stats && nslots <= 0) ||
      ldo > ((C % 4 == 0 && ldo % 4 == 0) ? 1024 : (ldo % 2 == 0 ? 512 : 256)))
    return fail(EVT_EINVAL, "unfold: bad shape (ldo <= 256; <= 512 if even; <= 1024 if C % 4 == 0)");
  if (dtype == EVT_DTYPE_F32 && !in_f32) return fail(EVT_EINVAL, "unfold: f32 path needs f32 input");
  EVT_HIP(unfold_launch(dtype, in_f32, in, B, H, W, C, k, stride, pad, out, ldo, stats, nslots,
                        (hipStream_t)stream),
          "unfold");
  return EVT_OK;
}

int64_t evt_performer_scratch(int B, int T) {
  if (B <= 0 || T <= 0) return 0;
  return (int64_t)performer_part_floats(B, T);
}

int evt_performer(int dtype, const void* kqv, int64_t ldq, int B, int T, const float* w,
                  const float* out_w, const float* out_b, const float* ln2_g, const float* ln2_b,
                  const float* fc1_w, const float* fc1_b, const float* fc2_w, const float* fc2_b,
                  float* part, void* out, int64_t ldo, void* stream) {
  if (!kqv || !w || !out_w || !out_b || !ln2_g || !ln2_b || !fc1_w || !fc1_b || !fc2_w ||
      !fc2_b || !part || !out || B < 0 || T <= 0 || ldq < 192 || ldo < 64 || ldq % 4 || ldo % 4)
    return fail(EVT_EINVAL, "performer: bad arguments (ldq >= 192, ldo >= 64, multiples of 4)");
  PerformerWeights pw{w, out_w, out_b, ln2_g, ln2_b, fc1_w, fc1_b, fc2_w, fc2_b};
  EVT_HIP(performer_launch(dtype, kqv, ldq, B, T, pw, part, out, ldo, (hipStream_t)stream),
          "performer");
  return EVT_OK;
}

}  // extern "C"
