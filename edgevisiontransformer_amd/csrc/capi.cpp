// C ABI of libevt_hip.so (declared in include/evt.h): model plumbing around the HIP kernels.
//
// The model handle owns the packed weights (kernel operand layout, zero padded) and one
// workspace sized for max_batch; evt_vit_forward enqueues the whole ViT forward of reference
// `modeling/models/vit.py:41-55` on the caller's stream with no host synchronisation.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
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

#define EVT_HIP(call, what)                          \
  do {                                               \
    hipError_t e__ = (call);                         \
    if (e__ != hipSuccess) return hip_fail(e__, what); \
  } while (0)

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
inline size_t elem_size(int dtype) { return dtype == DT_BF16 ? 2 : 4; }

struct DenseW {  // packed Dense layer
  void* w = nullptr;      // [npad][kpad] activation dtype
  float* b = nullptr;     // [npad] fp32, zero padded (may be null)
  int K = 0, N = 0, kpad = 0, npad = 0;
};

struct Layer {
  int heads = 0, inner = 0, ffn = 0, ffn_st = 0;
  float *ln1_g = nullptr, *ln1_b = nullptr, *ln2_g = nullptr, *ln2_b = nullptr;
  DenseW qkv, out, fc1, fc2;
};

struct Shape {
  int P = 0, T = 0, pd = 0, D = 0, max_inner = 0, max_ffn_st = 0, head_st = 0;
};

}  // namespace

struct evt_model {
  evt_vit_desc desc{};
  std::vector<int32_t> heads, head_dim, ffn;
  Shape sh;
  DenseW patch, head1, head2;
  float *cls = nullptr, *pos = nullptr;
  std::vector<Layer> layers;
  std::vector<void*> allocs;
  // workspace
  void* apatch = nullptr;  // [B*P, pd]      (aliases hbuf)
  float* x = nullptr;      // [B*T, D] fp32 token stream (pre-LN sum)
  void* y = nullptr;       // [B*T, D]       LN output = GEMM input = residual
  void* qkv = nullptr;     // [B*T, 3*inner]
  void* o = nullptr;       // [B*T, inner]
  void* hbuf = nullptr;    // [B*T, ffn_st]
  void* t = nullptr;       // [B, D]
  void* hh = nullptr;      // [B, head_st]
  size_t ws_bytes = 0;
};

namespace {

int dev_alloc(evt_model* m, void** p, size_t bytes) {
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) return fail(EVT_ENOMEM, std::string("hipMalloc failed: ") + hipGetErrorString(e));
  m->allocs.push_back(*p);
  return EVT_OK;
}

int validate(const evt_vit_desc* d, Shape* sh) {
  if (!d) return fail(EVT_EINVAL, "desc is NULL");
  if (d->dtype != EVT_DTYPE_F32 && d->dtype != EVT_DTYPE_BF16)
    return fail(EVT_EINVAL, "dtype must be EVT_DTYPE_F32 or EVT_DTYPE_BF16");
  if (d->patch_size <= 0 || d->image_size <= 0 || d->image_size % d->patch_size != 0)
    return fail(EVT_EINVAL, "image dimensions must be divisible by the patch size");
  if (d->in_chans <= 0 || d->num_classes <= 0 || d->depth < 0 || d->mlp_dim <= 0)
    return fail(EVT_EINVAL, "in_chans, num_classes, mlp_dim must be positive, depth >= 0");
  if (d->dim <= 0 || d->dim % 64 != 0 || d->dim > 1024)
    return fail(EVT_EINVAL, "dim must be a positive multiple of 64 and <= 1024");
  if (d->max_batch <= 0) return fail(EVT_EINVAL, "max_batch must be positive");
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
    if (d->head_dim[i] != 64) return fail(EVT_EINVAL, "head size must be 64 in this build");
    if (d->ffn[i] <= 0) return fail(EVT_EINVAL, "ffn width per layer must be positive");
    sh->max_inner = std::max(sh->max_inner, d->heads[i] * 64);
    sh->max_ffn_st = std::max<int>(sh->max_ffn_st, (int)round_up(d->ffn[i], PAD_N));
  }
  sh->head_st = (int)round_up(d->mlp_dim, PAD_N);
  return EVT_OK;
}

int make_dense(evt_model* m, DenseW* dw, const float* W, const float* b, int K, int N,
               hipStream_t s) {
  const int dt = m->desc.dtype;
  dw->K = K;
  dw->N = N;
  dw->kpad = (int)round_up(K, PAD_K);
  dw->npad = (int)round_up(N, PACK_N);
  int rc = dev_alloc(m, &dw->w, (size_t)dw->kpad * dw->npad * elem_size(dt));
  if (rc) return rc;
  EVT_HIP(pack_weight(dt, W, K, N, dw->w, dw->kpad, dw->npad, s), "pack_weight");
  if (b) {
    rc = dev_alloc(m, (void**)&dw->b, (size_t)dw->npad * sizeof(float));
    if (rc) return rc;
    EVT_HIP(hipMemsetAsync(dw->b, 0, (size_t)dw->npad * sizeof(float), s), "memset bias");
    EVT_HIP(hipMemcpyAsync(dw->b, b, (size_t)N * sizeof(float), hipMemcpyDeviceToDevice, s),
            "copy bias");
  }
  return EVT_OK;
}

int copy_vec(evt_model* m, float** dst, const float* src, size_t n, hipStream_t s) {
  int rc = dev_alloc(m, (void**)dst, n * sizeof(float));
  if (rc) return rc;
  EVT_HIP(hipMemcpyAsync(*dst, src, n * sizeof(float), hipMemcpyDeviceToDevice, s), "copy vec");
  return EVT_OK;
}

size_t workspace_bytes(const evt_vit_desc* d, const Shape& sh, int B) {
  const size_t es = elem_size(d->dtype);
  const size_t rows = (size_t)B * sh.T;
  const size_t hb = std::max(rows * sh.max_ffn_st, (size_t)B * sh.P * sh.pd) * es;
  return rows * sh.D * 4 + rows * sh.D * es + rows * 3 * sh.max_inner * es +
         rows * sh.max_inner * es + hb + (size_t)B * sh.D * es + (size_t)B * sh.head_st * es +
         8 * 256;
}

int dense(const evt_model* m, int flags, const DenseW& w, const void* A, int64_t lda, void* C,
          int64_t ldc, int M, int N, const void* resid, int64_t ldr, const float* pos,
          int64_t ldp, int P, hipStream_t s) {
  GemmParams p{};
  p.A = A;
  p.lda = lda;
  p.W = w.w;
  p.ldw = w.kpad;
  p.C = C;
  p.ldc = ldc;
  p.M = M;
  p.N = N;
  p.K = w.kpad;
  p.ntiles = w.npad / GEMM_BN;
  p.bias = w.b;
  p.resid = resid;
  p.ldr = ldr;
  p.pos = pos;
  p.ldp = ldp;
  p.P = P;
  p.vec_ok = (ldc % 4 == 0) && (ldr % 4 == 0) && (ldp % 4 == 0);
  EVT_HIP(gemm_launch(m->desc.dtype, flags, p, s), "dense");
  return EVT_OK;
}

#define EVT_RC(x)        \
  do {                   \
    int rc__ = (x);      \
    if (rc__) return rc__; \
  } while (0)

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
  return 4 + 11 * desc->depth + 4;
}

int evt_query_workspace(const evt_vit_desc* desc, int batch, size_t* bytes) {
  Shape sh;
  EVT_RC(validate(desc, &sh));
  if (!bytes || batch <= 0) return fail(EVT_EINVAL, "bytes must be non-null and batch positive");
  *bytes = workspace_bytes(desc, sh, batch);
  return EVT_OK;
}

int evt_model_destroy(evt_model* m) {
  if (!m) return EVT_OK;
  for (void* p : m->allocs) (void)hipFree(p);
  delete m;
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
  m->desc = *desc;
  m->heads.assign(desc->heads, desc->heads + desc->depth);
  m->head_dim.assign(desc->head_dim, desc->head_dim + desc->depth);
  m->ffn.assign(desc->ffn, desc->ffn + desc->depth);
  m->desc.heads = m->heads.data();
  m->desc.head_dim = m->head_dim.data();
  m->desc.ffn = m->ffn.data();
  m->sh = sh;
  const int D = desc->dim;
  int k = 0;
  auto run = [&]() -> int {
    EVT_RC(make_dense(m, &m->patch, w[0], w[1], sh.pd, D, s));
    EVT_RC(copy_vec(m, &m->cls, w[2], D, s));
    EVT_RC(copy_vec(m, &m->pos, w[3], (size_t)sh.T * D, s));
    k = 4;
    m->layers.resize(desc->depth);
    for (int i = 0; i < desc->depth; ++i) {
      Layer& L = m->layers[i];
      L.heads = desc->heads[i];
      L.inner = L.heads * 64;
      L.ffn = desc->ffn[i];
      L.ffn_st = (int)round_up(L.ffn, PAD_N);
      EVT_RC(copy_vec(m, &L.ln1_g, w[k + 0], D, s));
      EVT_RC(copy_vec(m, &L.ln1_b, w[k + 1], D, s));
      EVT_RC(make_dense(m, &L.qkv, w[k + 2], nullptr, D, 3 * L.inner, s));
      EVT_RC(make_dense(m, &L.out, w[k + 3], w[k + 4], L.inner, D, s));
      EVT_RC(copy_vec(m, &L.ln2_g, w[k + 5], D, s));
      EVT_RC(copy_vec(m, &L.ln2_b, w[k + 6], D, s));
      EVT_RC(make_dense(m, &L.fc1, w[k + 7], w[k + 8], D, L.ffn, s));
      EVT_RC(make_dense(m, &L.fc2, w[k + 9], w[k + 10], L.ffn, D, s));
      k += 11;
    }
    EVT_RC(make_dense(m, &m->head1, w[k + 0], w[k + 1], D, desc->mlp_dim, s));
    EVT_RC(make_dense(m, &m->head2, w[k + 2], w[k + 3], desc->mlp_dim, desc->num_classes, s));
    // workspace
    const int B = desc->max_batch;
    const size_t es = elem_size(desc->dtype);
    const size_t rows = (size_t)B * sh.T;
    EVT_RC(dev_alloc(m, (void**)&m->x, rows * D * 4));
    EVT_RC(dev_alloc(m, &m->y, rows * D * es));
    EVT_RC(dev_alloc(m, &m->qkv, rows * 3 * sh.max_inner * es));
    EVT_RC(dev_alloc(m, &m->o, rows * sh.max_inner * es));
    EVT_RC(dev_alloc(m, &m->hbuf, std::max(rows * sh.max_ffn_st, (size_t)B * sh.P * sh.pd) * es));
    m->apatch = m->hbuf;
    EVT_RC(dev_alloc(m, &m->t, (size_t)B * D * es));
    EVT_RC(dev_alloc(m, &m->hh, (size_t)B * sh.head_st * es));
    m->ws_bytes = workspace_bytes(desc, sh, B);
    EVT_HIP(hipStreamSynchronize(s), "create sync");
    return EVT_OK;
  };
  int rc = run();
  if (rc) {
    std::string keep = g_err;
    evt_model_destroy(m);
    g_err = keep;
    return rc;
  }
  *out = m;
  return EVT_OK;
}

int evt_vit_forward(evt_model* m, const float* img, int B, float* logits, void* stream) {
  if (!m || !img || !logits) return fail(EVT_EINVAL, "model, img and logits must be non-null");
  if (B <= 0 || B > m->desc.max_batch)
    return fail(EVT_EINVAL, "batch must be in [1, max_batch=" + std::to_string(m->desc.max_batch) + "]");
  hipStream_t s = (hipStream_t)stream;
  const evt_vit_desc& d = m->desc;
  const Shape& sh = m->sh;
  const int D = d.dim, T = sh.T, rows = B * T, dt = d.dtype;
  // patch embedding: rearrange -> Dense(D) (+pos, rows 1..P) ; CLS row = cls + pos[0]
  EVT_HIP(patchify_launch(dt, img, B, d.in_chans, d.image_size, d.patch_size, m->apatch, m->x,
                          m->cls, m->pos, D, s),
          "patchify");
  EVT_RC(dense(m, EPI_BIAS | EPI_POS | EPI_OUT_F32, m->patch, m->apatch, sh.pd, m->x, D, B * sh.P,
               D, nullptr, 0, m->pos, D, sh.P, s));
  const float log2e = 1.4426950408889634f;
  for (const Layer& L : m->layers) {
    // LayerNorm(Residual(Attention), pre=True): y = LN(x); x = Attn(y) + y
    EVT_HIP(layernorm_launch(dt, m->x, D, m->y, D, L.ln1_g, L.ln1_b, rows, D, 1e-5f, s), "ln1");
    EVT_RC(dense(m, 0, L.qkv, m->y, D, m->qkv, 3 * L.inner, rows, 3 * L.inner, nullptr, 0, nullptr,
                 0, 0, s));
    AttnParams ap{m->qkv, 3 * L.inner, m->o, L.inner, T, L.heads, B, 0.125f * log2e};
    EVT_HIP(attention_launch(dt, ap, s), "attention");
    EVT_RC(dense(m, EPI_BIAS | EPI_RESID | EPI_OUT_F32, L.out, m->o, L.inner, m->x, D, rows, D,
                 m->y, D, nullptr, 0, 0, s));
    // LayerNorm(Residual(FeedForward), pre=True): y = LN(x); x = FFN(y) + y
    EVT_HIP(layernorm_launch(dt, m->x, D, m->y, D, L.ln2_g, L.ln2_b, rows, D, 1e-5f, s), "ln2");
    EVT_RC(dense(m, EPI_BIAS | EPI_GELU, L.fc1, m->y, D, m->hbuf, L.ffn_st, rows, L.ffn_st,
                 nullptr, 0, nullptr, 0, 0, s));
    EVT_RC(dense(m, EPI_BIAS | EPI_RESID | EPI_OUT_F32, L.fc2, m->hbuf, L.ffn_st, m->x, D, rows, D,
                 m->y, D, nullptr, 0, 0, s));
  }
  // head on token 0: Dense(M, gelu) -> Dense(C)  (no final LayerNorm in ViT, vit.py:54-55)
  EVT_HIP(gather_cls_launch(dt, m->x, (int64_t)T * D, B, D, m->t, s), "gather_cls");
  EVT_RC(dense(m, EPI_BIAS | EPI_GELU, m->head1, m->t, D, m->hh, sh.head_st, B, sh.head_st,
               nullptr, 0, nullptr, 0, 0, s));
  EVT_RC(dense(m, EPI_BIAS | EPI_OUT_F32, m->head2, m->hh, sh.head_st, logits, d.num_classes, B,
               d.num_classes, nullptr, 0, nullptr, 0, 0, s));
  return EVT_OK;
}

// ---- op-level entry points --------------------------------------------------------------

int evt_set_gemm_variant(int variant) {
  if (variant < 0 || variant > 31) return fail(EVT_EINVAL, "variant must be 0..31");
  gemm_set_variant(variant);
  return EVT_OK;
}

int evt_pack_weight(int dtype, const float* W, int K, int N, void* Wp, int Kpad, int Npad,
                    void* stream) {
  if (!W || !Wp || K <= 0 || N <= 0 || Kpad < K || Npad < N || Kpad % PAD_K || Npad % GEMM_BN)
    return fail(EVT_EINVAL, "pack: bad shape (Npad % 128, Kpad % 64, Kpad >= K, Npad >= N)");
  EVT_HIP(pack_weight(dtype, W, K, N, Wp, Kpad, Npad, (hipStream_t)stream), "pack_weight");
  return EVT_OK;
}

int evt_dense(int dtype, int flags, const void* A, int64_t lda, const void* Wp, int Kpad, int Npad,
              void* C, int64_t ldc, int M, int N, const float* bias, const void* resid,
              int64_t ldr, const float* pos, int64_t ldp, int P, void* stream) {
  if (!A || !Wp || !C || M < 0 || N <= 0 || N > Npad || Kpad % PAD_K || Npad % GEMM_BN ||
      lda < Kpad || ldc < N)
    return fail(EVT_EINVAL, "dense: bad shape");
  if ((flags & EPI_BIAS) && !bias) return fail(EVT_EINVAL, "dense: bias flag without bias");
  if ((flags & EPI_RESID) && (!resid || ldr < N)) return fail(EVT_EINVAL, "dense: bad resid");
  if ((flags & EPI_POS) && (!pos || P <= 0 || ldp < N)) return fail(EVT_EINVAL, "dense: bad pos");
  GemmParams p{};
  p.A = A; p.lda = lda; p.W = Wp; p.ldw = Kpad; p.C = C; p.ldc = ldc;
  p.M = M; p.N = N; p.K = Kpad; p.ntiles = Npad / GEMM_BN;
  p.bias = bias; p.resid = resid; p.ldr = ldr; p.pos = pos; p.ldp = ldp; p.P = P;
  p.vec_ok = (ldc % 4 == 0) && (ldr % 4 == 0) && (ldp % 4 == 0);
  hipError_t e = gemm_launch(dtype, flags, p, (hipStream_t)stream);
  if (e == hipErrorInvalidValue) return fail(EVT_EINVAL, "dense: unsupported flags/shape");
  EVT_HIP(e, "dense");
  return EVT_OK;
}

int evt_attention(int dtype, const void* qkv, int64_t ldq, void* out, int64_t ldo, int B, int N,
                  int H, float scale, void* stream) {
  if (!qkv || !out || B < 0 || N <= 0 || N > 256 || H <= 0 || ldq < 3 * H * 64 || ldo < H * 64)
    return fail(EVT_EINVAL, "attention: bad shape (N <= 256, head size 64)");
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

int evt_patchify(int dtype, const float* img, int B, int C, int HW, int ps, void* out, float* x,
                 const float* cls, const float* pos, int D, void* stream) {
  if (!img || !out || !x || !cls || !pos || B < 0 || C <= 0 || ps <= 0 || HW % ps)
    return fail(EVT_EINVAL, "patchify: bad shape");
  EVT_HIP(patchify_launch(dtype, img, B, C, HW, ps, out, x, cls, pos, D, (hipStream_t)stream),
          "patchify");
  return EVT_OK;
}

}  // extern "C"
