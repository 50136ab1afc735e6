"""Round-6 reference point: the same DeiT-base/16-224 forward (the reference ViT's structure:
patchify (p1 p2 c) -> Dense 768 -> CLS + pos -> 12 x [LN1 -> qkv -> attention -> out-proj,
f(LN x) + LN x residual; LN2 -> FC1 -> tanh GELU -> FC2, same residual] -> LN -> head) written in
plain PyTorch-ROCm bf16 (F.linear = hipBLASLt, scaled_dot_product_attention = the flash
backend), eager and captured in a HIP graph, against the product library's evt_vit_forward on the
same box. Random weights, synthetic images; images / s over 20 forwards after 3 warm-up ones.
    python scripts/probe/torch_deit_bench.py [batch]"""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from edgevisiontransformer_amd.modeling.models import vit  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
D, H, L, P, FF, NC = 768, 12, 12, 16, 3072, 1000
N = (224 // P) ** 2 + 1
dev, dt = "cuda", torch.bfloat16
g = torch.Generator(device=dev).manual_seed(0)


def rnd(*shape, s=0.02):
    return (torch.randn(shape, generator=g, device=dev) * s).to(dt)


Wp, bp = rnd(D, 3 * P * P), rnd(D)
cls, pos = rnd(1, 1, D), rnd(1, N, D)
layers = [dict(ln1=(torch.ones(D, device=dev, dtype=dt), rnd(D)), qkv=(rnd(3 * D, D), rnd(3 * D)),
               o=(rnd(D, D), rnd(D)), ln2=(torch.ones(D, device=dev, dtype=dt), rnd(D)),
               f1=(rnd(FF, D), rnd(FF)), f2=(rnd(D, FF), rnd(D))) for _ in range(L)]
lnf, head = (torch.ones(D, device=dev, dtype=dt), rnd(D)), (rnd(NC, D), rnd(NC))


def forward(img):
    x = img.to(dt).view(B, 3, 14, P, 14, P).permute(0, 2, 4, 3, 5, 1).reshape(B, N - 1, 3 * P * P)
    x = F.linear(x, Wp, bp)
    x = torch.cat([cls.expand(B, 1, D), x], 1) + pos
    for ly in layers:
        y = F.layer_norm(x, (D,), *ly["ln1"], eps=1e-6)
        q, k, v = F.linear(y, *ly["qkv"]).view(B, N, 3, H, D // H).permute(2, 0, 3, 1, 4)
        a = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, N, D)
        x = F.linear(a, *ly["o"]) + y
        y = F.layer_norm(x, (D,), *ly["ln2"], eps=1e-6)
        x = F.linear(F.gelu(F.linear(y, *ly["f1"]), approximate="tanh"), *ly["f2"]) + y
    x = F.layer_norm(x[:, 0], (D,), *lnf, eps=1e-6)
    return F.linear(x, *head).float()


def rate(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return B * 20 / (e0.elapsed_time(e1) / 1e3)


img = torch.randn((B, 3, 224, 224), generator=g, device=dev)
res = {"batch": B}
with torch.no_grad():
    res["torch_eager_img_s"] = round(rate(lambda: forward(img)))
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        forward(img)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        forward(img)
    res["torch_graph_img_s"] = round(rate(graph.replay))
    m = vit.build_named("deit_base", dtype="bf16", seed=0, max_batch=B)
    res["product_img_s"] = round(rate(lambda: m(img)))
print(json.dumps(res), flush=True)
