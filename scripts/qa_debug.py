"""Locate fused / unfused QKV + attention mismatches by batch size, image and head."""
import math
import sys

import torch

sys.path.insert(0, ".")
from edgevisiontransformer_amd import _lib  # noqa: E402
from tests import _ops  # noqa: E402

_lib.ensure_device(0)
N, H, D = 197, 12, 768
for B in (2, 16, 64, 512):
    g = torch.Generator(device="cuda").manual_seed(0)
    x = (torch.randn((B * N, D), generator=g, device="cuda") * 1.3 + 0.3).bfloat16()
    W = torch.randn((D, 3 * H * 64), generator=g, device="cuda") / math.sqrt(D)
    gam = 1 + 0.1 * torch.randn(D, generator=g, device="cuda")
    bet = 0.1 * torch.randn(D, generator=g, device="cuda")
    wp, kpad, npad = _ops.pack(W, "bf16", row_scale=gam)
    colsum, cvec = _ops.ln_fold("bf16", wp, kpad, npad, W, bet)
    st = torch.zeros((B * N, 6, 2), device="cuda")
    xf = x.float()
    st[:, 0, 0], st[:, 0, 1] = xf.sum(-1), (xf * xf).sum(-1)
    out = _ops.qkv_attention(x, st, wp, colsum, cvec, B, N, H)
    qkv = _ops.dense("bf16", _lib.EPI_LNIN | _lib.EPI_BIAS, x, wp, kpad, npad, B * N, 3 * H * 64,
                     bias=cvec, colsum=colsum, stats_in=st, ln_width=D)
    ref = _ops.attention("bf16", qkv, B, N, H)
    torch.cuda.synchronize()
    d = (out.float() - ref.float()).abs().reshape(B, N, H, 64)
    per = d.amax(dim=(1, 3))  # [B, H]
    bad = (per > 0.05).nonzero()
    rows = d.amax(dim=(0, 2, 3))
    print(B, "max", d.max().item(), "bad (img, head) pairs", bad.shape[0], bad[:8].tolist(),
          "bad token rows", (rows > 0.05).nonzero().flatten()[:20].tolist(), flush=True)
