"""DeiT-base bs512 forward: EVT_DTYPE_MX8 vs bf16 in one process (images/s, synthetic inputs in HBM)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from edgevisiontransformer_amd.modeling.models import vit  # noqa: E402


def run(dtype, B=512, steps=10, warmup=3):
    m = vit.get_deit_base(dtype=dtype, seed=0, max_batch=B)
    g = torch.Generator(device="cuda").manual_seed(0)
    img = torch.randn((B, 3, 224, 224), generator=g, device="cuda")
    logits = torch.empty((B, 1000), device="cuda")
    for _ in range(warmup):
        m.forward_into(img, logits)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        m.forward_into(img, logits)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    out = logits.clone()
    del m
    torch.cuda.empty_cache()
    return ms, out


ms8, l8 = run("mx8")
msb, lb = run("bf16")
cos = torch.nn.functional.cosine_similarity(l8, lb, dim=1).min().item()
print(json.dumps({"workload": "deit_base bs512 forward", "mx8_ms": round(ms8, 3),
                  "mx8_img_s": round(512 / ms8 * 1e3, 1), "bf16_ms": round(msb, 3),
                  "bf16_img_s": round(512 / msb * 1e3, 1), "min_row_cosine_mx8_vs_bf16": round(cos, 5)}))
