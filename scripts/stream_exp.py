"""Experiment: the bs=512 (argv[2]) DeiT-base batch as S concurrent sub-batches on S HIP streams (one model
handle each), so that one sub-batch's GEMM tails / memory-bound kernels overlap another's work.
Interleaved rounds in one process; images/s per configuration."""
import sys
import time

import torch

sys.path.insert(0, ".")
from edgevisiontransformer_amd.modeling.models import vit as mod  # noqa: E402

B = int(sys.argv[2]) if len(sys.argv) > 2 else 512
g = torch.Generator(device="cuda").manual_seed(1)
img = torch.randn((B, 3, 224, 224), generator=g, device="cuda")
logits = torch.empty((B, 1000), device="cuda")
cfgs = [int(s) for s in (sys.argv[1] if len(sys.argv) > 1 else "1,2,4").split(",")]
models = {S: [mod.build_named("deit_base", dtype="bf16", seed=0, max_batch=B // S) for _ in range(S)]
          for S in cfgs}
streams = {S: [torch.cuda.Stream() for _ in range(S)] for S in cfgs}
ref = None


def step(S):
    cur = torch.cuda.current_stream()
    b = B // S
    for i in range(S):
        st = streams[S][i]
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            models[S][i].forward_into(img[i * b:(i + 1) * b], logits[i * b:(i + 1) * b])
    for i in range(S):
        cur.wait_stream(streams[S][i])


for S in cfgs:
    step(S)
    torch.cuda.synchronize()
    if ref is None:
        ref = logits.clone()
    print(S, "max|diff| vs first", float((logits - ref).abs().max()), flush=True)
res = {S: [] for S in cfgs}
for rnd in range(4):
    for S in cfgs:
        for _ in range(3):
            step(S)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            step(S)
        torch.cuda.synchronize()
        res[S].append(10 * B / (time.perf_counter() - t0))
for S in cfgs:
    print(f"streams {S}: {max(res[S]):.0f} img/s (rounds {[round(v) for v in res[S]]})", flush=True)
