"""Round-6 probe: the strong-scaling share (64 images per GPU) as k interleaved sub-batches on k
HIP streams (one model handle / workspace each, the same weights) against one 64-image forward.
Prints img/s per arm, alternating arms.   python scripts/stream_split_probe.py [batch]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from edgevisiontransformer_amd.modeling.models import vit  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda", 0)
g = torch.Generator(device="cuda").manual_seed(1000)
img = torch.randn((B, 3, 224, 224), generator=g, device="cuda")


def arm(k, steps=50, warm=5):
    models = [vit.build_named("deit_base", dtype="bf16", seed=0, max_batch=B // k) for _ in range(k)]
    streams = [torch.cuda.Stream() for _ in range(k)]
    outs = [torch.empty((B // k, 1000), device="cuda") for _ in range(k)]
    parts = [img[i * (B // k):(i + 1) * (B // k)] for i in range(k)]
    main = torch.cuda.current_stream()

    def step():
        for i in range(k):
            streams[i].wait_stream(main)
            with torch.cuda.stream(streams[i]):
                models[i].forward_into(parts[i], outs[i])
        for i in range(k):
            main.wait_stream(streams[i])
    for _ in range(warm):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ref = torch.cat(outs).clone()
    del models
    return B * steps / el, ref


res = {}
for rnd in range(2):
    for k in (1, 2, 4):
        v, out = arm(k)
        res.setdefault(k, []).append(round(v, 1))
        print(f"round {rnd} k={k}: {v:.1f} img/s", flush=True)
print({k: v for k, v in res.items()})
