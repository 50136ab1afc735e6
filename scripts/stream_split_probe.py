"""Round-6 probe: the strong-scaling share (64 images per GPU) as k interleaved sub-batches on k
HIP streams (one model handle / workspace each, the same weights) against one 64-image forward.
Prints img/s per arm, alternating arms.   python scripts/stream_split_probe.py [batch] [model]
(model: deit_base (default), t2t_vit_14 or swin_tiny)"""
import sys
import time

import torch

sys.path.insert(0, ".")
from edgevisiontransformer_amd.modeling.models import swin, t2t_vit, vit  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
MODEL = sys.argv[2] if len(sys.argv) > 2 else "deit_base"
MOD = swin if MODEL.startswith("swin") else t2t_vit if MODEL.startswith("t2t") else vit
DTYPE = __import__("os").environ.get("PROBE_DTYPE", "bf16")
SHAPE = (224, 224, 3) if MODEL.startswith("t2t") else (3, 224, 224)  # T2T-ViT is channel-last
dev = torch.device("cuda", 0)
g = torch.Generator(device="cuda").manual_seed(1000)
img = torch.randn((B, *SHAPE), generator=g, device="cuda")


def _raw_stream(cumask=False):
    """A HIP stream made by hipStreamCreateWithFlags(hipStreamNonBlocking), as the library's lanes
    make theirs (or, cumask, by hipExtStreamCreateWithCUMask with every CU enabled), wrapped for
    torch (tells stream origin apart from weight sharing)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")
    st = ctypes.c_void_p()
    if cumask:
        mask = (ctypes.c_uint32 * 8)(*([0xFFFFFFFF] * 8))
        assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), 8, mask) == 0
    else:
        assert hip.hipStreamCreateWithFlags(ctypes.byref(st), 1) == 0
    return torch.cuda.ExternalStream(st.value)


def arm(k, steps=50, warm=5, lanes=1, raw=False, cumask=False, libstreams=False):
    """k handles on k torch streams (lanes = 1 each), or (lanes > 1) ONE handle whose native
    batch lanes (evt_model_set_lanes) fork / join inside the forward."""
    import os
    kw = {"lanes": lanes} if MOD is not vit else {}
    os.environ["EVT_LANE_STREAMS"] = "" if libstreams else "torch"
    models = [MOD.build_named(MODEL, dtype=DTYPE, seed=0, max_batch=B // k, **kw) for _ in range(k)]
    os.environ["EVT_LANE_STREAMS"] = ""
    streams = [_raw_stream(cumask) if raw else torch.cuda.Stream() for _ in range(k)]
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


res, outs = {}, {}
arms = [(1, 1), (2, 1)] if B > 64 else [(1, 1), (2, 1), (4, 1)]
if MOD is not vit:
    arms.append((1, 2))  # native lanes on torch pool streams (EVT_LANE_STREAMS=torch)
    arms.append((1, -3))  # native lanes on the streams the library creates (the default)
    arms.append((2, -1))  # two handles on raw HIP streams
ONLY = sys.argv[3] if len(sys.argv) > 3 and sys.argv[3] != "all" else ""  # "torch" / "native": that arm alone (profiling)
if ONLY:
    arms = [(2, 1)] if ONLY == "torch" else [(1, 2)]
ROUNDS = int(sys.argv[4]) if len(sys.argv) > 4 else 2
for rnd in range(1 if ONLY else ROUNDS):
    for k, lanes in (arms if rnd % 2 == 0 else arms[::-1]):  # order alternates by round
        v, out = arm(k, lanes=2 if lanes == -3 else max(lanes, 1), raw=lanes in (-1, -2),
                     cumask=lanes == -2, libstreams=lanes == -3)
        key = (k if lanes == 1 else f"native{lanes}" if lanes > 1 else
               f"raw{k}" if lanes == -1 else f"cumask{k}" if lanes == -2 else "native2lib")
        res.setdefault(key, []).append(round(v, 1))
        outs[key] = out
        print(f"round {rnd} {key}: {v:.1f} img/s", flush=True)
print({k: v for k, v in res.items()})
if 1 in outs:
    print({f"k={k} bitwise vs k=1": bool(torch.equal(outs[k], outs[1])) for k in outs if k != 1})
