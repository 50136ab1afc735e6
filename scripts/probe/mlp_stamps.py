"""Where the Swin stage-1 fused MLP (swin_mlp96_kernel) spends a tile: s_memtime stamps of the first
4 tiles of every wave, from a lab build with -DEVT_MLP_STAMPS (scripts/gpu_run.sh does not build;
build on the CPU first):
    EVT_LAB=1 EVT_LAB_DEFS=-DEVT_MLP_STAMPS python -m edgevisiontransformer_amd.build
    EVT_LIB=<that .so> python scripts/probe/mlp_stamps.py
Stamps (per wave, per tile): 0 tile start, 1 LN'd operands ready, 2/5 FC1 of hidden chunk 0/1
issued, 3/6 its GELU packed, 4/7 FC2 issued, 8 chunk loop done, 9 tile stored; 10/11 realtime
(100 MHz) at start / end for the clock."""
import ctypes
import os

import numpy as np
import torch

from edgevisiontransformer_amd import _lib
from edgevisiontransformer_amd.modeling.models import swin as mod

B = int(os.environ.get("BATCH", "256"))
model = mod.build_named("swin_tiny", dtype="bf16", seed=0, max_batch=B)
img = torch.randn((B, 3, 224, 224), device="cuda", dtype=torch.float32)
logits = torch.empty((B, model.num_classes), device="cuda", dtype=torch.float32)
for _ in range(5):
    model.forward_into(img, logits)
torch.cuda.synchronize()
lib = _lib.load_library()
f = lib.evt_lab_mlp_stamps  # the loaded CDLL (EVT_LIB)
f.restype = ctypes.c_int
f.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
buf = np.zeros(1024 * 16 * 4 * 16, dtype=np.uint64)
assert f(buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(1024, 16, 4, 16).astype(np.int64)
ok = (st[..., 0] > 0) & (st[..., 9] > st[..., 0])
s = st[ok]
print(f"tiles stamped: {len(s)}")
clk = np.median((s[:, 9] - s[:, 0]) / np.maximum(s[:, 11] - s[:, 10], 1) * 100e6) / 1e9
print(f"in-kernel clock ~{clk:.2f} GHz")
names = [("load + LN", 0, 1), ("chunk0 FC1 issue", 1, 2), ("chunk0 GELU", 2, 3),
         ("chunk0 FC2 issue", 3, 4), ("chunk1 FC1 issue", 4, 5), ("chunk1 GELU", 5, 6),
         ("chunk1 FC2 issue", 6, 7), ("chunks 2-11", 7, 8), ("epilogue", 8, 9), ("whole tile", 0, 9)]
for nm, a, b in names:
    d = s[:, b] - s[:, a]
    print(f"{nm:18s} median {np.median(d):8.0f} cyc  p10 {np.percentile(d, 10):8.0f}  p90 {np.percentile(d, 90):8.0f}")
# first tile vs later tiles
for it in range(4):
    sel = st[:, :, it][ok[:, :, it]]
    if len(sel):
        print(f"tile {it}: whole {np.median(sel[:, 9] - sel[:, 0]):8.0f} cyc  (n={len(sel)})")
