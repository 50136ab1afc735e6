"""Per-phase timeline of the persistent GEMM's 8-phase main loop: s_memtime stamps of one SIMD's two
waves (waves 0 and 4 of block 0) at every phase event, from a lab build with -DEVT_ABL_PHSTAMP:
    git apply scripts/probe/ph_stamps.patch && EVT_LAB=1 EVT_LAB_DEFS=-DEVT_ABL_PHSTAMP python -m edgevisiontransformer_amd.build
    EVT_LIB=<that .so> PYTHONPATH=. python scripts/probe/ph_stamps.py [K N]
Events per phase: 0 start, 1 reads issued, 2 DMA issued, 3 wait done, 4 past the barrier,
5 MFMAs issued, 6 past the closing barrier."""
import ctypes
import sys

import numpy as np
import torch

from edgevisiontransformer_amd import _lib
from tests import _ops

K, N = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (768, 3072)
M = 100864
A = torch.randn((M, K), device="cuda").bfloat16()
W = torch.randn((K, N), device="cuda") / K ** 0.5
wp, kpad, npad = _ops.pack(W, "bf16")
for _ in range(5):
    _ops.dense("bf16", 0, A, wp, kpad, npad, M, N)
torch.cuda.synchronize()
f = _lib.load_library().evt_lab_ph_stamps
f.restype = ctypes.c_int
f.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
buf = np.zeros(2 * 64 * 4 * 8, dtype=np.uint64)
assert f(buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(2, 64, 4, 8).astype(np.int64)
nk = K // 64
t0 = st[0, 0, 0, 0]
names = ["reads", "dma", "wait", "bar1", "mfma", "bar2"]
print(f"K={K} N={N}: nk={nk}; per wave, K-tiles 2..{nk - 3}, cycles (median over those K-tiles)")
for w in range(2):
    rows = []
    for ph in range(4):
        d = [np.median([st[w, t, ph, e + 1] - st[w, t, ph, e] for t in range(2, nk - 2)]) for e in range(6)]
        rows.append(d)
        print(f" wave {4 * w} phase {ph}: " + "  ".join(f"{n} {v:6.0f}" for n, v in zip(names, d)))
    kt = [st[w, t + 1, 0, 0] - st[w, t, 0, 0] for t in range(2, nk - 3)]
    print(f" wave {4 * w}: K-tile period median {np.median(kt):.0f} cycles")
# interleaving of the two waves in one K-tile (absolute, relative to wave 0's phase-0 start)
t = nk // 2
base = st[0, t, 0, 0]
for ph in range(4):
    print(f" t={t} ph{ph} wave0 " + " ".join(f"{st[0, t, ph, e] - base:6d}" for e in range(7)) +
          "   wave4 " + " ".join(f"{st[1, t, ph, e] - base:6d}" for e in range(7)))
