"""Determine the operand / scale layout of v_mfma_scale_f32_16x16x128_f8f6f4 with exact data."""
import ctypes, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import mx8_ref

torch.cuda.init()
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "mx8_probe.so"))
dev = torch.device("cuda", 0)

def run(Abytes, Bbytes, sa, sb):
    a = torch.from_numpy(np.ascontiguousarray(Abytes).view(np.int32).reshape(-1)).to(dev)
    b = torch.from_numpy(np.ascontiguousarray(Bbytes).view(np.int32).reshape(-1)).to(dev)
    sa_t = torch.from_numpy(np.asarray(sa, np.int32)).to(dev)
    sb_t = torch.from_numpy(np.asarray(sb, np.int32)).to(dev)
    d = torch.zeros(256, device=dev)
    assert lib.run_probe(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()),
                         ctypes.c_void_p(sa_t.data_ptr()), ctypes.c_void_p(sb_t.data_ptr()),
                         ctypes.c_void_p(d.data_ptr())) == 0
    return d.cpu().numpy().reshape(64, 4)

rng = np.random.default_rng(0)
# small integers exactly representable in e4m3
Av = rng.integers(-3, 4, (16, 128)).astype(np.float32)
Bv = rng.integers(-3, 4, (128, 16)).astype(np.float32)
ref = Av @ Bv
enc = lambda v: mx8_ref.e4m3_encode(v)

def pack(kmap):
    """kmap(lane, j) -> k. A lane holds A[l&15][k], B lane holds B[k][l&15]."""
    Ab = np.zeros((64, 32), np.uint8); Bb = np.zeros((64, 32), np.uint8)
    for l in range(64):
        for j in range(32):
            k = kmap(l, j)
            Ab[l, j] = enc(np.float32(Av[l & 15, k])); Bb[l, j] = enc(np.float32(Bv[k, l & 15]))
    return Ab, Bb

hyps = {
    "k=32g+j": lambda l, j: 32 * (l >> 4) + j,
    "k=16g+j | 64+16g+j-16": lambda l, j: 16 * (l >> 4) + j if j < 16 else 64 + 16 * (l >> 4) + j - 16,
    "k=8g+j per 32": lambda l, j: 32 * (j >> 3) + 8 * (l >> 4) + (j & 7),
}
one = [127] * 64
for name, km in hyps.items():
    Ab, Bb = pack(km)
    d = run(Ab, Bb, one, one)
    # C layout: col = l & 15, row = 4 (l >> 4) + r
    D = np.zeros((16, 16), np.float32)
    for l in range(64):
        for r in range(4):
            D[4 * (l >> 4) + r, l & 15] = d[l, r]
    print(name, "match" if np.array_equal(D, ref) else f"max err {np.abs(D - ref).max()}")

# scale semantics under k=32g+j: lane l's scale byte scales its own 32 elements?
km = hyps["k=32g+j"]
Ab, Bb = pack(km)
sa = rng.integers(120, 135, 64); sb = rng.integers(120, 135, 64)
d = run(Ab, Bb, sa, sb)
D = np.zeros((16, 16))
for l in range(64):
    for r in range(4):
        D[4 * (l >> 4) + r, l & 15] = d[l, r]
ref2 = np.zeros((16, 16))
for i in range(16):
    for jj in range(16):
        s = 0.0
        for k in range(128):
            g = k // 32
            s += Av[i, k] * 2.0 ** (sa[16 * g + i] - 127) * Bv[k, jj] * 2.0 ** (sb[16 * g + jj] - 127)
        ref2[i, jj] = s
print("scale per (lane-group, row):", "match" if np.allclose(D, ref2, rtol=1e-6) else f"max rel {np.abs(D-ref2).max()/np.abs(ref2).max()}")
# garbage in the upper scale bits ignored?
d3 = run(Ab, Bb, [int(x) | (0x5A << 8) | (0x33 << 16) for x in sa], [int(x) | (0x77 << 24) for x in sb])
print("upper scale bytes ignored:", np.array_equal(d3, d))

# which lane's scale applies to byte j of lane group g (row 0)?  A: one 1.0 at (lane 16g, byte j),
# B all ones, scale of lane-group h = 2^h (unit elsewhere)
onesB = np.full((64, 32), enc(np.float32(1.0)), np.uint8)
onesA = onesB.copy()
sa_g = [127 + (l >> 4) for l in range(64)]
print("A scale group of (g, j):")
for g in range(4):
    row = []
    for j in range(32):
        Ab = np.zeros((64, 32), np.uint8); Ab[16 * g, j] = enc(np.float32(1.0))
        d = run(Ab, onesB, sa_g, one)
        v = d[0, 0]  # D[row 0][col 0]: lane 0, r 0
        row.append(int(np.log2(v)) if v > 0 else -1)
    print(g, row)
print("B scale group of (g, j):")
for g in range(4):
    row = []
    for j in range(32):
        Bb = np.zeros((64, 32), np.uint8); Bb[16 * g, j] = enc(np.float32(1.0))
        d = run(onesA, Bb, one, sa_g)
        v = d[0, 0]
        row.append(int(np.log2(v)) if v > 0 else -1)
    print(g, row)
