"""Debug: where does the persistent-kernel output differ from the 256x256 reference kernel?"""
import sys
import torch
sys.path.insert(0, ".")
from edgevisiontransformer_amd import _lib  # noqa: E402
from tests import _ops  # noqa: E402

lib = _lib.load_library()
_lib.ensure_device(0)
for (M, K, N) in [(256, 64, 256), (256, 192, 256), (197, 192, 576)]:
    g = torch.Generator().manual_seed(0)
    A = torch.randn((M, K), generator=g).bfloat16().cuda()
    W = (torch.randn((K, N), generator=g) / K ** 0.5).cuda()
    wp, kpad, npad = _ops.pack(W, "bf16")
    outs = {}
    for v in (2, 9):
        lib.evt_set_gemm_variant(v)
        outs[v] = _ops.dense("bf16", 0, A, wp, kpad, npad, M, N).float()
        torch.cuda.synchronize()
    lib.evt_set_gemm_variant(0)
    d = (outs[2] - outs[9]).abs()
    bad = (d > 1e-2)
    print(M, K, N, "bad frac", bad.float().mean().item())
    if bad.any():
        # pattern within 16x16 blocks and per-row / per-col counts
        r, c = bad.nonzero(as_tuple=True)
        print(" rows mod 32:", torch.bincount(r % 32, minlength=32).tolist())
        print(" cols mod 16:", torch.bincount(c % 16, minlength=16).tolist())
        print(" row blocks (16):", torch.bincount(r // 16).tolist())
        print(" col blocks (16):", torch.bincount(c // 16).tolist())
        # try to find where value at (i,j) of ref landed in out9
        ref, o9 = outs[2], outs[9]
        for (i, j) in [(0, 0), (0, 5), (1, 0), (16, 0), (0, 8), (0, 16), (17, 9)]:
            hits = ((o9 - ref[i, j]).abs() < 1e-6).nonzero().tolist()[:4]
            print(f"  ref[{i},{j}]={ref[i, j].item():.4f} found at {hits} ; o9[{i},{j}]={o9[i, j].item():.4f}")
