import ctypes, os, numpy as np, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "dot2_probe.so"))
n = 4096
g = np.random.default_rng(0)
x = torch.from_numpy(g.standard_normal((n, 2)).astype(np.float32)).bfloat16()
y = torch.from_numpy(g.standard_normal((n, 2)).astype(np.float32)).bfloat16()
c = torch.from_numpy(g.standard_normal(n).astype(np.float32))
A = x.view(torch.int32).view(-1) if False else x.contiguous().view(torch.int16).view(torch.int32).view(-1)
B = y.contiguous().view(torch.int16).view(torch.int32).view(-1)
dA, dB, dc = A.cuda(), B.cuda(), c.cuda()
out = torch.empty(n, device="cuda")
assert lib.dot2_probe(ctypes.c_void_p(dA.data_ptr()), ctypes.c_void_p(dB.data_ptr()), ctypes.c_void_p(dc.data_ptr()), ctypes.c_void_p(out.data_ptr()), n) == 0
ref = (x.double() * y.double()).sum(1) + c.double()
err = (out.cpu().double() - ref).abs()
print("dot2 max err", err.max().item(), "max rel", (err / ref.abs().clamp_min(1e-3)).max().item())
print("samples", out[:4].cpu().tolist(), ref[:4].tolist())
