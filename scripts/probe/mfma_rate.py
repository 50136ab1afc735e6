import ctypes, os
import torch
torch.cuda.init()
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "mx8_probe.so"))
lib.run_rate.restype = ctypes.c_float
out = torch.zeros(256, device="cuda")
for which, name, flop in ((0, "mx8 16x16x128", 2 * 16 * 16 * 128), (1, "bf16 16x16x32", 2 * 16 * 16 * 32)):
    blocks, iters = 2048, 2000
    ms = lib.run_rate(which, blocks, iters, ctypes.c_void_p(out.data_ptr()))
    n = blocks * 4 * iters * 8
    print(f"{name}: {ms:.3f} ms, {n * flop / ms / 1e9:.1f} TFLOP/s")
