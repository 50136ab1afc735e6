"""HBM write-pattern microbenchmark (torch fill_ on strided views): bandwidth of writing row
segments of S bytes at a row pitch of P bytes, to see how segment length affects write rate."""
import torch

def bench(rows, pitch_elems, seg_elems, dtype):
    buf = torch.empty((rows, pitch_elems), dtype=dtype, device="cuda")
    view = buf[:, :seg_elems]
    for _ in range(3):
        view.fill_(1.0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    n = 10
    for _ in range(n):
        view.fill_(1.0)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / n / 1e3
    byt = rows * seg_elems * view.element_size()
    print(f"{str(dtype):15s} seg {seg_elems * view.element_size():6d} B pitch {pitch_elems * view.element_size():6d} B "
          f"rows {rows:8d}: {byt / 1e6:8.1f} MB in {t * 1e6:7.1f} us = {byt / t / 1e12:5.2f} TB/s")

M = 100864
for dt in (torch.bfloat16, torch.float32):
    es = 2 if dt == torch.bfloat16 else 4
    for seg_b in (256, 512, 1024, 2048):
        seg = seg_b // es
        pitch = 6144 // es
        if seg <= pitch:
            bench(M, pitch, seg, dt)
bench(M * 12, 256, 256, torch.bfloat16)   # contiguous 620 MB bf16
bench(M, 3072, 3072, torch.bfloat16)      # contiguous
