"""Achievable HBM write and read+write rates on this box (torch kernels), to
calibrate the OFFSETS passes' store rates: fill of 12 GB, copy of 8 GB."""
import torch

def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(reps):
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b))
    return best

n = 12 * 10**9
x = torch.empty(n, dtype=torch.uint8, device="cuda")
ms = t(lambda: x.fill_(7))
print("fill 12 GB: %.3f ms = %.2f TB/s" % (ms, n / ms / 1e9))
y = torch.empty(n // 4, dtype=torch.int32, device="cuda")
ms = t(lambda: y.fill_(7))
print("fill int32 12 GB: %.3f ms = %.2f TB/s" % (ms, n / ms / 1e9))
del y
m = 8 * 10**9
src = torch.empty(m, dtype=torch.uint8, device="cuda")
dst = x[:m]
ms = t(lambda: dst.copy_(src))
print("copy 8 GB: %.3f ms = %.2f TB/s moved (r+w)" % (ms, 2 * m / ms / 1e9))
ms = t(lambda: src.sum(dtype=torch.int64))
print("read 8 GB (sum): %.3f ms = %.2f TB/s" % (ms, m / ms / 1e9))
