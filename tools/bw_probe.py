"""Plain bandwidth references on the GPU box (torch ops, for calibration only)."""
import torch, time
def t(f, it=20):
    f(); torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it): f()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e-3
x = torch.rand(300_000_000, device="cuda")          # 1.2 GB
y = torch.empty_like(x)
l = torch.zeros(100_000_000, dtype=torch.int16, device="cuda")
s = t(lambda: x.sum()); print("read 1.2GB sum      %.0f GB/s" % (1.2e9 / s / 1e9))
s = t(lambda: y.copy_(x)); print("copy 1.2GB (r+w)     %.0f GB/s" % (2.4e9 / s / 1e9))
s = t(lambda: l.add_(1)); print("int16 rmw 0.2GB      %.0f GB/s" % (0.4e9 / s / 1e9))
