"""Write-then-read bandwidth vs working-set size (is a 100-300 MB intermediate served
by the 256 MB Infinity Cache?): chains of device copies a -> b -> c over buffers of S
bytes, timed with HIP events."""
import torch

dev = torch.device("cuda")
for mb in (16, 32, 64, 96, 128, 192, 256, 512, 2048):
    n = mb * (1 << 20) // 4
    a = torch.randn(n, device=dev)
    b = torch.empty_like(a)
    c = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a); c.copy_(b)
    torch.cuda.synchronize()
    reps = max(3, int(4096 / mb))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
        c.copy_(b)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / (2 * reps)
    print("%5d MB  copy %.3f ms  %.2f TB/s (read+write)" % (mb, ms, 2 * n * 4 / ms / 1e9), flush=True)
