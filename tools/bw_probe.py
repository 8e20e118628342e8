"""Practical HBM bandwidth on this GPU: torch sum (read) and copy (read + write) over 4 GiB."""
import torch, time
x = torch.empty(4 << 30, dtype=torch.uint8, device="cuda").view(torch.bfloat16)  # 4 GiB
x.normal_()
def t(fn, n=10):
    fn(); torch.cuda.synchronize()
    a=torch.cuda.Event(enable_timing=True); b=torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n): fn()
    b.record(); b.synchronize()
    return a.elapsed_time(b)/n/1e3
s = t(lambda: x.sum(dtype=torch.float32))
print(f"sum read: {x.numel()*2/s/1e12:.2f} TB/s")
y = torch.empty_like(x)
s = t(lambda: y.copy_(x))
print(f"copy: {2*x.numel()*2/s/1e12:.2f} TB/s (read+write)")
