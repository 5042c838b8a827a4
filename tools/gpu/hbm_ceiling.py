"""Write-only and copy HBM rates with torch's own kernels (fill_, copy_,
u8->f32 convert) on 2 GiB buffers: the ceiling the replay gather's store-heavy
mix (4 B written per 1.25 B moved... 80 % stores) is judged against."""
import torch

n = 1 << 29                      # 2 GiB of f32
a = torch.empty(n, device="cuda")
b = torch.empty(n, device="cuda")
u = torch.randint(0, 255, (n,), device="cuda", dtype=torch.uint8)


def t(fn, nbytes, it=20):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record(); torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / it
    return "%.0f us, %.2f TB/s" % (us, nbytes / us / 1e6)


print("fill f32 (write only):", t(lambda: a.fill_(1.0), 4 * n))
print("copy f32:", t(lambda: a.copy_(b), 8 * n))
print("u8->f32 convert:", t(lambda: a.copy_(u), 5 * n))
