import torch, time
dev = torch.device("cuda", 0)
def t(fn, it=50):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it
for (m, n, k) in [(4096, 512, 512), (512, 512, 4096), (4096, 512, 12), (4096, 512, 64)]:
    for dt in (torch.float32, torch.bfloat16):
        a = torch.randn(m, k, device=dev, dtype=dt); b = torch.randn(k, n, device=dev, dtype=dt)
        ms = t(lambda: torch.mm(a, b))
        print(f"mm {m}x{n}x{k} {dt}: {ms*1e3:.1f} us  {2*m*n*k/ms/1e9:.1f} TF/s")
a = torch.randn(4096, 512, device=dev); b = torch.randn(512, 512, device=dev)
torch.backends.cuda.matmul.allow_tf32 = True
ms = t(lambda: torch.mm(a, b)); print(f"tf32 allowed 4096x512x512: {ms*1e3:.1f} us {2*4096*512*512/ms/1e9:.1f} TF/s")
