import torch, time
x = torch.rand(128*1024*1024, dtype=torch.float64, device="cuda")  # 1 GiB
y = torch.empty_like(x)
for f, name, nb in ((lambda: x.sum(), "sum", x.numel()*8), (lambda: y.copy_(x), "copy", 2*x.numel()*8)):
    f(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20): f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 20
    print(name, f"{dt*1e3:.3f} ms", f"{nb/dt/1e12:.2f} TB/s")
