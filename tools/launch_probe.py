import torch, time
x = torch.zeros(64, device="cuda")
s = torch.cuda.Stream()
for n in (10, 100):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        for _ in range(3): x.add_(1)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n): x.add_(1)
    torch.cuda.synchronize()
    for _ in range(5): g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50): g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 50
    print(f"graph of {n} tiny kernels: {dt*1e6:.1f} us per replay, {dt*1e6/n:.2f} us per kernel")
# eager back-to-back
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(1000): x.add_(1)
torch.cuda.synchronize()
print(f"eager tiny kernel: {(time.perf_counter()-t0)*1e3:.2f} us each")
