"""Probe: do parallel branches of a captured graph run concurrently on this ROCm?"""
import time

import torch

a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
c1 = torch.empty_like(a)
c2 = torch.empty_like(a)
s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()


def work(serial):
    with torch.cuda.stream(s0):
        torch.mm(a[:1024], b, out=c1[:1024])
        if serial:
            torch.mm(a[1024:2048], b, out=c2[:1024])
        else:
            ev = torch.cuda.Event()
            ev.record(s0)
            s1.wait_event(ev)
            with torch.cuda.stream(s1):
                torch.mm(a[1024:2048], b, out=c2[:1024])
            ev2 = torch.cuda.Event()
            ev2.record(s1)
            s0.wait_event(ev2)


for serial in (True, False):
    for _ in range(3):
        work(serial)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s0):
        work(serial)
    torch.cuda.synchronize()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 50 * 1e6
    # eager
    t0 = time.perf_counter()
    for _ in range(50):
        work(serial)
    torch.cuda.synchronize()
    de = (time.perf_counter() - t0) / 50 * 1e6
    print(f"{'serial' if serial else 'branches'}: graph {dt:.1f} us, eager {de:.1f} us")
