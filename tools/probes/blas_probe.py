"""hipBLASLt (torch.matmul) on the prefill GEMM shapes, cold weights, graph-replayed: the library's
rate as a yardstick for kernels_gemm.hip.  usage (GPU box): python tools/probes/blas_probe.py"""
import torch

SHAPES = {"t_gateup": (288, 32768, 2048), "t448_gateup": (1056, 32768, 2048), "b8_t_gateup": (2304, 32768, 2048),
          "t448_down": (1056, 2048, 16384), "t448_qkv": (1056, 2560, 2048), "v448_fc1": (1024, 4304, 1152),
          "v448_fc2": (1024, 1152, 4304), "t_down": (288, 2048, 16384), "v_fc1": (256, 4304, 1152)}
for name, (M, N, K) in SHAPES.items():
    A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    nw = max(1, -(-(320 << 20) // (N * K * 2)))
    Ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) for _ in range(nw)]
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    it = max(20, nw)
    for w in Ws[:3]:
        torch.matmul(A, w.t(), out=out)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(it):
            torch.matmul(A, Ws[i % nw].t(), out=out)
    g.replay()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    g.replay()
    t1.record()
    t1.synchronize()
    us = t0.elapsed_time(t1) * 1e3 / it
    print(f"{name:12s} M={M} N={N} K={K}: {us:7.1f} us {2.0 * M * N * K / us / 1e6:6.0f} TF", flush=True)
