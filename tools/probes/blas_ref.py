"""Probe: what the vendor GEMM (torch.mm -> hipBLASLt) reaches on the prefill shapes, random bf16
operands, to calibrate the panel GEMM's MFMA fraction against an achievable ceiling on this box.
    python tools/probes/blas_ref.py
"""
import torch

shapes = [  # (M, N, K) as C[M,N] = A[M,K] . W[N,K]^T
    (288, 32768, 2048), (288, 2048, 16384), (1056, 32768, 2048), (1056, 2048, 16384),
    (1024, 4304, 1152), (4096, 4096, 4096), (8192, 8192, 8192)]
torch.manual_seed(0)
for M, N, K in shapes:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ w.t()
    n = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        c = a @ w.t()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / n * 1e3
    tf = 2.0 * M * N * K / us / 1e6
    print(f"M={M:5d} N={N:6d} K={K:6d}  {us:9.1f} us  {tf:7.1f} TFLOP/s  {tf / 2500 * 100:5.1f}% of 2.5 PF", flush=True)
