"""How much of a small-M prefill GEMM's time is the cold weight read?  For each shape (default plan),
times graph-replayed calls with (hot) the same weights every call, (cold) rotating weight copies
> 256 MiB in all, (mall) rotating copies each read once by a plain reduction right before its GEMM
(its time measured alone and subtracted).  Usage (GPU box): python tools/probes/warm_probe.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"))
sys.path.insert(0, REPO)
from oracle import weights as W  # noqa: E402
from pgmi import Engine, _native as N  # noqa: E402

SHAPES = {"v_qkv": (256, 3456, 1152, 1), "v_out": (256, 1152, 1152, 3), "v_fc1": (256, 4304, 1152, 2),
          "v_fc2": (256, 1152, 4304, 3), "t_qkv": (288, 2560, 2048, 0), "t_o": (288, 2048, 2048, 4),
          "t_gateup": (288, 16384, 2048, 7), "t_down": (288, 2048, 16384, 4)}


def graph_us(fn, n):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(n):
            fn(i, torch.cuda.current_stream().cuda_stream)
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        g.replay()
        t1.record()
        t1.synchronize()
        best = min(best, t0.elapsed_time(t1) * 1e3 / n)
    return best


def main():
    e = Engine(W.small_config(1, 1, 1024), max_batch=1, max_seq=320, max_kv=512)
    e.fill_synthetic(1, W.init_policy)
    e.prepare()
    lib = e.lib
    torch.manual_seed(0)
    sink = torch.zeros((), device="cuda", dtype=torch.int32)
    for name, (M, Nn, K, epi) in SHAPES.items():
        A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        Wt = ((torch.rand(Nn * (2 if epi == 7 else 1), K, device="cuda") * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        nw = max(2, -(-(320 << 20) // (Wt.numel() * 2)))
        Ws = [Wt] + [Wt.clone() for _ in range(nw - 1)]
        bias = torch.randn(Nn, device="cuda").to(torch.bfloat16)
        res = torch.randn(M, Nn, device="cuda").to(torch.bfloat16)
        out = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16)

        def gemm(w, st):
            N.check(lib.pgmi_op_gemm(e.ctx, A.data_ptr(), w.data_ptr(), M, Nn, K, epi, bias.data_ptr(),
                                     res.data_ptr(), out.data_ptr(), st))

        def touch(w):
            torch.sum(w.view(torch.int16), dim=(0, 1), dtype=torch.int32, out=sink)

        n = max(nw, 24)
        hot = graph_us(lambda i, st: gemm(Ws[0], st), n)
        cold = graph_us(lambda i, st: gemm(Ws[i % nw], st), n)
        t_only = graph_us(lambda i, st: touch(Ws[i % nw]), n)
        both = graph_us(lambda i, st: (touch(Ws[i % nw]), gemm(Ws[i % nw], st)), n)
        print(f"{name:9s} M={M} N={Nn} K={K} W={Wt.numel() * 2 / 1e6:6.1f} MB: hot {hot:7.2f} us  cold {cold:7.2f} us  "
              f"mall-warm {both - t_only:7.2f} us  (touch {t_only:6.2f}, touch+gemm {both:7.2f})", flush=True)


if __name__ == "__main__":
    main()
