"""Sweep prefill GEMM plans (tile config x split-K) on the PaliGemma prefill shapes; prints
us per call for each.  Usage (GPU box): python tools/gemm_sweep.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"))
sys.path.insert(0, REPO)
from oracle import weights as W  # noqa: E402
from pgmi import Engine, _native as N  # noqa: E402

SHAPES = {  # name: (M, N, K, epi)
    "t_qkv": (288, 2560, 2048, 0), "t_o": (288, 2048, 2048, 4), "t_gateup": (288, 16384, 2048, 7),
    "t_down": (288, 2048, 16384, 4), "v_qkv": (256, 3456, 1152, 1), "v_out": (256, 1152, 1152, 3),
    "v_fc1": (256, 4304, 1152, 2), "v_fc2": (256, 1152, 4304, 3), "v_patch": (256, 1152, 640, 1),
}


def main():
    e = Engine(W.small_config(1, 1, 1024), max_batch=1, max_seq=320, max_kv=512)
    e.fill_synthetic(1, W.init_policy)
    e.prepare()
    lib = e.lib
    s = torch.cuda.current_stream().cuda_stream
    for name, (M, Nn, K, epi) in SHAPES.items():
        A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        Wt = (torch.randn(Nn * (2 if epi == 7 else 1), K, device="cuda") / K ** 0.5).to(torch.bfloat16)
        bias = torch.randn(Nn, device="cuda").to(torch.bfloat16)
        res = torch.randn(M, Nn, device="cuda").to(torch.bfloat16)
        out = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16)
        res_line = []
        for cfg, split in [(-1, 0)] + [(c, sp) for c in range(6) for sp in (1, 2, 4, 8)]:
            if epi == 7 and split > 1:
                continue
            N.check(lib.pgmi_tune_gemm(cfg, split))
            f = lambda: N.check(lib.pgmi_op_gemm(e.ctx, A.data_ptr(), Wt.data_ptr(), M, Nn, K, epi, bias.data_ptr(),  # noqa: E731
                                                 res.data_ptr(), out.data_ptr(), s))
            for _ in range(3):
                f()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(20):
                f()
            t1.record()
            t1.synchronize()
            res_line.append((t0.elapsed_time(t1) * 1e3 / 20, cfg, split))
        N.check(lib.pgmi_tune_gemm(-1, 0))
        auto = res_line[0][0]
        best = sorted(res_line[1:])[:4]
        print(f"{name:9s} M={M} N={Nn} K={K}: auto {auto:7.1f} us | best " +
              ", ".join(f"cfg{c}/s{sp}: {t:6.1f}" for t, c, sp in best), flush=True)


if __name__ == "__main__":
    main()
