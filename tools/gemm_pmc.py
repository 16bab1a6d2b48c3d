"""Run one prefill GEMM shape/plan repeatedly (for rocprofv3 --pmc passes).
usage: python tools/gemm_pmc.py <shape> <cfg> <split> [iters]   (shapes: tools/gemm_sweep.py)"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"), REPO, os.path.join(REPO, "tools")]
from gemm_sweep import SHAPES  # noqa: E402
from oracle import weights as W  # noqa: E402
from pgmi import Engine, _native as N  # noqa: E402


def main():
    name, cfg, split = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    M, Nn, K, epi = SHAPES[name]
    e = Engine(W.small_config(1, 1, 1024), max_batch=1, max_seq=320, max_kv=512)
    e.fill_synthetic(1, W.init_policy)
    e.prepare()
    s = torch.cuda.current_stream().cuda_stream
    A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    Wt = ((torch.rand(Nn * (2 if epi == 7 else 1), K, device="cuda") * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(Nn, device="cuda").to(torch.bfloat16)
    res = torch.randn(M, Nn, device="cuda").to(torch.bfloat16)
    out = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16)
    N.check(e.lib.pgmi_tune_gemm(cfg, split))
    for _ in range(iters):
        N.check(e.lib.pgmi_op_gemm(e.ctx, A.data_ptr(), Wt.data_ptr(), M, Nn, K, epi, bias.data_ptr(), res.data_ptr(),
                                   out.data_ptr(), s))
    torch.cuda.synchronize()
    print("done", name, cfg, split)


if __name__ == "__main__":
    main()
