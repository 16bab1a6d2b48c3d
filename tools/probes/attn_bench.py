"""Probe: prefill attention kernel time at the PaliGemma shapes (SigLIP / Gemma, 224 / 448 px)
for every variant of pgmi_tune_attention (0 = 16-row kernel, RK = tiled with R row groups and
K key splits, 7 / 8 = the one-pass short-range kernels, 9 / 9N = the one-pass key-split kernel
(auto / N key ranges), -1 = the default choice), plus a rel-L2 check against a torch fp32 attention with
the reference's rounding points.
    python tools/probes/attn_bench.py [variants...]
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"), REPO]
from oracle import weights as W  # noqa: E402
from pgmi import Engine  # noqa: E402
from pgmi import _native as NN  # noqa: E402

eng = Engine(W.small_config(vision_layers=1, text_layers=1, vocab=1024), max_batch=1, max_seq=64, max_kv=64)
eng.fill_synthetic(1, W.init_policy)
eng.prepare()
shapes = [("siglip224", 256, 16, 16, 72), ("siglip448", 1024, 16, 16, 72),
          ("gemma224", 288, 8, 1, 256), ("gemma448", 1056, 8, 1, 256)]
if os.environ.get("ATTN_SHAPES"):
    shapes = [sh for sh in shapes if sh[0] in os.environ["ATTN_SHAPES"].split(",")]
torch.manual_seed(0)
variants = [int(v) for v in sys.argv[1:]] or [-1, 7, 8, 42, 44, 24, 9, 91, 92, 94]
for var, (name, L, H, Hkv, d) in [(v, sh) for sh in shapes for v in variants]:
    if var % 100 in (44, 24) and d != 72:
        continue
    if (var == 7 and name != "siglip224") or (var == 8 and name != "gemma224"):
        continue
    NN.check(eng.lib.pgmi_tune_attention(var))
    scale = d ** -0.5
    q = (torch.randn(1, L, H, d, device="cuda") * 2).bfloat16()
    k = (torch.randn(1, L, Hkv, d, device="cuda") * 2).bfloat16()
    v = torch.randn(1, L, Hkv, d, device="cuda").bfloat16()
    o = torch.empty_like(q)
    s = NN.stream_handle()

    def run():
        NN.check(eng.lib.pgmi_op_attention(eng.ctx, q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                           1, L, L, H, Hkv, d, scale, s))
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    # GPU time: the calls replayed from a captured graph (ctypes host launches would floor them)
    n = 20
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = torch.cuda.current_stream().cuda_stream
        for _ in range(n):
            run()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / n * 1e3
    del g
    s = NN.stream_handle()
    qh = q.float().transpose(1, 2)
    kh = k.float().transpose(1, 2).repeat_interleave(H // Hkv, 1)
    vh = v.float().transpose(1, 2).repeat_interleave(H // Hkv, 1)
    sc = ((qh @ kh.transpose(-1, -2)).bfloat16().float() * scale).bfloat16().float()
    p = torch.softmax(sc, -1).bfloat16().float()
    ref = (p @ vh).bfloat16().float().transpose(1, 2)
    rel = ((o.float() - ref).norm() / ref.norm()).item()
    fl = 2 * 2 * L * L * d * H
    print(f"variant {var:3d} {name:10s} {us:8.1f} us  "
          f"{fl / us / 1e6:7.1f} TFLOP/s (2-matmul flops)  rel-L2 {rel:.2e}", flush=True)
