"""Probe: device top-p draw time (pgmi_sample_top_p) on PaliGemma-sized logit rows.
    python tools/probes/sample_bench.py
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"), REPO]
from oracle import weights as W  # noqa: E402
from pgmi import Engine  # noqa: E402

eng = Engine(W.small_config(vision_layers=1, text_layers=1, vocab=1024), max_batch=1, max_seq=64, max_kv=64)
eng.prepare()
g = torch.Generator(device="cuda").manual_seed(0)
for rows, V, scale, T, p in [(1, 257216, 4.0, 0.8, 0.9), (8, 257216, 4.0, 0.8, 0.9), (1, 257216, 0.3, 1.0, 0.9)]:
    lg = torch.randn((rows, V), device="cuda", generator=g) * scale
    u = torch.rand((23, rows), device="cuda", generator=g)
    for i in range(3):
        eng.sample_top_p(lg, p, T, u=u[i])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(20):
        eng.sample_top_p(lg, p, T, u=u[3 + i])
    e1.record()
    e1.synchronize()
    print(f"rows {rows} V {V} logit-scale {scale}: {e0.elapsed_time(e1) * 1e3 / 20:.1f} us per draw", flush=True)
