"""Probe: each decode projection kernel in isolation (pgmi_decode_kernel) at batch B, cycling
the 18 layers' weights (>> the 256 MiB MALL), HIP events on the launch stream.
    python tools/probes/decode_kernels.py [B ...]
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"), REPO]
from pgmi import Engine  # noqa: E402
from pgmi import _native as N  # noqa: E402
from pgmi.synthetic import init_policy, paligemma_3b_config  # noqa: E402

cfg = paligemma_3b_config(224)
eng = Engine(cfg, max_batch=8, max_seq=300, max_kv=512)
eng.fill_synthetic(1234, init_policy)
eng.prepare()
s = torch.cuda.current_stream()
H, I, V = 2048, 16384, 257216
names = {1: ("o_proj+res", 2 * H * H), 2: ("gate/up+geglu", 2 * 2 * I * H), 3: ("down+res", 2 * I * H),
         4: ("lm_head", 2 * V * H)}
for B in [int(b) for b in sys.argv[1:]] or [1, 8]:
    for k, (nm, byt) in names.items():
        iters = 18 if k != 4 else 6
        for i in range(4):
            N.check(eng.lib.pgmi_decode_kernel(eng.ctx, k, i % 18, B, s.cuda_stream))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for i in range(iters):
            N.check(eng.lib.pgmi_decode_kernel(eng.ctx, k, i % 18, B, s.cuda_stream))
        e1.record(s)
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / iters
        print(f"B={B} {nm:14s} {us:8.2f} us  {byt / us / 1e3:7.1f} GB/s", flush=True)
