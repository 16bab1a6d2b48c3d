"""Probe: does a decode GEMV run faster when its weights were read into the Infinity Cache (MALL,
256 MiB) just before?  Times the batch-1 gate/up GEMV (pgmi_decode_kernel 2) and down GEMV (3) of
layer i from cold caches (after streaming 600 MB of other data) against the same launch right after
a torch read of that layer's weights (default cache policy), and against a concurrent read on a
second stream while a chain of small kernels runs (the decode step's qkv/attention/o_proj window).
    python tools/probes/mall_probe.py
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"), REPO]
from oracle import weights as W  # noqa: E402
from pgmi import Engine  # noqa: E402
from pgmi import _native as N  # noqa: E402


def main():
    e = Engine(W.full_config(224), max_batch=1, max_seq=320, max_kv=512)
    e.fill_synthetic(1234, W.init_policy)
    e.prepare()
    s = torch.cuda.current_stream()
    flush = torch.empty(600 << 20, dtype=torch.uint8, device="cuda")
    sink = torch.empty(1, dtype=torch.float32, device="cuda")

    def kern(which, layer):
        N.check(e.lib.pgmi_decode_kernel(e.ctx, which, layer, 1, s.cuda_stream))

    def timed(fn):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        fn()
        b.record(s)
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3

    def read(t):  # a full read of the tensor through the default cache policy
        torch.sum(t.view(-1)[::1].float() if False else t.view(torch.int32), dtype=torch.int64, out=None)

    pre = "language_model.model.layers.%d."
    for which, names, label in ((2, ["mlp.gate_proj.weight", "mlp.up_proj.weight"], "gate/up"),
                                (3, ["mlp.down_proj.weight"], "down")):
        cold, warm, part = [], [], []
        for rep in range(6):
            layer = rep % 18
            ws = [e.views[(pre % layer) + n] for n in names]
            flush.fill_(rep)  # evict: 600 MB of writes
            torch.cuda.synchronize()
            cold.append(timed(lambda: kern(which, layer)))
            flush.fill_(rep + 1)
            for w in ws:
                sink += w.view(torch.int16).sum(dtype=torch.int32).float()  # read the weights (allocate)
            torch.cuda.synchronize()
            warm.append(timed(lambda: kern(which, layer)))
            # half of the weights pre-read
            flush.fill_(rep + 2)
            for w in ws:
                h = w.view(-1)[: w.numel() // 2]
                sink += h.view(torch.int16).sum(dtype=torch.int32).float()
            torch.cuda.synchronize()
            part.append(timed(lambda: kern(which, layer)))
        med = lambda v: sorted(v)[len(v) // 2]
        print(f"{label:8s}: cold {med(cold):7.2f} us | weights pre-read {med(warm):7.2f} us | half pre-read "
              f"{med(part):7.2f} us", flush=True)


if __name__ == "__main__":
    main()
