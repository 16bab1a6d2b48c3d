"""Probe: does a weight stream read faster from the Infinity Cache (256 MiB) than from HBM?  Times the
decode gate|up GEMV (pgmi_decode_kernel 2, 134 MB of weights per layer) with its weights cold
(a 320 MB junk sweep in between) and after pgmi_op_prefetch of the first `frac` of them, and
the prefetch kernel's own rate per grid size.

    python tools/probes/prefetch_probe.py
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"))
from pgmi import Engine, _native as N  # noqa: E402
from pgmi.synthetic import init_policy, paligemma_3b_config  # noqa: E402


def main():
    cfg = paligemma_3b_config(224)
    eng = Engine(cfg, max_batch=1, max_seq=320, max_kv=512)
    eng.fill_synthetic(1234, init_policy)
    eng.prepare()
    s = torch.cuda.current_stream()
    junk = torch.empty(320 << 20, dtype=torch.uint8, device="cuda")
    gu_bytes = 2 * 16384 * 2048 * 2

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def flush():
        N.check(eng.lib.pgmi_op_prefetch(eng.ctx, junk.data_ptr(), junk.numel(), 512, s.cuda_stream))

    def gateup(layer):
        N.check(eng.lib.pgmi_decode_kernel(eng.ctx, 2, layer, 1, s.cuda_stream))

    for i in range(18):
        gateup(i)
    torch.cuda.synchronize()
    for blocks in (64, 128, 256, 512, 1024):
        flush()
        e0, e1 = ev(), ev()
        e0.record(s)
        N.check(eng.lib.pgmi_op_prefetch(eng.ctx, eng.views["language_model.model.layers.3.mlp.gate_proj.weight"].data_ptr(),
                                         gu_bytes, blocks, s.cuda_stream))
        e1.record(s)
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3
        print(f"prefetch 134 MB with {blocks} WGs: {us:.1f} us = {gu_bytes / us / 1e6:.2f} TB/s", flush=True)
    for frac in (0.0, 0.25, 0.5, 0.75, 1.0):
        ts = []
        for rep in range(5):
            layer = 2 + rep
            flush()
            base = eng.views[f"language_model.model.layers.{layer}.mlp.gate_proj.weight"]
            nb = int(frac * 16384 * 2048 * 2)  # the first frac of the gate rows and of the up rows
            if nb:
                N.check(eng.lib.pgmi_op_prefetch(eng.ctx, base.data_ptr(), nb, 512, s.cuda_stream))
                N.check(eng.lib.pgmi_op_prefetch(eng.ctx, base.data_ptr() + 16384 * 2048 * 2, nb, 512, s.cuda_stream))
            e0, e1 = ev(), ev()
            e0.record(s)
            gateup(layer)
            e1.record(s)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        print(f"gate|up after prefetching {frac:.2f} of its weights: median {ts[2]:.2f} us (min {ts[0]:.2f})", flush=True)


if __name__ == "__main__":
    main()
