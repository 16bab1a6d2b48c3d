"""Probe: the B = 1 decode step (bench.py's workload: 224 px prompt, greedy, graph replay) with the
per-layer gate|up weight prefetch into the Infinity Cache (pgmi_set_decode_prefetch) at several
sizes and grid widths; tokens must be identical to the prefetch-off run.

    python tools/probes/decode_prefetch_sweep.py [--steps 128] [--batch 1]
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"))
from pgmi import Engine, _native as N  # noqa: E402
from pgmi.synthetic import init_policy, paligemma_3b_config, prompt_ids  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--mb", default="0,16,32,48,64,96,134")
    ap.add_argument("--blocks", default="32,64,128")
    a = ap.parse_args()
    cfg = paligemma_3b_config(224)
    B, L = a.batch, 288
    cap = 1024
    e = Engine(cfg, max_batch=B, max_seq=L, max_kv=cap)
    e.fill_synthetic(1234, init_policy)
    e.prepare()
    g = torch.Generator(device="cuda").manual_seed(1000)
    px = (torch.rand((B, 3, 224, 224), generator=g, device="cuda") * 2 - 1).contiguous()
    ids = torch.from_numpy(prompt_ids(cfg["image_token_index"], 256, cfg["text_config"]["vocab_size"])).cuda()
    ids = ids.expand(B, -1).contiguous()
    kv = e.new_kv(B, cap)
    feats = e.project(e.vision(px))
    lg = e.lm_forward(kv, 0, torch.arange(L).expand(B, L), ids=ids, image_feats=feats, logits_rows=2)
    first = e.argmax(lg[:, 0])
    logits = torch.empty((B, cfg["text_config"]["vocab_size"]), dtype=torch.float32, device="cuda")

    def run(steps):
        cur = first.clone()
        toks = []
        for t in range(steps):
            e.decode(cur, kv, L + t, L + t + 1, logits=logits, next_ids=cur, graph=True)
            toks.append(cur.clone())
        return torch.stack(toks, 1)

    ref = None
    for mb in [int(x) for x in a.mb.split(",")]:
        for blocks in ([64] if mb == 0 else [int(x) for x in a.blocks.split(",")]):
            N.check(e.lib.pgmi_set_decode_prefetch(e.ctx, mb << 20, blocks))
            run(8)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            toks = run(a.steps)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / a.steps
            same = True if ref is None else bool(torch.equal(toks, ref))
            if ref is None:
                ref = toks
            print(f"prefetch {mb:4d} MB/layer, {blocks:4d} WGs: {ms:.4f} ms/step = {B / ms * 1e3:7.1f} tok/s"
                  f"  tokens {'identical' if same else 'DIFFER'}", flush=True)
    N.check(e.lib.pgmi_set_decode_prefetch(e.ctx, 0, 64))


if __name__ == "__main__":
    main()
