"""Probe: the headline decode step alone (configs[1]: B = 1 after the 288-token prefill, graph replay, greedy
feedback in place) as bench.py times it, in blocks; prints one line with the median and every block's ms per
step.  For same-box A/Bs of library builds (PGMI_LIB_PATH, tools/ab_abba.sh).
    python tools/probes/decode_only.py [--blocks 5] [--steps 40] [--batch 1]"""
import argparse
import os
import statistics
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"))
from pgmi import Engine  # noqa: E402
from pgmi.synthetic import init_policy, paligemma_3b_config, prompt_ids  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=5)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--batch", type=int, default=1)
    a = ap.parse_args()
    cfg = paligemma_3b_config(224)
    L, B = 288, a.batch
    cap = (L + 16 + a.blocks * a.steps + 8 + 63) // 64 * 64
    eng = Engine(cfg, max_batch=B, max_seq=L, max_kv=cap)
    eng.fill_synthetic(1234, init_policy)
    eng.prepare()
    g = torch.Generator(device="cuda").manual_seed(1000)
    px = (torch.rand((B, 3, 224, 224), generator=g, device="cuda") * 2 - 1).contiguous()
    ids = torch.from_numpy(prompt_ids(cfg["image_token_index"], 256, cfg["text_config"]["vocab_size"])).cuda()
    ids = ids.expand(B, -1).contiguous()
    kv = eng.new_kv(B, cap)
    lg = eng.lm_forward(kv, 0, torch.arange(L).expand(B, L), ids=ids, image_feats=eng.project(eng.vision(px)),
                        logits_rows=2)
    cur = eng.argmax(lg[:, 0])
    logits = torch.empty((B, cfg["text_config"]["vocab_size"]), dtype=torch.float32, device="cuda")
    step = 0

    def run(n):
        nonlocal step
        for _ in range(n):
            eng.decode(cur, kv, L + step, L + step + 1, logits=logits, next_ids=cur, graph=True)
            step += 1

    run(16)
    ms = []
    for _ in range(a.blocks):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(a.steps)
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t0) * 1e3 / a.steps)
    print(f"{os.environ.get('PGMI_LIB_PATH', 'libpgmi.so')}: median {statistics.median(ms):.4f} ms/step; "
          + " ".join(f"{x:.4f}" for x in ms), flush=True)


if __name__ == "__main__":
    main()
