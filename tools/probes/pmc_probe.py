"""Probe for per-kernel PMC passes (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ counters): the
PaliGemma-3B 224 px path with few dispatches -- one prefill and a few eager decode steps at batch
1, then the same at batch 8 (configs[3]) -- so a counter pass finishes in seconds (bench.py's
every-leg run is too long for a FETCH_SIZE pass).  Synthetic weights and inputs.
    rocprofv3 --pmc FETCH_SIZE -- python3 tools/probes/pmc_probe.py [steps] [448]
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"), REPO]
from pgmi import Engine  # noqa: E402
from pgmi.synthetic import init_policy, paligemma_3b_config, prompt_ids  # noqa: E402


def run(eng, cfg, B, steps, size=224):
    n_img = (size // 14) ** 2
    L = n_img + 32
    px = (torch.rand((B, 3, size, size), device="cuda") * 2 - 1).contiguous()
    ids = torch.from_numpy(prompt_ids(cfg["image_token_index"], n_img, cfg["text_config"]["vocab_size"])).cuda()
    ids = ids.expand(B, -1).contiguous()
    pos = torch.arange(L).expand(B, L)
    kv = eng.new_kv(B, L + steps + 64)
    feats = eng.project(eng.vision(px))
    lg = eng.lm_forward(kv, 0, pos, ids=ids, image_feats=feats, logits_rows=1)
    cur = eng.argmax(lg[:, 0])
    logits = torch.empty((B, cfg["text_config"]["vocab_size"]), dtype=torch.float32, device="cuda")
    for step in range(1, steps + 1):
        eng.decode(cur, kv, L + step - 1, L + step, logits=logits, next_ids=cur, graph=False)
    torch.cuda.synchronize()
    print(f"B={B} {size} px: prefill + {steps} decode steps done", flush=True)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    cfg = paligemma_3b_config(224)
    eng = Engine(cfg, max_batch=8, max_seq=288, max_kv=288 + steps + 64)
    eng.fill_synthetic(1234, init_policy)
    eng.prepare()
    torch.manual_seed(0)
    run(eng, cfg, 1, steps)
    run(eng, cfg, 8, steps)
    if len(sys.argv) > 2 and sys.argv[2] == "448":  # configs[4]: the 448 px prefill (M = 1,056 GEMMs on k_gemm_8p)
        del eng
        torch.cuda.empty_cache()
        cfg4 = paligemma_3b_config(448)
        e4 = Engine(cfg4, max_batch=1, max_seq=1056, max_kv=1056 + steps + 64)
        e4.fill_synthetic(1234, init_policy)
        e4.prepare()
        run(e4, cfg4, 1, steps, 448)


if __name__ == "__main__":
    main()
