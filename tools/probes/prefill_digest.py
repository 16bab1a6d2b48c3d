"""Probe: sha1 of the 224 px prefill outputs (last-row logits with logits_rows 1 and 2, every row's
logits, the KV cache) at full PaliGemma-3B shapes on synthetic weights -- run once per library
build (PGMI_LIB_PATH) to check that a kernel rewrite is bit-identical.
    python tools/probes/prefill_digest.py"""
import hashlib
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"), REPO]
from pgmi import Engine  # noqa: E402
from pgmi.synthetic import init_policy, paligemma_3b_config, prompt_ids  # noqa: E402


def sha(t):
    return hashlib.sha1(t.contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:16]


eng = Engine(paligemma_3b_config(224), max_batch=2, max_seq=300, max_kv=320)
eng.fill_synthetic(1234, init_policy)
eng.prepare()
g = torch.Generator().manual_seed(7)
px = (torch.rand((2, 3, 224, 224), generator=g) * 2 - 1).cuda()
cfg = eng.cfgd
ids = torch.from_numpy(prompt_ids(cfg["image_token_index"], 256, cfg["t_vocab"])).cuda().expand(2, -1).contiguous()
L = ids.shape[1]
pos = torch.arange(L).expand(2, L)
feats = eng.project(eng.vision(px))
out = {"vision": sha(feats)}
for rows in (0, 1, 2):
    kv = eng.new_kv(2, 320)
    lg = eng.lm_forward(kv, 0, pos, ids=ids, image_feats=feats, logits_rows=rows)
    torch.cuda.synchronize()
    out[f"logits_rows{rows}"] = sha(lg)
    out[f"kv_rows{rows}"] = sha(kv[:, :, :, :L])
print(out, flush=True)
