"""Probe: sha1 of B-row lock-step decode outputs (logits of a few eager steps + the KV cache) at full
PaliGemma-3B shapes on synthetic weights, under each environment setting given on the command
line (KEY=VALUE,...; '-' = defaults) -- a bit-identity check of alternative batched-decode kernels.
    python tools/probes/batched_decode_digest.py - PGMI_MF_QKV_ROWS=0"""
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


B = 8
eng = Engine(paligemma_3b_config(224), max_batch=B, max_seq=300, max_kv=320)
eng.fill_synthetic(1234, init_policy)
eng.prepare()
cfg = eng.cfgd
g = torch.Generator().manual_seed(7)
px = (torch.rand((B, 3, 224, 224), generator=g) * 2 - 1).cuda()
ids = torch.from_numpy(prompt_ids(cfg["image_token_index"], 256, cfg["t_vocab"])).cuda().expand(B, -1).contiguous()
L = ids.shape[1]
feats = eng.project(eng.vision(px))
for setting in sys.argv[1:] or ["-"]:
    saved = dict(os.environ)
    if setting != "-":
        for kv in setting.split(","):
            k, v = kv.split("=")
            os.environ[k] = v
    kv = eng.new_kv(B, 320)
    lg = eng.lm_forward(kv, 0, torch.arange(L).expand(B, L), ids=ids, image_feats=feats, logits_rows=1)[:, 0]
    tok = eng.argmax(lg)
    outs = []
    for t in range(3):
        lg = eng.decode(tok, kv, L + t, L + 1 + t).clone()
        outs.append(lg)
        tok = eng.argmax(lg)
    torch.cuda.synchronize()
    print(setting, "logits", sha(torch.stack(outs)), "kv", sha(kv[:, :, :, :L + 3]), flush=True)
    os.environ.clear()
    os.environ.update(saved)
