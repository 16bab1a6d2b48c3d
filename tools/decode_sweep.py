"""Whole-step decode timing (hipGraph, batch 1, full PaliGemma-3B shapes) for launch-shape
overrides given as env assignments, one configuration per command-line argument, e.g.
  python tools/decode_sweep.py "" "PGMI_GU_RPW=1 PGMI_GU_CAP=1024" ...   (or one .txt, a line each)
Each configuration gets a fresh KV buffer, hence a fresh graph capture with its shapes."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"), REPO]
import torch  # noqa: E402

from oracle import weights as W  # noqa: E402
from pgmi import Engine  # noqa: E402

KEYS = ["PGMI_QKV_RPW", "PGMI_QKV_CAP", "PGMI_QKV_UPB", "PGMI_QKV_DEPTH", "PGMI_O_RPW", "PGMI_O_CAP", "PGMI_GU_RPW", "PGMI_GU_CAP", "PGMI_DOWN_RPW",
        "PGMI_DOWN_CAP", "PGMI_LM_RPW", "PGMI_LM_CAP", "PGMI_GU_DEPTH", "PGMI_DOWN_DEPTH", "PGMI_LM_DEPTH"]


def main():
    e = Engine(W.full_config(224), max_batch=1, max_seq=320, max_kv=512)
    e.fill_synthetic(1234, W.init_policy)
    e.prepare()
    L = 288
    base = e.new_kv(1, 512)
    ids = torch.randint(3, 4000, (1, L), device="cuda")
    e.lm_forward(base, 0, torch.arange(L)[None], ids=ids, logits_rows=1)
    tok = torch.tensor([5], device="cuda")
    logits = torch.empty((1, e.cfgd["t_vocab"]), dtype=torch.float32, device="cuda")
    nxt = torch.empty(1, dtype=torch.int64, device="cuda")
    confs = sys.argv[1:] or [""]
    if len(confs) == 1 and confs[0].endswith(".txt"):
        confs = [ln.strip() for ln in open(confs[0])]
    for conf in confs:
        for k in KEYS:
            os.environ.pop(k, None)
        for kv_ in conf.split():
            k, v = kv_.split("=")
            os.environ[k] = v
        kv = base.clone()
        best = 1e9
        for rep in range(3):
            for t in range(4):
                e.decode(tok, kv, L + t, L + t + 1, logits=logits, next_ids=nxt, graph=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 64
            for t in range(n):
                e.decode(tok, kv, L + 4 + t, L + 5 + t, logits=logits, next_ids=nxt, graph=True)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / n)
        print(f"{best * 1e3:7.4f} ms/step  {1 / best:7.1f} tok/s   [{conf or 'defaults'}]", flush=True)


if __name__ == "__main__":
    main()
