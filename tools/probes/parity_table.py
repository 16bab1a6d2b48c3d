"""Model-level parity table: per-step logits rel-L2 against the reference bf16
(<= 2e-2) and the reference bf16's own rel-L2 against its fp32 truth, on every
full-size fixture, with the default prefill attention and with the exactly-rounded kernels forced
(pgmi_tune_attention 8: k_attn_full_pre for Gemma <= 320 keys, k_attn_full for SigLIP).

  python tools/probes/parity_table.py [--out gpurun_out/parity.jsonl] [--quick]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"), REPO,
          os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import weights as W  # noqa: E402
from tests_helpers import logit_stats, pixels_from_u8  # noqa: E402

GOLD = os.path.join(REPO, "tests", "golden")
SEED = 1234


def load(n):
    return np.load(os.path.join(GOLD, n))


def engine(size, max_batch=1, max_seq=320, max_kv=576):
    from pgmi import Engine
    e = Engine(W.full_config(size), max_batch=max_batch, max_seq=max_seq, max_kv=max_kv)
    e.fill_synthetic(SEED, W.init_policy)
    e.prepare()
    return e


@torch.no_grad()
def teacher_forced(e, px, gb, n):
    ids = torch.from_numpy(gb["ids"]).cuda()
    L = ids.shape[1]
    ref = gb["tokens"].reshape(-1)
    kv = e.new_kv(1, 576)
    feats = e.project(e.vision(px))
    out = [e.lm_forward(kv, 0, torch.arange(L)[None], ids=ids, image_feats=feats, logits_rows=1)[:, 0]]
    for t in range(1, n):
        cur = torch.tensor([int(ref[t - 1])], device="cuda")
        out.append(e.decode(cur, kv, L + t - 1, L + t, graph=True).clone())
    return torch.cat(out, 0)[:, torch.from_numpy(gb["sample_idx"]).cuda()].cpu().numpy()


@torch.no_grad()
def batch8(e, G, F, B=8, n=64):
    px = torch.from_numpy(np.stack([pixels_from_u8(G["u8"][b]) for b in range(B)])).cuda()
    ids = torch.from_numpy(G["ids"][:B]).cuda()
    L = ids.shape[1]
    kv = e.new_kv(B, 384)
    feats = e.project(e.vision(px))
    lg = e.lm_forward(kv, 0, torch.arange(L).expand(B, L), ids=ids, image_feats=feats, logits_rows=1)[:, 0]
    steps = [lg.clone()]
    logits = torch.empty_like(lg)
    for t in range(1, n):
        cur = torch.from_numpy(G["tokens"][:B, t - 1].copy()).cuda()
        e.decode(cur, kv, L + t - 1, L + t, logits=logits, graph=True)
        steps.append(logits.clone())
    ours = torch.stack(steps, 1)[:, :, torch.from_numpy(G["sample_idx"]).cuda()].cpu().numpy()
    return ours


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "parity.jsonl"))
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    os.environ["PGMI_PARITY_LOG"] = a.out
    from pgmi import _native as N
    lib = N.lib()
    px = load("pixels.npz")
    px224 = torch.from_numpy(pixels_from_u8(px["u8_0_224"])[None]).cuda()
    e = engine(224)
    g64, f64 = load("full_bf16.npz"), load("full_fp32.npz")
    g256, f256 = load("full256_bf16.npz"), load("full256_fp32.npz")
    for variant, name in ((-1, "default"), (8, "exact")):
        lib.pgmi_tune_attention(variant)
        e.set_prefill_graph(True)  # drops captured prefill graphs: the next prefill runs the forced kernel
        logit_stats(f"tf64/{name}", teacher_forced(e, px224, g64, 64), g64["sample_vals"], f64["sample_vals"])
        if not a.quick:
            logit_stats(f"tf256/{name}", teacher_forced(e, px224, g256, 256), g256["sample_vals"],
                        f256["sample_vals"])
    lib.pgmi_tune_attention(-1)
    del e
    torch.cuda.empty_cache()
    if not a.quick:
        G, F = load("full_batch8_bf16.npz"), load("full_batch8_fp32.npz")
        e = engine(224, max_batch=8, max_seq=288, max_kv=384)
        ours = batch8(e, G, F)
        for b in range(8):
            logit_stats(f"batch8/row{b}", ours[b], G["sample_vals"][b], F["sample_vals"][b])
        del e
        torch.cuda.empty_cache()
    # smoke's small configuration against the oracle in bf16 and in fp32-truth mode
    from oracle import paligemma_np as O
    from pgmi import Engine
    cfg = W.small_config(vision_layers=1, text_layers=2, vocab=4096)
    es = Engine(cfg, device="cuda:0", max_batch=1, max_seq=320, max_kv=512)
    es.fill_synthetic(SEED, W.init_policy)
    es.prepare()
    rng = np.random.default_rng(0)
    pxs = O.bf16(rng.uniform(-1, 1, (1, 3, 224, 224)).astype(np.float32))
    n_img = W.num_image_tokens(cfg)
    ids = np.array([[cfg["image_token_index"]] * n_img + [2] + list(rng.integers(3, 4000, 30)) + [108]])
    P = W.synthetic_state_dict_f32(cfg, SEED)
    _, ref_b = O.greedy_generate(P, cfg, ids, pxs, 1)
    with O.fp32_truth():
        _, ref_f = O.greedy_generate(P, cfg, ids, pxs, 1)
    kv = es.new_kv(1, 512)
    L = ids.shape[1]
    feats = es.project(es.vision(torch.from_numpy(pxs).cuda()))
    lg = es.lm_forward(kv, 0, torch.arange(L)[None], ids=torch.from_numpy(ids).cuda(), image_feats=feats,
                       logits_rows=1)[0, 0].cpu().numpy()
    logit_stats("smoke/prefill", lg[None], ref_b[0, :1], ref_f[0, :1])


if __name__ == "__main__":
    main()
