"""Diagnose fused-step mismatches: fused graph / fused eager / per-phase graph vs per-phase
eager (reference), small config with the golden prompt, 40 steps."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"), REPO, os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import paligemma_np as O  # noqa: E402
from oracle import weights as W  # noqa: E402
from pgmi import Engine  # noqa: E402


def main():
    gold = np.load(os.path.join(REPO, "tests", "golden", "small_bf16.npz"))
    cfg = W.small_config()
    e = Engine(cfg, max_batch=4, max_seq=640, max_kv=1024)
    e.fill_synthetic(1234, W.init_policy)
    e.prepare()
    px = torch.from_numpy(O.from_bits(gold["pixels_bits"])).cuda()
    ids = torch.from_numpy(gold["ids"]).cuda()
    L = ids.shape[1]
    feats = e.project(e.vision(px))
    kv0 = e.new_kv(1, 1024)
    kv0.zero_()
    e.lm_forward(kv0, 0, torch.arange(L)[None], ids=ids, image_feats=feats, logits_rows=1)
    modes = {"fused_graph": (True, True), "fused_eager": (True, False), "phase_graph": (False, True),
             "phase_eager": (False, False)}
    kvs = {m: kv0.clone() for m in modes}
    tok = torch.tensor([108], device="cuda")
    bad = 0
    for t in range(int(sys.argv[1]) if len(sys.argv) > 1 else 40):
        out = {}
        for m, (fu, gr) in modes.items():
            e.set_decode_fused(fu)
            out[m] = e.decode(tok, kvs[m], L + t, L + t + 1, graph=gr).clone()
        torch.cuda.synchronize()
        ref = out["phase_eager"]
        msg = []
        for m in modes:
            if m != "phase_eager" and not torch.equal(out[m], ref):
                msg.append(f"{m}:{(out[m] - ref).abs().max().item():.3g}")
                bad += 1
        st = e.decode_status()
        print(f"t={t} status={st} " + (" ".join(msg) if msg else "all equal"), flush=True)
        # resync every cache to the reference so a mismatch does not propagate
        for m in modes:
            if m != "phase_eager":
                kvs[m].copy_(kvs["phase_eager"])
        tok = ref.argmax(-1)
    print("mismatching (mode, step) pairs:", bad)


if __name__ == "__main__":
    main()
