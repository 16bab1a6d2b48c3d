"""First contact with the fused decode step: one small-config step, eager then graph, status
and bit-equality against the per-phase launches.  Exits non-zero on any mismatch."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"), REPO]
import torch  # noqa: E402

from oracle import weights as W  # noqa: E402
from pgmi import Engine  # noqa: E402


def main():
    cfg = W.small_config(vision_layers=1, text_layers=2, vocab=4096)
    e = Engine(cfg, max_batch=1, max_seq=320, max_kv=512)
    e.fill_synthetic(1234, W.init_policy)
    e.prepare()
    kv = e.new_kv(1, 512)
    kv.zero_()
    L = 20
    ids = torch.randint(3, 4000, (1, L), device="cuda")
    e.lm_forward(kv, 0, torch.arange(L)[None], ids=ids, logits_rows=1, image_feats=None)
    kv2 = kv.clone()
    tok = torch.tensor([5], device="cuda")
    e.set_decode_fused(True)
    la = e.decode(tok, kv, L, L + 1, graph=False).clone()
    torch.cuda.synchronize()
    st = e.decode_status()
    print("fused eager status", st, flush=True)
    e.set_decode_fused(False)
    lb = e.decode(tok, kv2, L, L + 1, graph=False).clone()
    torch.cuda.synchronize()
    d = (la - lb).abs().max().item()
    print("max |fused - per-phase| =", d, "equal:", torch.equal(la, lb), flush=True)
    if st != 0 or not torch.equal(la, lb):
        sys.exit(1)
    e.set_decode_fused(True)
    for t in range(1, 6):
        la = e.decode(tok, kv, L + t, L + t + 1, graph=True).clone()
        e.set_decode_fused(False)
        lb = e.decode(tok, kv2, L + t, L + t + 1, graph=True).clone()
        e.set_decode_fused(True)
        torch.cuda.synchronize()
        print("graph step", t, "equal:", torch.equal(la, lb), "status", e.decode_status(), flush=True)
        if not torch.equal(la, lb):
            sys.exit(1)
    print("fused smoke ok")


if __name__ == "__main__":
    main()
