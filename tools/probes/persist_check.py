"""Decode-step probe of the one-launch MLP half (kernels_persist.hip) at the full 3B shapes.

Runs a 64-token text prefill and 48 teacher-forced graph-replayed decode steps (B = 1) on synthetic
weights, prints pgmi_persist_status and writes the per-step logits (every 16th vocabulary entry) and
argmax to an npz.  Run it with PGMI_PERSIST=0 and =1 (the switch is read once per process) and
compare the two files with --compare a.npz b.npz: per-step rel-L2 and argmax agreement.
usage: python tools/probes/persist_check.py OUT.npz | --compare A.npz B.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "multimodal-financial-analysis-tool-using-paligemma_amd"))


def run(out):
    import ctypes

    import torch

    from pgmi import Engine
    from pgmi.synthetic import init_policy, paligemma_3b_config

    cfg = paligemma_3b_config(224)
    eng = Engine(cfg, device="cuda:0", max_batch=1, max_seq=64, max_kv=256)
    eng.fill_synthetic(7, init_policy)
    eng.prepare()
    V = cfg["text_config"]["vocab_size"]
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(3, V - 1000, (1, 64), generator=g)
    forced = torch.randint(3, V - 1000, (48,), generator=g)
    kv = eng.new_kv(1, 256)
    eng.lm_forward(kv, 0, torch.arange(64), ids=ids.cuda(), logits_rows=2)
    logits = torch.empty((1, V), dtype=torch.float32, device="cuda:0")
    rows, top = [], []
    tok = torch.empty((1,), dtype=torch.int64, device="cuda:0")
    for t in range(48):
        tok.fill_(int(forced[t]))
        eng.decode(tok, kv, 64 + t, 64 + t, logits=logits, graph=True)
        rows.append(logits[0, ::16].float().cpu().numpy())
        top.append(int(logits[0].argmax()))
    torch.cuda.synchronize()
    act, gave = ctypes.c_int(0), ctypes.c_int(0)
    rc = eng.lib.pgmi_persist_status(eng.ctx, ctypes.byref(act), ctypes.byref(gave))
    print(f"persist_status rc={rc} active={act.value} gave_up={gave.value}")
    if os.environ.get("PGMI_PERSIST_DBG") == "1":
        buf = (ctypes.c_uint64 * (256 * 16))()
        eng.lib.pgmi_persist_debug(eng.ctx, ctypes.addressof(buf), 256 * 16)
        d = np.array(buf, dtype=np.int64).reshape(256, 16)
        t0 = d[:, 0].min()
        names = {1: "ldr first gu issued", 2: "ldr first down issued", 3: "ldr end", 5: "cw0 combine done",
                 6: "cw0 x ready", 8: "cw0 act gathered", 9: "cw1 act gathered", 10: "cw2 act gathered",
                 11: "act barrier", 12: "cw0 end", 13: "cw1 end", 14: "cw2 end"}
        print("start spread (us): %.2f" % ((d[:, 0].max() - t0) / 100.0))
        for k, nm in names.items():
            v = (d[:, k] - t0) / 100.0
            print(f"  {nm:24s} min {v.min():7.2f} med {np.median(v):7.2f} max {v.max():7.2f} us")
        print("  loader waited on free: med %.2f max %.2f us" % (np.median(d[:, 4]) / 100.0, d[:, 4].max() / 100.0))
    np.savez(out, logits=np.stack(rows), top=np.array(top), active=act.value, gave_up=gave.value)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    la, lb = A["logits"].astype(np.float64), B["logits"].astype(np.float64)
    rel = np.linalg.norm(la - lb, axis=1) / np.linalg.norm(lb, axis=1)
    agree = float((A["top"] == B["top"]).mean())
    print(f"active {int(A['active'])}/{int(B['active'])} gave_up {int(A['gave_up'])}/{int(B['gave_up'])} "
          f"rel-L2 mean {rel.mean():.3e} max {rel.max():.3e} argmax agreement {agree:.3f}")
    return rel.max(), agree


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        r, ag = compare(sys.argv[2], sys.argv[3])
        sys.exit(0 if r < 2e-2 else 1)
    run(sys.argv[1])
