"""Host time of one graphed decode-step call (pgmi_decode through pgmi/engine.py), full PaliGemma-3B shapes,
batch 1, the GPU drained before each call so nothing but the call itself is timed.

Two forms: the ids buffer is the step's next_ids (in-place feedback, no staging copy; the bench's form), and a
fresh ids tensor per call (the drop-in loop's form: the step stages it into the context's buffer with a
device-to-device copy before the graph launch).  Prints the median host microseconds of each over 200 calls.
usage: python tools/probes/decode_host_cost.py
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "multimodal-financial-analysis-tool-using-paligemma_amd"))


def main():
    import torch

    from pgmi import Engine
    from pgmi.synthetic import init_policy, paligemma_3b_config

    e = Engine(paligemma_3b_config(224), device=torch.device("cuda:0"), max_batch=1, max_seq=320, max_kv=576)
    e.fill_synthetic(7, init_policy)
    e.prepare()
    kv = e.new_kv(1, 576)
    logits = e.logits_buffer(1)
    nxt = torch.zeros(1, dtype=torch.int64, device="cuda")
    res = {}
    for form in ("in_place", "fresh_ids", "in_place", "fresh_ids"):
        ts = []
        for t in range(8 + 200):
            ids = nxt if form == "in_place" else torch.full((1,), 3, dtype=torch.int64, device="cuda")
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e.decode(ids, kv, 300 + (t % 200), 300 + (t % 200), logits=logits, next_ids=nxt, graph=True)
            t1 = time.perf_counter()
            if t >= 8:
                ts.append((t1 - t0) * 1e6)
        torch.cuda.synchronize()
        res.setdefault(form, []).append(statistics.median(ts))
    for k, v in res.items():
        print(f"{k:10s} host us per call (median of 200), two passes: " + " / ".join(f"{x:.1f}" for x in v))


if __name__ == "__main__":
    main()
