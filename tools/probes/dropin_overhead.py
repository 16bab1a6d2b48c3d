"""Host-side cost of the drop-in decode loop (inference.py:55-78 through modeling_gemma.py).

Times, per token over 64 tokens after 8 warm-up tokens, the user-side ops of the reference loop
(argmax + .item(), the next ids and the float mask column) and the module forward call, and prints
a cProfile of 32 forward calls (cumulative, top entries).  The GPU step itself is ~1.05 ms; what the
forward call's host time adds before the graph launch is exposed by the loop's .item() sync.
usage: python tools/probes/dropin_overhead.py
"""
import cProfile
import os
import pstats
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "multimodal-financial-analysis-tool-using-paligemma_amd"))


def main():
    import torch

    import modeling_gemma as MG
    import utils as U
    from pgmi.synthetic import init_policy, paligemma_3b_config, prompt_ids

    dev = torch.device("cuda:0")
    cfg = paligemma_3b_config(224)
    pcfg = MG.PaliGemmaConfig(**{k: v for k, v in cfg.items() if k not in ("bos_token_id", "eos_token_id")})
    m = U.build_model(pcfg, device=dev)
    m.tie_weights()
    eng = m._pgmi_engine()
    eng.fill_synthetic(7, init_policy)
    eng.prepare()
    ids0 = torch.from_numpy(prompt_ids(cfg["image_token_index"], 256, cfg["text_config"]["vocab_size"])).to(dev)
    px = (torch.rand((1, 3, 224, 224), device=dev) * 2 - 1).contiguous()
    marks = {}
    orig_decode = eng.decode

    def timed_decode(*a, **k):
        marks["d0"] = time.perf_counter()
        r = orig_decode(*a, **k)
        marks["d1"] = time.perf_counter()
        return r

    eng.decode = timed_decode
    pre, dec, post, cat_t = [], [], [], []
    with torch.no_grad():
        kv = MG.KVCache()
        mask = torch.ones_like(ids0)
        out = m(input_ids=ids0, pixel_values=px, attention_mask=mask, kv_cache=kv)
        t_user, t_fwd, t_tot = [], [], []
        prof = cProfile.Profile()
        for step in range(8 + 64 + 32):
            t0 = time.perf_counter()
            nxt = torch.argmax(out["logits"][:, -1, :], dim=-1, keepdim=True).squeeze(0)
            _ = nxt.item()
            ta = time.perf_counter()
            ids = nxt.unsqueeze(-1)
            mask = torch.cat([mask, torch.ones((1, 1), device=dev)], dim=-1)
            t1 = time.perf_counter()
            if step >= 72:
                prof.enable()
            out = m(input_ids=ids, pixel_values=px, attention_mask=mask, kv_cache=kv)
            if step >= 72:
                prof.disable()
            t2 = time.perf_counter()
            if 8 <= step < 72:
                pre.append((marks["d0"] - t1) * 1e6)
                dec.append((marks["d1"] - marks["d0"]) * 1e6)
                post.append((t2 - marks["d1"]) * 1e6)
                cat_t.append((t1 - ta) * 1e6)
                t_user.append((t1 - t0) * 1e3)
                t_fwd.append((t2 - t1) * 1e3)
                t_tot.append((t2 - t0) * 1e3)
        torch.cuda.synchronize()
    print(f"per token (ms, median of 64): user ops incl. .item() wait {statistics.median(t_user):.4f}, "
          f"forward call {statistics.median(t_fwd):.4f}, total {statistics.median(t_tot):.4f}")
    print(f"us, median: after .item() to forward call {statistics.median(cat_t):.1f}; forward entry to "
          f"eng.decode {statistics.median(pre):.1f}; eng.decode {statistics.median(dec):.1f}; after it "
          f"{statistics.median(post):.1f}")
    st = pstats.Stats(prof)
    st.sort_stats("cumulative").print_stats(28)


if __name__ == "__main__":
    main()
