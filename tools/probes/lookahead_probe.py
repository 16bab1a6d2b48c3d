"""Timeline of the drop-in decode loop with the greedy lookahead (pgmi/lookahead.py).

Drives inference.py:55-78's loop through the drop-in module (as bench.py time_api) and records, per token:
host time of the user ops (argmax + .item()), of the forward call and of its parts inside
GreedyLookahead.step (before the check's host wait, the wait itself); on the GPU, timing events around
every graphed step (on whichever stream runs it), so the gaps between consecutive steps show what the
chain of steps waits for.  Prints medians over 48 tokens after 16 warm-up tokens, for lookahead on and off.
usage: python tools/probes/lookahead_probe.py
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "multimodal-financial-analysis-tool-using-paligemma_amd"))


def main():
    import torch

    import modeling_gemma as MG
    import utils as U
    from pgmi import lookahead as LA
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

    gpu = []   # (start event, end event) of every step, in enqueue order
    host = {}
    orig_decode = eng.decode

    def timed_decode(*a, **k):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        r = orig_decode(*a, **k)
        e.record()
        gpu.append((s, e))
        return r

    eng.decode = timed_decode
    orig_sync = torch.cuda.Event.synchronize

    def run(lookahead):
        m.pgmi_lookahead = lookahead
        gpu.clear()
        rows = []
        with torch.no_grad():
            kv = MG.KVCache()
            mask = torch.ones_like(ids0)
            out = m(input_ids=ids0, pixel_values=px, attention_mask=mask, kv_cache=kv)
            for step in range(16 + 48):
                t0 = time.perf_counter()
                nxt = torch.argmax(out["logits"][:, -1, :], dim=-1, keepdim=True).squeeze(0)
                _ = nxt.item()
                t1 = time.perf_counter()
                ids = nxt.unsqueeze(-1)
                mask = torch.cat([mask, torch.ones((1, 1), device=dev)], dim=-1)
                host.clear()
                t2 = time.perf_counter()
                out = m(input_ids=ids, pixel_values=px, attention_mask=mask, kv_cache=kv)
                t3 = time.perf_counter()
                rows.append((t1 - t0, t2 - t1, t3 - t2, host.get("sync", 0.0)))
            torch.cuda.synchronize()
        rows = rows[16:]
        med = lambda i: statistics.median(r[i] for r in rows) * 1e6  # noqa: E731
        tot = statistics.median(sum(r[:3]) for r in rows) * 1e6
        starts = [s for s, _ in gpu]
        ref = starts[0]
        st = [ref.elapsed_time(s) * 1e3 for s, _ in gpu]
        du = [s.elapsed_time(e) * 1e3 for s, e in gpu]
        gaps = [st[i + 1] - (st[i] + du[i]) for i in range(len(st) - 1)]
        tail = slice(len(gaps) - 48, len(gaps))
        print(f"lookahead={lookahead}: per token (us, median of 48): total {tot:.1f}; user argmax+.item() {med(0):.1f}; "
              f"ids/mask {med(1):.1f}; forward {med(2):.1f} (of which the check's host wait {med(3):.1f})")
        print(f"  GPU steps: duration median {statistics.median(du[tail]):.1f} us; gap to the next step median "
              f"{statistics.median(gaps[tail]):.1f}, min {min(gaps[tail]):.1f}, max {max(gaps[tail]):.1f} us; "
              f"steps recorded {len(gpu)}")

    def timed_sync(self):
        t = time.perf_counter()
        orig_sync(self)
        host["sync"] = host.get("sync", 0.0) + time.perf_counter() - t

    torch.cuda.Event.synchronize = timed_sync
    for la in (False, True, False, True):
        run(la)
    hits = getattr(getattr(eng, "_lookahead", None), "hits", None)
    print("lookahead hits", hits, "LA module", LA.__file__)
    if os.environ.get("LA_PROBE_NOCHECK"):
        # what the padding check's GPU ops (a side stream's compare + copy per token) cost the loop: the
        # check replaced by nothing (probe only)
        class _NoCheck:
            def __init__(self, mask):
                pass

            def launch(self):
                pass

            def wait(self):
                pass

        MG._PaddingCheck = _NoCheck
        print("# padding check off")
        for la in (True, True):
            run(la)
    if os.environ.get("LA_PROBE_NOCLONE"):
        # what the hit's logits copy on the caller's stream costs: the slot handed out as is (probe only -- the
        # slot is rewritten three steps later)
        def take_noclone(self, kv_cache, slab, cache_len, position, s, done, ne, graph, after_launch):
            main = torch.cuda.current_stream(self.eng.device)
            self.flag.copy_(ne, non_blocking=True)
            self.ev_chk.record(main)
            if after_launch is not None:
                after_launch()
            self._ahead(kv_cache, slab, cache_len + 1, position + 1, (s + 1) % LA.NSLOT, graph, False)
            self.ev_chk.synchronize()
            done.synchronize()
            if not bool(self.flag):
                kv_cache._pgmi_misses = 0
                self.hits += 1
                return self.logits[s].unsqueeze(1)
            kv_cache._pgmi_misses = getattr(kv_cache, "_pgmi_misses", 0) + 1
            self.pending = None
            return None

        LA.GreedyLookahead._take = take_noclone
        print("# logits copy off")
        for la in (True, True):
            run(la)


if __name__ == "__main__":
    main()
