"""Why the drop-in lookahead's steps run slower than steps on demand (tools/probes/lookahead_probe.py: 1.166 vs
1.073 ms per graphed step).  Times the graphed decode step back to back (48 steps after 8 warm-up) in four
settings, GPU events around each call on the stream that runs it:
  A  the caller's stream, one logits / ids buffer (the on-demand form)
  B  a side stream, same buffers
  C  the caller's stream, the lookahead's three rotating logits / ids / next_ids slots
  D  as C on a side stream, with the drop-in loop's small per-token ops (argmax, ne/any, clone) on the caller's
     stream beside each step
usage: python tools/probes/stream_probe.py
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "multimodal-financial-analysis-tool-using-paligemma_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch

    from oracle import weights as W
    from pgmi import Engine
    from pgmi.synthetic import init_policy, prompt_ids

    cfg = W.full_config(224)
    e = Engine(cfg, max_batch=1, max_seq=320, max_kv=576)
    e.fill_synthetic(7, init_policy)
    e.prepare()
    dev = e.device
    ids0 = torch.from_numpy(prompt_ids(cfg["image_token_index"], 256, cfg["text_config"]["vocab_size"])).to(dev)
    L = ids0.shape[1]
    px = (torch.rand((1, 3, 224, 224), device=dev) * 2 - 1).contiguous()
    V = cfg["text_config"]["vocab_size"]

    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")

    def hip_stream(flags, prio=None):
        h = ctypes.c_void_p()
        if prio is None:
            assert hip.hipStreamCreateWithFlags(ctypes.byref(h), ctypes.c_uint(flags)) == 0
        else:
            assert hip.hipStreamCreateWithPriority(ctypes.byref(h), ctypes.c_uint(flags), ctypes.c_int(prio)) == 0
        return torch.cuda.ExternalStream(h.value)

    def run(label, side, rotate, extra, graph=True, waits=False, nowait=False):
        kv = e.new_kv(1, 576)
        feats = e.project(e.vision(px))
        e.lm_forward(kv, 0, torch.arange(L)[None], ids=ids0, image_feats=feats, logits_rows=1)
        lg = [torch.empty((1, V), device=dev) for _ in range(3)]
        ids = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(3)]
        st = (side if isinstance(side, torch.cuda.Stream) else torch.cuda.Stream()) if side else torch.cuda.current_stream()
        main = torch.cuda.current_stream()
        evs = []
        torch.cuda.synchronize()
        for t in range(56):
            s = t % 3 if rotate else 0
            nxt = ids[(s + 1) % 3] if rotate else None
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(st):
                a.record()
                e.decode(ids[s], kv, L + t, L + t + 1, logits=lg[s], next_ids=nxt, graph=graph)
                b.record()
            if waits and t > 0:
                main.wait_event(prev)  # the caller's stream waits for the previous step (a barrier packet)
            if extra:
                _ = torch.ne(ids[s], ids[(s + 2) % 3]).any()
                _ = lg[(s + 2) % 3].clone()
                _ = torch.argmax(lg[(s + 2) % 3], dim=-1)
            prev = b
            if t >= 8:
                evs.append((a, b))
            if side and t % 4 == 3 and not nowait:
                main.wait_stream(st)
        torch.cuda.synchronize()
        du = [a.elapsed_time(b) * 1e3 for a, b in evs]
        span = evs[0][0].elapsed_time(evs[-1][1]) * 1e3 / len(evs)
        print(f"{label}: step duration median {statistics.median(du):.1f} us (min {min(du):.1f}, max {max(du):.1f}); "
              f"wall per step {span:.1f} us")

    print("current stream", torch.cuda.current_stream(), "null?", torch.cuda.current_stream().cuda_stream)
    nb = hip_stream(1)
    for _ in range(2):
        run("A main, fixed buffers", False, False, False)
        run("Hf non-blocking side, fixed buffers", nb, False, False)
        run("Hn non-blocking side, the caller's stream never waits for it", nb, False, False, nowait=True)
        run("Hs torch side stream, the caller's stream never waits for it", True, False, False, nowait=True)
        run("H2n non-blocking side, caller's small ops, no waits", nb, True, True, nowait=True)
    for _ in range(0):
        run("A main, fixed buffers", False, False, False)
        run("B side, fixed buffers", True, False, False)
        run("C main, rotating slots", False, True, False)
        run("D side, rotating slots + caller ops", True, True, True)
    return
    run("E main, eager (no graph)", False, False, False, graph=False)
    run("F side, eager (no graph)", True, False, False, graph=False)
    run("G torch stream priority -1", torch.cuda.Stream(priority=-1), False, False)
    run("H hipStreamNonBlocking", hip_stream(1), False, False)
    run("I hipStreamDefault flags", hip_stream(0), False, False)
    run("J hip priority stream -1", hip_stream(0, -1), False, False)
    s2 = torch.cuda.Stream()
    with torch.cuda.stream(s2):
        run("K a torch stream made current (as main)", False, False, False)


if __name__ == "__main__":
    main()
