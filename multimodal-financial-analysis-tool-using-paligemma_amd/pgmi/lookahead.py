"""Greedy lookahead for the drop-in decode loop (host runtime of the MI355X path; no reference counterpart).

The reference's loop (inference.py:56-78) waits on every token: `next_token.item()` syncs the host, and
only then does it build the next input and call forward() again.  Everything the host does between that
sync and the next step's launch -- the loop's own ops, the forward call, the graph launch -- leaves the GPU
idle (≈90 µs per token at the 3B shapes: bench.py dropin_api against the native step).

GreedyLookahead runs the NEXT step before it is asked for, on a side stream: after the step the caller
asked for, it enqueues the step whose input is that step's on-device argmax (torch.argmax semantics,
written by the lm_head's last workgroup) into another logits buffer and the next KV row.  The caller's own
ops (its argmax, `.item()`) stay on its stream and do not wait for it, so the GPU runs the next step while
the host does its per-token work.  When the caller's next forward() brings that same token at the next
position of the same cache, its stream checks the token against the one the lookahead used, the following
lookahead is enqueued, the host waits for the check and the lookahead, and the caller's stream copies the
lookahead's logits out -- the caller's stream never waits on the side stream (a pending cross-queue wait
slows the other queue's graphed step by ~0.09 ms: tools/probes/stream_probe.py, profiles/
r05_stream_probe.txt), and nothing runs between two lookaheads on the side stream.
Any other input (a sampled token, another position, another cache) runs the asked step on the caller's
stream behind the lookahead, whose KV row lies past the cache's length and is overwritten.  A lookahead that is not
asked for (the check fails, or the next call brings another cache or position) is a miss of its cache; after two
misses in a row the lookahead stands down for that cache (a sampling loop, inference.py:64-66, or a loop that
interleaves sequences would otherwise pay a wasted step per token).

Ordering: the lookahead uses the engine's workspace and the cache's slab, so (1) the side stream waits for
the caller's stream before a lookahead that follows a step (or any engine call) on the caller's stream --
after a hit it follows its own previous step and waits for nothing else, so the caller's check and per-token
ops stay off the chain of steps, (2) every later engine call on any other stream waits for the last
lookahead (Engine._s() runs the guard installed here), and (3) the slab is marked as used by the side
stream for the caching allocator.  Three ids / logits slots rotate, so the token check of one step never
races the write of the step after it.  What the caller gets is bit-identical to the step run on demand:
the same graphed step over the same inputs.
"""
from __future__ import annotations

import weakref

import torch

NSLOT = 3


class GreedyLookahead:
    """Held by its engine (Engine._lookahead, and Engine._stream_guard as a bound method); it refers back to
    the engine weakly, so dropping the engine frees its context and memory at once, not at the next cyclic
    garbage collection (Engine.__del__ first waits for the last lookahead step)."""

    def __init__(self, eng, B: int):
        self._eng, self.B = weakref.ref(eng), B
        V = eng.cfgd["t_vocab"]
        dev = eng.device
        # slot s: ids[s] is the input token of the step whose logits go to logits[s]; that step's argmax goes
        # to ids[(s + 1) % NSLOT], the input of the step after it
        self.logits = [torch.empty((B, V), dtype=torch.float32, device=dev) for _ in range(NSLOT)]
        self.ids = [torch.zeros(B, dtype=torch.int64, device=dev) for _ in range(NSLOT)]
        self.side = torch.cuda.Stream(device=dev)
        self.flag = torch.zeros((), dtype=torch.bool).pin_memory()
        self.ev_chk = torch.cuda.Event()
        self.pending = None    # (weakref to the KVCache, kv_len, position, slot, event on the side stream)
        self.last = None       # event of the last lookahead enqueued (what other streams must wait for)
        self.hits = 0
        self.main_touched = False  # an engine call ran on another stream since the last lookahead
        eng._stream_guard = self._guard

    @property
    def eng(self):
        e = self._eng()
        if e is None:
            raise RuntimeError("the engine of this greedy lookahead has been released")
        return e

    def _guard(self, handle) -> None:
        """Engine._s(): an engine call about to run on stream `handle` waits for the last lookahead (and the
        next lookahead will wait for it: it shares the engine's workspace)."""
        if handle != self.side.cuda_stream:
            self.main_touched = True
            if self.last is not None:
                torch.cuda.current_stream(self.eng.device).wait_event(self.last)

    def _run(self, slab, kv_len, position, s, graph):
        self.eng.decode(self.ids[s], slab, kv_len, position, logits=self.logits[s],
                        next_ids=self.ids[(s + 1) % NSLOT], graph=graph)

    def _ahead(self, kv_cache, slab, kv_len, position, s, graph, after_main: bool):
        """Enqueue on the side stream the step in slot s (its input ids[s]: the previous step's argmax).
        after_main: the previous step ran on the caller's stream, so the side stream waits for it; after a
        hit (and no engine call on another stream since the last lookahead) the previous step is the side
        stream's own last one and nothing on the caller's stream is waited for -- the caller's check, clone
        and own ops stay off the chain of steps (slots read on the caller's stream are rewritten three steps
        later, behind the host's wait for that step's check)."""
        if kv_len + 1 > slab.shape[3] or getattr(kv_cache, "_pgmi_misses", 0) >= 2:
            self.pending = None
            return
        if after_main or self.main_touched:
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream(self.eng.device))
            self.side.wait_event(ready)
        self.main_touched = False
        with torch.cuda.stream(self.side):
            self._run(slab, kv_len, position, s, graph)
            ev = torch.cuda.Event()
            ev.record(self.side)
        slab.record_stream(self.side)
        self.last = ev
        self.pending = (weakref.ref(kv_cache), kv_len, position, s, ev)

    def _take(self, kv_cache, slab, cache_len, position, s, done, ne, graph, after_launch):
        """The hit path's tail: ne (a device bool, on the caller's stream) says whether the asked step differs
        from the lookahead in slot s (done: its event on the side stream).  Hands back the lookahead's logits
        (None on a miss)."""
        main = torch.cuda.current_stream(self.eng.device)
        self.flag.copy_(ne, non_blocking=True)
        self.ev_chk.record(main)
        if after_launch is not None:
            after_launch()
        # the next lookahead goes in before the host waits: the side stream never runs dry
        self._ahead(kv_cache, slab, cache_len + 1, position + 1, (s + 1) % NSLOT, graph, False)
        # the host waits for the check and for the lookahead itself; the caller's stream then copies its
        # logits out with no GPU-side wait on the side stream (a pending cross-queue wait slows the other
        # queue's steps by ~9 %: tools/probes/stream_probe.py), and nothing sits between two lookaheads
        self.ev_chk.synchronize()
        done.synchronize()
        if not bool(self.flag):
            kv_cache._pgmi_misses = 0
            self.hits += 1
            return self.logits[s].clone().unsqueeze(1)
        # a miss (sampling, a forced token): the asked step runs on the caller's stream behind the
        # lookahead just enqueued, over the same KV rows
        kv_cache._pgmi_misses = getattr(kv_cache, "_pgmi_misses", 0) + 1
        self.pending = None
        return None

    @staticmethod
    def _wasted(p) -> None:
        """The pending lookahead p was not asked for (another cache, position or batch came next): a miss of
        its cache, so a loop that interleaves sequences stops paying a wasted step per token."""
        c = p[0]()
        if c is not None:
            c._pgmi_misses = getattr(c, "_pgmi_misses", 0) + 1

    def step(self, kv_cache, slab, input_ids, cache_len: int, position: int, graph: bool, after_launch=None):
        """The logits (B, 1, V) of the decode step for input_ids at KV row cache_len / rotary `position`
        (a fresh tensor, as the reference returns); `after_launch` runs once the asked step is enqueued."""
        main = torch.cuda.current_stream(self.eng.device)
        ids = input_ids.reshape(-1).to(self.eng.device, torch.int64)
        p = self.pending
        self.pending = None
        s = 0
        if p is not None and not (p[0]() is kv_cache and p[1] == cache_len and p[2] == position
                                  and ids.numel() == self.B):
            self._wasted(p)
            p = None
        if p is not None:
            s = p[3]
            # the check on the caller's stream: the lookahead's input ids[s] was written by the step before
            # it, which the host has already waited for, so nothing here waits for the side stream
            out = self._take(kv_cache, slab, cache_len, position, s, p[4], torch.ne(ids, self.ids[s]).any(), graph,
                             after_launch)
            if out is not None:
                return out
            s = (s + 2) % NSLOT
        # the asked step on the caller's stream, behind any lookahead still in flight (it shares the slots,
        # the engine's workspace and possibly this cache's rows)
        if self.last is not None:
            main.wait_event(self.last)
        self.ids[s].copy_(ids)
        self._run(slab, cache_len, position, s, graph)
        out = self.logits[s].clone().unsqueeze(1)
        if after_launch is not None:
            after_launch()
        self._ahead(kv_cache, slab, cache_len + 1, position + 1, (s + 1) % NSLOT, graph, True)
        return out

    def step_embeds(self, kv_cache, slab, input_ids, embeds, row, position, mask, cache_len: int, graph: bool):
        """The ablation harness's q_len == 1 step (ablation_study_fixed.py:215-221,239-243: its patched merge,
        then pgmi_decode_embeds_dev over the merged row, the merge's device position and additive mask).
        embeds: this call's own lookup of input_ids (Engine.embed); row: the merge's output row.  The
        lookahead (the ids step at the predicted next position, no mask) stands for the asked step when the
        token is the lookahead's, the merge passed its embedding through unchanged, the position is the
        predicted one and the mask is all zeros -- the same arithmetic (a zero additive mask leaves every
        bf16 score as it is), checked on the device.  Otherwise the asked step runs on the caller's stream."""
        main = torch.cuda.current_stream(self.eng.device)
        ids = input_ids.reshape(-1).to(self.eng.device, torch.int64)
        p = self.pending
        self.pending = None
        s = 0
        if p is not None and not (p[0]() is kv_cache and p[1] == cache_len and ids.numel() == 1 == self.B):
            self._wasted(p)
            p = None
        if p is not None:
            s = p[3]
            ne = torch.ne(ids, self.ids[s]).any()
            ne = ne | torch.ne(row.reshape(-1), embeds.reshape(-1)).any()
            ne = ne | torch.ne(torch.round(position.reshape(-1)[:1].to(torch.float64)), float(p[2])).any()
            if mask is not None:
                ne = ne | torch.ne(mask, 0).any()
            out = self._take(kv_cache, slab, cache_len, p[2], s, p[4], ne, graph, None)
            if out is not None:
                return out
            s = (s + 2) % NSLOT
        # the asked step on the caller's stream; the next lookahead's position is the merge's position + 1,
        # read on the host before the step is enqueued (the read waits for the merge's own ops only)
        pos = int(round(float(position.reshape(-1)[0].item())))
        if self.last is not None:
            main.wait_event(self.last)
        lg = self.eng.decode_embeds_dev(row, slab, cache_len, position, mask, logits=self.logits[s],
                                        next_ids=self.ids[(s + 1) % NSLOT], graph=graph)
        out = lg.clone().unsqueeze(1)
        self._ahead(kv_cache, slab, cache_len + 1, pos + 1, (s + 1) % NSLOT, graph, True)
        return out


def lookahead_for(eng, B: int) -> GreedyLookahead:
    la = getattr(eng, "_lookahead", None)
    if la is None or la.B != B:
        if la is not None and la.last is not None:
            # the replaced lookahead's last step may still run on its side stream, in the engine's workspace:
            # whatever the new one enqueues waits for it (its guard is replaced below)
            torch.cuda.current_stream(eng.device).wait_event(la.last)
        la = eng._lookahead = GreedyLookahead(eng, B)
        la.main_touched = True  # the first lookahead of the new object waits for the caller's stream
    return la
