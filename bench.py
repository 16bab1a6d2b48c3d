#!/usr/bin/env python
"""bench.py -- PaliGemma-3B on MI355X through libpgmi: KV-cached decode tokens/s (+ prefill ms).

Workload (BASELINE.json configs[1]): PaliGemma-3B-PT-224 shapes, bf16, batch 1 per GPU, a
224x224 synthetic image + 32-token prompt (L = 288), greedy KV-cached decode.  A "step" is one
decode token for the whole batch (one pass of the hot path: 18 decoder layers + lm_head +
argmax), replayed as one hipGraph.  Inputs and weights are resident in HBM before the timed
region; weights are deterministic synthetic values of the 3B architecture (no checkpoint is
available offline).

    python bench.py [--gpus N --steps K --warmup W]

N > 1 (BASELINE.json configs[3]: images sharded 8 per GPU): one process per GPU.  Launched by
torchrun (WORLD_SIZE set) it runs as that rank; started directly with --gpus N > 1 it re-launches
itself under torch.distributed.run with N ranks (a child process started before any GPU call) and
exits with the child's status.  Each rank is an independent replica; the weights are generated on
rank 0 and RCCL-broadcast through libpgmi's C ABI (pgmi_broadcast_weights); --batch defaults to 8
images per GPU, and value = tokens of all ranks / the max-over-ranks timed region.

Prints ONE JSON line on rank 0 (contract in the task statement), with
  roofline      the dominant decode kernel (fused RMSNorm + gate/up GEMV + GeGLU), timed with
                HIP events on its own stream, algorithmic bytes per launch / average duration
  cpu_baseline  the decode step on this host's cores: a torch bf16 port (oracle/torch_cpu.py), with the
                numpy oracle (oracle/paligemma_np.py) and the survey container's reference figure beside it
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec (MI355X_MICROARCH.md)
REF_DECODE_TOKS = 10.17          # RTX 2060 fp16, KV cache, 256 tokens (summary_statistics.json:52-53)
DECODE_WEIGHT_BYTES = 5_017_325_568  # decoder + lm_head weights streamed per token
KV_BYTES_PER_TOKEN = 18_432      # 18 layers x (K + V) x 256 x 2 B read per cached token per step


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--batch", type=int, default=None,
                    help="images (sequences) per GPU (default 1 on one GPU -- configs[1]; 8 with N > 1 -- configs[3])")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--prefill-iters", type=int, default=20)
    ap.add_argument("--kernel-iters", type=int, default=90)
    ap.add_argument("--cpu-steps", type=int, default=12)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-448", action="store_true", help="skip the 448 px prefill measurement (configs[4])")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the configs[2] (no KV cache) and configs[3] (8 images per GPU) measurements")
    ap.add_argument("--nokv-tokens", type=int, default=16)
    ap.add_argument("--no-api", action="store_true",
                    help="skip the drop-in module API leg (inference.py's loop through PaliGemmaForConditionalGeneration)")
    ap.add_argument("--api-tokens", type=int, default=32)
    ap.add_argument("--dry-run", action="store_true",
                    help="rank logic only (world / batch / image shards / max-over-ranks timing / token gather) "
                         "over gloo with no GPU call: the CPU test of the N > 1 flow")
    return ap.parse_args()


def cpu_share() -> int:
    """CPUs this process may use: len(sched_getaffinity), capped by a cgroup v2 cpu.max quota."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_baseline(cfg, seed, L, steps, torch_steps=32):
    """The decode step on this host's cores, beside the GPU number (never the GPU's work):
      value  oracle/torch_cpu.py -- a builder-written torch bf16 restatement of the KV-cached decode step
             (full PaliGemma-3B text shapes, batch 1, cache of L tokens), `torch_steps` greedy steps;
      numpy_port  the numpy oracle (oracle/paligemma_np.py: fp32 math with the reference's bf16 rounding
             points) over a bounded `steps` sample;
      reference_cpu  the reference's own modules as timed in the survey container (they cannot travel)."""
    import numpy as np
    import threadpoolctl
    import torch

    from oracle import paligemma_np as O
    from oracle import weights as OW
    from oracle.torch_cpu import TorchCpuDecoder
    # torch port: the process's CPU share (nproc shows the whole machine): its affinity mask, capped by a
    # cgroup v2 cpu.max quota and by the box's 16-core share
    threads = min(16, cpu_share())
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    t0 = time.time()
    dec = TorchCpuDecoder(cfg, seed, max_kv=L + torch_steps + 8)
    tgen_s = time.time() - t0
    dec.fill_cache(L)
    tok = 108
    for s_ in range(2):  # warm (page in weights, oneDNN primitives)
        tok = int(dec.step(tok, L + 1 + s_).argmax())
    t0 = time.perf_counter()
    for s_ in range(torch_steps):
        tok = int(dec.step(tok, L + 3 + s_).argmax())
    torch_dt = time.perf_counter() - t0
    torch.set_num_threads(prev)
    del dec

    t0 = time.time()
    shapes = {n: s for n, s in OW.param_shapes(cfg).items() if n.startswith("language_model")}
    P = {n: OW.gen_f32(n, s, seed) for n, s in shapes.items()}
    gen_s = time.time() - t0
    t = cfg["text_config"]
    rng = np.random.default_rng(0)
    kv = O.KV()
    for i in range(t["num_hidden_layers"]):
        kv.update(O.bf16(rng.standard_normal((1, 1, L, 256)).astype(np.float32)),
                  O.bf16(rng.standard_normal((1, 1, L, 256)).astype(np.float32)), i)
    tok = np.array([108])
    O.paligemma_decode(P, cfg, tok, kv, L + 1)  # warm (page in weights)
    t0 = time.perf_counter()
    for s in range(steps):
        lg = O.paligemma_decode(P, cfg, tok, kv, L + 2 + s)
        tok = np.argmax(lg[:, -1], -1)
    dt = time.perf_counter() - t0
    np_threads = max([i.get("num_threads", 1) for i in threadpoolctl.threadpool_info()] or [1])
    return {"value": round(torch_steps / torch_dt, 3), "unit": "tokens/s", "cores": int(threads), "kind": "port",
            "sample": f"{torch_steps} KV-cached greedy decode steps of oracle/torch_cpu.py (torch {torch.__version__} "
                      f"CPU, bf16 weights and activations, the reference's rounding points) at full PaliGemma-3B "
                      f"text shapes, batch 1, cache {L} tokens, {threads} threads; weight generation ({tgen_s:.0f}s) "
                      f"untimed",
            "numpy_port": {"value": round(steps / dt, 4), "unit": "tokens/s", "cores": int(np_threads),
                           "sample": f"{steps} decode steps of oracle/paligemma_np.py (numpy fp32 math, bf16 rounding "
                                     f"points), same shapes and cache; weight generation ({gen_s:.0f}s) untimed"},
            "reference_cpu": {"value": 12.2, "unit": "tokens/s", "cores": 8, "dtype": "bf16",
                              "inference_py_semantics_tok_s": 5.2, "prefill_ms": 640,
                              "where": "the reference's own modules timed in the survey container (8 Xeon cores, "
                                       "torch 2.10 CPU), BASELINE.md sec.2; the reference cannot travel to the GPU box"}}


MFMA_BF16_PEAK_TFS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)


def time_prefill(eng, px, ids, pos, kv, iters):
    """Median wall time (HIP events on the current stream) of pixels + ids -> last-row logits ->
    argmax, with its vision / language-model split."""
    import torch

    def prefill():
        feats = eng.project(eng.vision(px))
        lg = eng.lm_forward(kv, 0, pos, ids=ids, image_feats=feats, logits_rows=2)
        return eng.argmax(lg[:, 0]), lg

    for _ in range(3):
        prefill()
    torch.cuda.synchronize()
    pre = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        prefill()
        e1.record()
        e1.synchronize()
        pre.append(e0.elapsed_time(e1))
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record()
    feats = eng.project(eng.vision(px))
    e1.record()
    lg = eng.lm_forward(kv, 0, pos, ids=ids, image_feats=feats, logits_rows=2)
    e2.record()
    e2.synchronize()
    return statistics.median(pre), e0.elapsed_time(e1), e1.elapsed_time(e2), lg


def time_preprocess(eng, dev, size, iters=20):
    """GPU process_images (pgmi_preprocess: PIL-exact BICUBIC resize + normalize) of one decoded
    480x640 RGB image already on the device -> float32 pixel_values, HIP events."""
    import torch
    from pgmi import _native as N
    src = torch.randint(0, 256, (480, 640, 3), dtype=torch.uint8, device=dev)
    out = torch.empty((3, size, size), dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream()

    def run():
        N.check(eng.lib.pgmi_preprocess(eng.ctx, src.data_ptr(), 480, 640, size, size, out.data_ptr(), s.cuda_stream))

    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        run()
    e1.record(s)
    e1.synchronize()
    return round(e0.elapsed_time(e1) / iters, 4)


def gemm_roofline(eng, rows, iters=36, reps=4):
    """The prefill's dominant MFMA GEMMs (gate|up + GeGLU, down) of all 18 layers over `rows`
    token rows.  `iters` launches cycling the layers (cold weights: 18 layers x 134 / 67 MB stream
    past the 256 MiB MALL) are captured into one graph and replayed `reps` times back to back;
    HIP events on the replay stream give the average launch, graph gaps included (an eager
    ctypes loop is host-bound for a ~20 us kernel: round 3 read 38 us for a 23 us kernel)."""
    import torch
    from pgmi import _native as N
    t = eng.cfgd
    H, I, nl = t["t_hidden"], t["t_intermediate"], t["t_layers"]
    out = {}
    for which, name, flops in ((0, "gate_up_geglu", 2.0 * rows * 2 * I * H), (1, "down", 2.0 * rows * H * I)):
        cur = torch.cuda.current_stream()
        for i in range(nl):  # eager warm-up (kernel attributes are set on first use, outside the capture)
            N.check(eng.lib.pgmi_prefill_kernel(eng.ctx, which, i, rows, cur.cuda_stream))
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            cs = torch.cuda.current_stream()
            for i in range(iters):
                N.check(eng.lib.pgmi_prefill_kernel(eng.ctx, which, i % nl, rows, cs.cuda_stream))
        g.replay()
        torch.cuda.synchronize()
        k0, k1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        k0.record()
        for _ in range(reps):
            g.replay()
        k1.record()
        k1.synchronize()
        us = k0.elapsed_time(k1) * 1e3 / (iters * reps)
        del g
        tfs = flops / (us * 1e-6) / 1e12
        out[name] = {"bound": "mfma", "rows": rows, "flop_per_launch": int(flops), "avg_launch_us": round(us, 2),
                     "achieved": round(tfs, 1), "peak": MFMA_BF16_PEAK_TFS, "unit": "TFLOP/s",
                     "frac": round(tfs / MFMA_BF16_PEAK_TFS, 4),
                     "timing": f"{iters} launches cycling the {nl} layers in one graph, replayed {reps}x, HIP events"}
    return out


def gemm_insitu(eng, px, ids, pos, kv, reps=3):
    """The same GEMMs timed in situ: pgmi_prefill_probe brackets every layer's gate|up and down GEMM
    with HIP events inside eager LM prefills (logits_rows 1: every layer runs its MLP GEMMs); the median
    over reps x 18 layers.  The events are the GEMM kernel's own (hipExtLaunchKernelGGL start / stop:
    the kernel's execution alone, as a kernel trace times it, not the stream's packets around it)."""
    import ctypes
    import torch
    from pgmi import _native as N
    nl = eng.cfgd["t_layers"]
    feats = eng.project(eng.vision(px))
    N.check(eng.lib.pgmi_prefill_probe(eng.ctx, 1))
    gu, dn = [], []
    try:
        for _ in range(reps + 1):
            eng.lm_forward(kv, 0, pos, ids=ids, image_feats=feats, logits_rows=1)
            torch.cuda.synchronize()
            us = (ctypes.c_float * (2 * nl))()
            N.check(eng.lib.pgmi_prefill_probe_times(eng.ctx, us, 2 * nl))
            gu.append(list(us[:nl]))
            dn.append(list(us[nl:]))
    finally:
        N.check(eng.lib.pgmi_prefill_probe(eng.ctx, 0))
    gu, dn = sum(gu[1:], []), sum(dn[1:], [])  # the first forward warms up
    return statistics.median(gu), statistics.median(dn)


def with_insitu(iso, gu_us, dn_us):
    """prefill_gemm_roofline entries: the in-situ timing as the headline (avg_launch_us, achieved, frac),
    the isolated back-to-back graph timing beside it."""
    out = {}
    for name, us in (("gate_up_geglu", gu_us), ("down", dn_us)):
        e = iso[name]
        tfs = e["flop_per_launch"] / (us * 1e-6) / 1e12
        out[name] = {"bound": "mfma", "rows": e["rows"], "flop_per_launch": e["flop_per_launch"],
                     "avg_launch_us": round(us, 2), "achieved": round(tfs, 1), "peak": MFMA_BF16_PEAK_TFS,
                     "unit": "TFLOP/s", "frac": round(tfs / MFMA_BF16_PEAK_TFS, 4),
                     "timing": "in situ: the GEMM kernel's own start/stop events (hipExtLaunchKernelGGL) in eager "
                               "LM prefills (pgmi_prefill_probe), median over the 18 layers x 3 forwards",
                     "isolated": {k: e[k] for k in ("avg_launch_us", "achieved", "frac", "timing")}}
    return out


def time_no_kv(eng, px, ids, tokens):
    """BASELINE configs[2]: KV cache disabled with ablation semantics
    (ablation_study_fixed.py:244-251): every token re-runs the vision tower (pixel_values are
    passed again) and a full non-causal forward over prompt + generated tokens, last-row
    logits, greedy pick.  Returns ms per token over `tokens` tokens."""
    import torch
    L = ids.shape[1]
    kv = eng.scratch_kv(1, L + tokens)

    def run():
        cur = ids
        for _ in range(tokens):
            feats = eng.project(eng.vision(px))
            lg = eng.lm_forward(kv, 0, torch.arange(cur.shape[1])[None], ids=cur, image_feats=feats, logits_rows=2)
            cur = torch.cat([cur, eng.argmax(lg[:, 0])[:, None]], 1)
        return cur
    run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / tokens


def time_sampling(eng, V, iters=20):
    """Device top-p draw (inference.py:64-66, T = 0.8, p = 0.9) over one row of V logits."""
    import torch
    g = torch.Generator(device=eng.device).manual_seed(0)
    lg = torch.randn((1, V), device=eng.device, generator=g) * 4
    u = torch.rand((iters + 3, 1), device=eng.device, generator=g)
    for i in range(3):
        eng.sample_top_p(lg, 0.9, 0.8, u=u[i])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(iters):
        eng.sample_top_p(lg, 0.9, 0.8, u=u[3 + i])
    e1.record()
    e1.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / iters, 2)


def decode_chunk(B, steps, warmup, graph=True):
    """Greedy steps per hipGraph launch for a B-row decode run (Engine.generate's form): GEN_CHUNK
    (pgmi_decode_steps) for the batched rows, where it measured faster (B = 8 step 1.279 -> 1.271 ms,
    tools/probes/multistep_probe.py, profiles/r06_multistep_probe.txt); one step per launch at B <= 2, where it
    measured slower (1.056 -> 1.060 ms).  Halved until it divides the timed steps and two chunks fit in the
    warmup (the first call with a buffer set runs eagerly, the second captures the graph)."""
    from pgmi import Engine
    c = Engine.GEN_CHUNK if (graph and B >= Engine.GEN_MIN_BATCH) else 1
    while c > 1 and (steps % c or warmup < 2 * c):
        c //= 2
    return c


def run_decode(eng, cur, kv, L, step0, n, chunk, logits, graph):
    """n greedy steps from KV row L + step0 (position one past it), the argmax fed back in place: chunks of
    `chunk` steps per pgmi_decode_steps call (one graph launch), single pgmi_decode calls otherwise."""
    t = 0
    while t < n:
        k = chunk if n - t >= chunk else 1
        s0 = step0 + t
        if k > 1:
            eng.decode_steps(cur, kv, L + s0, L + s0 + 1, k, logits=logits, graph=graph)
        else:
            eng.decode(cur, kv, L + s0, L + s0 + 1, logits=logits, next_ids=cur, graph=graph)
        t += k


def time_batch(cfg, dev, seed, g, B, steps, warmup):
    """BASELINE configs[3], per GPU: B images (8 of the 64) through a B-row prefill, then
    lock-step KV-cached greedy decode of B sequences (graph replay, device argmax)."""
    import torch
    from pgmi import Engine
    from pgmi.synthetic import init_policy, prompt_ids
    n_img = (cfg["vision_config"]["image_size"] // 14) ** 2
    L = n_img + 32
    cap = ((L + warmup + steps + 8) + 63) // 64 * 64
    e = Engine(cfg, device=dev, max_batch=B, max_seq=L, max_kv=cap)
    e.fill_synthetic(seed, init_policy)
    e.prepare()
    px = (torch.rand((B, 3, 224, 224), generator=g, device=dev) * 2 - 1).contiguous()
    ids = torch.from_numpy(prompt_ids(cfg["image_token_index"], n_img, cfg["text_config"]["vocab_size"])).to(dev)
    ids = ids.expand(B, -1).contiguous()
    kv = e.new_kv(B, cap)
    pm, _, _, lg = time_prefill(e, px, ids, torch.arange(L).expand(B, L), kv, 5)
    cur = e.argmax(lg[:, 0])
    logits = torch.empty((B, cfg["text_config"]["vocab_size"]), dtype=torch.float32, device=dev)
    chunk = decode_chunk(B, steps, warmup)
    run_decode(e, cur, kv, L, 0, warmup, chunk, logits, True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_decode(e, cur, kv, L, warmup, steps, chunk, logits, True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    del e
    torch.cuda.empty_cache()
    return {"images_per_gpu": B, "prefill_ms": round(pm, 3), "decode_tok_s": round(B * steps / dt, 1),
            "ms_per_step": round(dt * 1e3 / steps, 4), "steps": steps, "steps_per_graph_launch": chunk}


def time_b1_full_length(eng, first, L, n_tokens=256):
    """configs[1] at its stated length: 256 greedy KV-cached steps after the 288-token prefill (KV length
    289 .. 544), graph-replayed with the argmax fed back in place -- the same step as the headline `value`,
    whose K timed steps (the driver's --steps) sit at the start of that range.  A cache of its own (the
    headline's capacity is untouched); one short untimed pass captures the step's graph, then the timed pass
    restarts at KV row L."""
    import torch
    V = eng.cfgd["t_vocab"]
    kv = eng.new_kv(1, (L + n_tokens + 8 + 63) // 64 * 64)
    logits = torch.empty((1, V), dtype=torch.float32, device=eng.device)

    def run(n):
        cur = first.clone()
        for t in range(n):
            eng.decode(cur, kv, L + t, L + t + 1, logits=logits, next_ids=cur, graph=True)
        return cur

    run(4)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(n_tokens)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / n_tokens
    t_mean = L + 1 + (n_tokens - 1) / 2.0  # keys attended per step, averaged over the run
    step_bytes = DECODE_WEIGHT_BYTES + KV_BYTES_PER_TOKEN * t_mean
    del kv
    return {"tokens": n_tokens, "kv_len_range": [L + 1, L + n_tokens], "ms_per_step": round(ms, 4),
            "tok_s": round(1e3 / ms, 1),
            "decode_step_hbm": {"algorithmic_bytes_mean": int(step_bytes),
                                "achieved_GBs": round(step_bytes / (ms * 1e-3) / 1e9, 1),
                                "frac": round(step_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}}


def relaunch_multi(a) -> int:
    """--gpus N > 1 without a torchrun environment: N ranks under torch.distributed.run, as a child
    process started before anything touches the GPU (no exec from this process)."""
    import socket
    import subprocess
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def csrc_digest() -> str:
    """sha1 over the HIP sources of libpgmi (ties a committed PMC traffic file to the code it measured)."""
    import glob
    import hashlib
    h = hashlib.sha1()
    for f in sorted(glob.glob(os.path.join(PKG, "csrc", "*.hip")) + glob.glob(os.path.join(PKG, "csrc", "*.h"))):
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()


def pmc_traffic(kernel_key):
    """HBM bytes per launch of the dominant kernel from the FETCH_SIZE / WRITE_SIZE passes
    (tools/gpu_pmc.sh -> tools/pmc_traffic.py -> profiles/pmc_traffic.json).  Used only when the
    file was produced from the same csrc sources as this build; otherwise null."""
    tf = os.path.join(REPO, "profiles", "pmc_traffic.json")
    src = {"file": "profiles/pmc_traffic.json", "matches_build": False}
    if not os.path.exists(tf):
        return None, src
    try:
        d = json.load(open(tf))
        src.update(round=d.get("round"), csrc_sha1=d.get("csrc_sha1"))
        if d.get("csrc_sha1") != csrc_digest():
            return None, src
        src["matches_build"] = True
        return d[kernel_key]["hbm_bytes_per_launch"], src
    except Exception:
        return None, src


def time_api(cfg, dev, seed, tokens):
    """The drop-in module path exactly as inference.py:55-78 drives it: PaliGemmaForConditionalGeneration
    (synthetic 3B weights in its engine slab), prefill forward with the reference's (B, L, V)
    logits -- the default lazy form, and the eager all-row form -- then `tokens` decode steps through
    forward() with pixel_values re-passed, the attention mask grown by a float column, argmax of
    logits[:, -1, :] and next_token.item() per token (the reference's host sync)."""
    import torch
    import modeling_gemma as MG
    import utils as U
    from pgmi.synthetic import init_policy, prompt_ids
    pcfg = MG.PaliGemmaConfig(**{k: v for k, v in cfg.items() if k not in ("bos_token_id", "eos_token_id")})
    m = U.build_model(pcfg, device=dev)
    m.tie_weights()
    eng = m._pgmi_engine()
    eng.fill_synthetic(seed, init_policy)
    eng.prepare()
    n_img = (cfg["vision_config"]["image_size"] // 14) ** 2
    ids0 = torch.from_numpy(prompt_ids(cfg["image_token_index"], n_img, cfg["text_config"]["vocab_size"])).to(dev)
    g = torch.Generator(device=dev).manual_seed(7)
    px = (torch.rand((1, 3, 224, 224), generator=g, device=dev) * 2 - 1).contiguous()

    def prefill(mode):
        m.pgmi_prefill_logits = mode
        kv = MG.KVCache()
        out = m(input_ids=ids0, pixel_values=px, attention_mask=torch.ones_like(ids0), kv_cache=kv)
        return out, kv

    res = {}
    with torch.no_grad():
        for mode in ("lazy", "all"):
            for _ in range(3):
                prefill(mode)
            ts = []
            for _ in range(10):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                out, kv = prefill(mode)
                _ = torch.argmax(out["logits"][:, -1, :], dim=-1).item()
                ts.append((time.perf_counter() - t0) * 1e3)
            res[f"prefill_ms_{mode}_logits"] = round(statistics.median(ts), 3)
        m.pgmi_prefill_logits = "lazy"

        def decode_run():
            ids, mask = ids0, torch.ones_like(ids0)
            out, kv = prefill("lazy")
            n = 0
            t0 = None
            for step in range(tokens + 8):
                if step == 8:  # past the first steps' graph captures (the lookahead's three slots among them)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                nxt = torch.argmax(out["logits"][:, -1, :], dim=-1, keepdim=True).squeeze(0)
                _ = nxt.item()
                ids = nxt.unsqueeze(-1)
                mask = torch.cat([mask, torch.ones((1, 1), device=dev)], dim=-1)
                out = m(input_ids=ids, pixel_values=px, attention_mask=mask, kv_cache=kv)
                n += step >= 8
            torch.cuda.synchronize()
            return time.perf_counter() - t0, n

        # the step on demand (no lookahead, pgmi/lookahead.py) beside the default, alternating, best of 2
        m.pgmi_lookahead = False
        d0 = min(decode_run()[0] for _ in range(2))
        m.pgmi_lookahead = True
        dt, n = min(decode_run() for _ in range(2))
        res["decode_ms_per_token_no_lookahead"] = round(d0 * 1e3 / n, 4)
    res.update(decode_ms_per_token=round(dt * 1e3 / n, 4), decode_tok_s=round(n / dt, 1), tokens_timed=n,
               semantics="inference.py:55-78 through the drop-in module: pixel_values re-passed, float mask column "
                         "appended, argmax of logits[:, -1, :], .item() per token; the module's greedy lookahead "
                         "(pgmi/lookahead.py) runs each next step ahead of the caller")
    res["ablation_harness"] = time_ablation(m, ids0, px, tokens)
    del m, eng
    torch.cuda.empty_cache()
    return res


def time_ablation(m, ids0, px, tokens, warmup=32):
    """The paper's own benchmark loop (ablation_study_fixed.py:185-251, KV mode, temperature 0.0)
    through the drop-in model with load_model_simple's two patches installed (:335-342; restated in
    tests/tests_helpers.py): model.to(bf16), a discarded prefill, step 0 re-feeding the prompt +
    pixels into the filled cache, then one-token steps (pixel_values None, float mask column,
    argmax on the device, no .item()).  Timed like the harness's steady state: the tokens after
    WARMUP_TOKENS = 32 (:23,209-213,260-264)."""
    import torch
    import modeling_gemma as MG
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from tests_helpers import install_ablation_patches, remove_ablation_patches
    dev = ids0.device
    install_ablation_patches(m)
    try:
        with torch.no_grad():
            m = m.to(torch.bfloat16)
            kv = MG.KVCache()
            mask = torch.ones_like(ids0)
            pxb = px.to(torch.bfloat16)
            m(input_ids=ids0, pixel_values=pxb, attention_mask=mask, kv_cache=kv)
            ids, pixel = ids0, pxb
            gen = []
            t0 = None
            for step in range(warmup + tokens):
                if step == warmup:
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                out = m(input_ids=ids, pixel_values=pixel, attention_mask=mask, kv_cache=kv)
                nxt = torch.argmax(out["logits"][:, -1, :], dim=-1, keepdim=True).squeeze(0)
                gen.append(nxt)
                ids = nxt.unsqueeze(-1)
                mask = torch.cat([mask, torch.ones((1, 1), device=dev)], dim=-1)
                pixel = None
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
    finally:
        remove_ablation_patches(m)
    return {"steady_ms_per_token": round(dt * 1e3 / tokens, 4), "steady_tok_s": round(tokens / dt, 1),
            "tokens_timed": tokens, "warmup_tokens": warmup,
            "semantics": "ablation_study_fixed.py run_inference (KV mode) with its merge + rotary patches: "
                         "q_len == 1 steps on the graphed decode step over the patched merge's row "
                         "(pgmi_decode_embeds); steady state after 32 tokens as the harness reports it"}


def rank_plan(a, world, rank):
    """Images per rank and this rank's contiguous shard [lo, hi) of the job's images (configs[3]:
    64 images = 8 per GPU x 8; pgmi.dist.shard_range)."""
    from pgmi.dist import shard_range
    B = a.batch if a.batch is not None else (8 if world > 1 else 1)
    lo, hi = shard_range(B * world, rank, world)
    assert hi - lo == B
    return B, lo, hi


def max_over_ranks(elapsed, world, device):
    """The timed region of the slowest rank (all_reduce MAX; a CPU tensor over gloo)."""
    if world <= 1:
        return elapsed
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def run_dry(a, world, rank):
    """--dry-run: the N-rank flow of main() with the GPU work replaced by host stand-ins -- the same
    plan, barrier + timed region + max over ranks, gather of every image's tokens -- so the
    multi-rank logic runs in the CPU tests (gloo, world_size 2)."""
    import torch
    import torch.distributed as dist
    from pgmi.dist import gather_tokens
    B, lo, hi = rank_plan(a, world, rank)
    images = torch.arange(lo, hi, dtype=torch.int64)
    toks = torch.empty((B, a.steps), dtype=torch.int64)
    for _ in range(a.warmup):
        pass
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for step in range(a.steps):
        toks[:, step] = images * 100_000 + step   # stand-in for one lock-step decode of this rank's images
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    elapsed = max(max_over_ranks(elapsed, world, torch.device("cpu")), 1e-9)
    allt = gather_tokens(toks)
    if rank == 0:
        print(json.dumps({
            "metric": "decode tokens/sec per GPU + prefill ms (224px img + 32-tok prompt), PaliGemma-3B",
            "value": round(world * B * a.steps / elapsed, 3), "unit": "tokens/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed * 1e3 / a.steps, 6),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "dry run",
            "dry_run": True,
            "config": {"batch_per_gpu": B, "global_batch": B * world, "parallelism": f"replicas x{world}"},
            "gathered_images": [int(v) // 100_000 for v in allt[:, 0].tolist()],
            "gathered_steps_ok": bool(torch.equal(allt % 100_000, torch.arange(a.steps).expand(B * world, -1)))}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_multi(a))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and not (a.gpus == 1 and world == 1):
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    if a.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
        return run_dry(a, world, rank)
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", torch.cuda.current_device())

    from pgmi import Engine
    from pgmi.dist import broadcast_weights, gather_tokens
    from pgmi.synthetic import init_policy, paligemma_3b_config, prompt_ids

    cfg = paligemma_3b_config(a.image_size)
    n_img = (a.image_size // 14) ** 2
    L = n_img + 32
    B, img_lo, img_hi = rank_plan(a, world, rank)
    kv_cap = ((L + a.warmup + a.steps + 8) + 63) // 64 * 64
    # capacity: the headline's cache (kv_cap) and the 256-token configs[1] leg's own (time_b1_full_length)
    eng = Engine(cfg, device=dev, max_batch=B, max_seq=L + a.nokv_tokens, max_kv=max(kv_cap, (L + 264 + 63) // 64 * 64))
    slab_bytes = eng.slab.numel()

    # ---- weights: rank 0 generates, one RCCL broadcast of the packed slab over xGMI (C ABI)
    bcast_ms = None
    if rank == 0:
        eng.fill_synthetic(a.seed, init_policy)
    if world > 1:
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        comm = broadcast_weights(eng, src=0)
        torch.cuda.synchronize()
        bcast_ms = (time.perf_counter() - t0) * 1e3
        comm.close()
    eng.prepare()

    # ---- inputs (synthetic, resident in HBM): this rank's shard of the job's images (image i seeded
    # 1000 + i, whichever rank holds it), same prompt
    px = torch.empty((B, 3, a.image_size, a.image_size), device=dev)
    for j in range(B):
        gi = torch.Generator(device=dev).manual_seed(1000 + img_lo + j)
        px[j] = torch.rand((3, a.image_size, a.image_size), generator=gi, device=dev) * 2 - 1
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    ids = torch.from_numpy(prompt_ids(cfg["image_token_index"], n_img, cfg["text_config"]["vocab_size"])).to(dev)
    ids = ids.expand(B, -1).contiguous()
    pos = torch.arange(L).expand(B, L)
    kv = eng.new_kv(B, kv_cap)

    prefill_ms, vision_ms, lm_ms, lg = time_prefill(eng, px, ids, pos, kv, a.prefill_iters)
    prefill_gemms = with_insitu(gemm_roofline(eng, B * L), *gemm_insitu(eng, px, ids, pos, kv))
    pre_ms = time_preprocess(eng, dev, a.image_size)

    # ---- decode: warmup, then exactly K timed steps (graph replay, device-side argmax)
    first = eng.argmax(lg[:, 0])
    cur = first.clone()
    logits = torch.empty((B, cfg["text_config"]["vocab_size"]), dtype=torch.float32, device=dev)
    graph = not a.no_graph
    # greedy feedback in place (the step reads cur's tokens first and writes the next ones last); the
    # batched rows (B >= 3: configs[3], the multi-GPU runs) launch several steps per graph (decode_chunk)
    chunk = decode_chunk(B, a.steps, a.warmup, graph)
    run_decode(eng, cur, kv, L, 0, a.warmup, chunk, logits, graph)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    run_decode(eng, cur, kv, L, a.warmup, a.steps, chunk, logits, graph)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(elapsed, world, dev)
    # every image's last token on every rank (a few bytes per image; outside the timed region)
    gathered = gather_tokens(cur.reshape(B, 1))
    ms_per_step = elapsed * 1e3 / a.steps
    tok_s = world * B * a.steps / elapsed
    T_mid = L + a.warmup + a.steps // 2
    step_bytes = DECODE_WEIGHT_BYTES + B * KV_BYTES_PER_TOKEN * T_mid

    # ---- dominant kernel: fused RMSNorm + gate/up GEMV + GeGLU (kernel id 2), HIP events on
    # the stream it is launched on; cycling the 18 layers streams 2.4 GB (>> 256 MiB MALL)
    t = cfg["text_config"]
    H, I = t["hidden_size"], t["intermediate_size"]
    s = torch.cuda.current_stream()
    from pgmi import _native as N
    for i in range(18):
        N.check(eng.lib.pgmi_decode_kernel(eng.ctx, 2, i % 18, B, s.cuda_stream))
    k0, k1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    k0.record(s)
    for i in range(a.kernel_iters):
        N.check(eng.lib.pgmi_decode_kernel(eng.ctx, 2, i % 18, B, s.cuda_stream))
    k1.record(s)
    k1.synchronize()
    k_us = k0.elapsed_time(k1) * 1e3 / a.kernel_iters
    k_bytes = 2 * I * H * 2 + B * H * 2 + H * 2 + B * I * 2
    k_gbs = k_bytes / (k_us * 1e-6) / 1e9
    traffic, traffic_src = pmc_traffic("gateup") if B == 1 else (None, None)

    # ---- configs[1] at its stated length (256 output tokens, KV length up to 544), beside the K-step value
    full256 = None
    if world == 1 and not a.no_extra and B == 1:
        full256 = time_b1_full_length(eng, first, L)

    # ---- configs[2]: no KV cache (ablation semantics), top-p sampling cost, then configs[3]
    nokv = None
    sample_us = time_sampling(eng, cfg["text_config"]["vocab_size"])
    if world == 1 and not a.no_extra and B == 1:
        ms_tok = time_no_kv(eng, px[:1], ids[:1], a.nokv_tokens)
        nokv = {"tokens": a.nokv_tokens, "ms_per_token": round(ms_tok, 3), "tok_s": round(1e3 / ms_tok, 1),
                "semantics": "vision re-run + full forward over prompt + generated tokens per token"}
    del eng, kv
    torch.cuda.empty_cache()
    batch8 = None
    if world == 1 and not a.no_extra and B == 1:
        # configs[3] at its stated length: 256 output tokens per image (SURVEY sec.8d cfg 4)
        batch8 = time_batch(cfg, dev, a.seed, g, 8, 256, 16)
    api = None
    if world == 1 and not a.no_api and B == 1 and a.image_size == 224:
        api = time_api(cfg, dev, a.seed, a.api_tokens)

    # ---- configs[4]: 448 px prefill (1024 image tokens, L = 1056) on a second context
    p448 = None
    if world == 1 and not a.no_448 and a.image_size == 224:
        cfg4 = paligemma_3b_config(448)
        n4 = (448 // 14) ** 2
        L4 = n4 + 32
        e4 = Engine(cfg4, device=dev, max_batch=1, max_seq=L4, max_kv=L4 + 8)
        e4.fill_synthetic(a.seed, init_policy)
        e4.prepare()
        px4 = (torch.rand((1, 3, 448, 448), generator=g, device=dev) * 2 - 1).contiguous()
        ids4 = torch.from_numpy(prompt_ids(cfg4["image_token_index"], n4, cfg4["text_config"]["vocab_size"])).to(dev)
        kv4 = e4.new_kv(1, L4 + 8)
        pm, vm, lmm, _ = time_prefill(e4, px4, ids4, torch.arange(L4)[None], kv4, max(5, a.prefill_iters // 4))
        p448 = {"prefill_ms": round(pm, 3), "prefill_vision_ms": round(vm, 3), "prefill_lm_ms": round(lmm, 3),
                "prompt_len": L4,
                "gemm_roofline": with_insitu(gemm_roofline(e4, L4), *gemm_insitu(e4, px4, ids4, torch.arange(L4)[None],
                                                                                 kv4))}
        del e4

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import weights as OW
        cpu = cpu_baseline(OW.full_config(a.image_size), a.seed, L, a.cpu_steps)

    if rank == 0:
        if world > 1 or B > 1:
            workload = (f"configs[3]: paligemma-3b-pt-{a.image_size}, {B} synthetic images per GPU x {world} GPU(s) "
                        f"(global batch {B * world}), lock-step greedy KV-cached decode after a {n_img}-image-token "
                        f"+ 32-text-token prefill")
        else:
            workload = (f"configs[1]: paligemma-3b-pt-{a.image_size} greedy KV-cached decode, batch 1, after a "
                        f"{n_img}-image-token + 32-text-token prefill")
        out = {
            "metric": "decode tokens/sec per GPU + prefill ms (224px img + 32-tok prompt), PaliGemma-3B",
            "value": round(tok_s, 3),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "vs_baseline_note": "BASELINE.md publishes no number for this hardware/dtype; its only decode figure is "
                                "10.17 tok/s per GPU (RTX 2060, fp16, KV cache, 256 tokens)",
            "per_gpu_tok_s": round(tok_s / world, 3),
            # N > 1 runs configs[3] (8 images per GPU), N = 1 configs[1] (batch 1): the like-for-like single-GPU
            # figure for a scaling ratio of the N > 1 lines is the N = 1 line's config4_images_per_gpu leg
            "scaling_reference": ("config4_images_per_gpu.decode_tok_s of the N = 1 line (the same per-GPU work: "
                                  "8 images)" if world > 1 else None),
            "dtype": "bf16",
            "data": "synthetic (deterministic random-init PaliGemma-3B weights, seeded random 224x224 images, "
                    "synthetic 32-token prompt)",
            "config": {"workload": workload, "batch_per_gpu": B, "global_batch": B * world, "prompt_len": L,
                       "images_gathered": int(gathered.shape[0]),
                       "decode_tokens_timed": a.steps, "parallelism": f"replicas x{world} (weights RCCL-broadcast)",
                       "hipgraph": graph, "steps_per_graph_launch": chunk},
            "prefill_ms": round(prefill_ms, 3),
            "prefill_vision_ms": round(vision_ms, 3),
            "prefill_lm_ms": round(lm_ms, 3),
            "decode_step_hbm": {"algorithmic_bytes": step_bytes,
                                "achieved_GBs": round(step_bytes / (ms_per_step * 1e-3) / 1e9, 1),
                                "frac": round(step_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "roofline": {"kernel": f"k_gemv<{B},...,GV_GEGLU> (RMSNorm + gate/up GEMV + GeGLU)",
                         "bound": "hbm", "achieved": round(k_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(k_gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                         "bytes_per_launch": k_bytes, "avg_launch_us": round(k_us, 3)},
            "preprocess_ms": pre_ms,
            "preprocess_workload": f"one decoded 480x640 RGB image -> {a.image_size}x{a.image_size} pixel_values (GPU)",
            "config1_256": full256,
            "prefill_gemm_roofline": prefill_gemms,
            "prefill_448": p448,
            "config3_no_kv": nokv,
            "config4_images_per_gpu": batch8,
            "dropin_api": api,
            "sample_top_p_us": sample_us,
            "cpu_baseline": cpu,
        }
        if bcast_ms is not None:
            out["weight_broadcast_ms"] = round(bcast_ms, 2)
            out["weight_broadcast_bytes"] = slab_bytes
            out["weight_broadcast_GBs"] = round(slab_bytes / (bcast_ms * 1e-3) / 1e9, 1)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
