"""Sweep prefill GEMM plans (tile config x split-K) on the PaliGemma prefill shapes; prints
us per call, TFLOP/s and the max deviation from the reference plan (cfg 4/5 register-staged
GEMM, checked by tests/test_gpu_ops.py).  Usage (GPU box):
    python tools/gemm_sweep.py [shape-name ...] [--cfgs 6,7,9] [--splits 1,2,4,8]"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"))
sys.path.insert(0, REPO)
from oracle import weights as W  # noqa: E402
from pgmi import Engine, _native as N  # noqa: E402

SHAPES = {  # name: (M, N, K, epi)
    "t_qkv": (288, 2560, 2048, 0), "t_o": (288, 2048, 2048, 4), "t_gateup": (288, 16384, 2048, 7),
    "t_down": (288, 2048, 16384, 4), "v_qkv": (256, 3456, 1152, 1), "v_out": (256, 1152, 1152, 3),
    "v_fc1": (256, 4304, 1152, 2), "v_fc2": (256, 1152, 4304, 3), "v_patch": (256, 1152, 640, 1),
    "v_proj": (256, 2048, 1152, 1),
    "t448_qkv": (1056, 2560, 2048, 0), "t448_o": (1056, 2048, 2048, 4), "t448_gateup": (1056, 16384, 2048, 7),
    "t448_down": (1056, 2048, 16384, 4), "v448_fc1": (1024, 4304, 1152, 2), "v448_qkv": (1024, 3456, 1152, 1),
    "v448_out": (1024, 1152, 1152, 3), "v448_fc2": (1024, 1152, 4304, 3),
    # diagnostics: fc1 without the GELU (bias only), and with N padded to a multiple of 128
    "v448_fc1_bias": (1024, 4304, 1152, 1), "v448_fc1_n4352": (1024, 4352, 1152, 2),
    # configs[3] prefill: 8 images per GPU as one batch (vision 8 x 256 rows, text 8 x 288 rows)
    "b8_v_qkv": (2048, 3456, 1152, 1), "b8_v_out": (2048, 1152, 1152, 3), "b8_v_fc1": (2048, 4304, 1152, 2),
    "b8_v_fc2": (2048, 1152, 4304, 3), "b8_v_proj": (2048, 2048, 1152, 1), "b8_t_qkv": (2304, 2560, 2048, 0),
    "b8_t_o": (2304, 2048, 2048, 4), "b8_t_gateup": (2304, 16384, 2048, 7), "b8_t_down": (2304, 2048, 16384, 4),
    # batched decode (configs[3]: 8 lock-step sequences) as GEMMs with 8 rows
    "b8_gateup": (8, 16384, 2048, 7), "b8_down": (8, 2048, 16384, 4), "b8_o": (8, 2048, 2048, 4),
    "b8_qkv": (8, 2560, 2048, 0),
    # calibration against cdna_hip_programming.md's 256^2 8-phase template figures (square, plain store)
    "sq4096": (4096, 4096, 4096, 0), "sq8192": (8192, 8192, 8192, 0),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shapes", nargs="*")
    ap.add_argument("--cfgs", default="0,2,4,5,6,7,8,9,10,11")
    ap.add_argument("--splits", default="1,2,4,8")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--all", action="store_true", help="print every (cfg, split) row, not the best five")
    ap.add_argument("--cold", action="store_true",
                    help="rotate over distinct weight copies (> 256 MiB in all) so every call reads its weights "
                         "from HBM, as the layer loop of a forward does")
    args = ap.parse_args()
    e = Engine(W.small_config(1, 1, 1024), max_batch=1, max_seq=320, max_kv=512)
    e.fill_synthetic(1, W.init_policy)
    e.prepare()
    lib = e.lib
    s = torch.cuda.current_stream().cuda_stream
    cfgs = [int(c) for c in args.cfgs.split(",")]
    splits = [int(c) for c in args.splits.split(",")]
    torch.manual_seed(0)
    for name in (args.shapes or SHAPES):
        M, Nn, K, epi = SHAPES[name]
        A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        Wt = ((torch.rand(Nn * (2 if epi == 7 else 1), K, device="cuda") * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        nw = max(1, -(-(320 << 20) // (Wt.numel() * 2))) if args.cold else 1
        Ws = [Wt] + [Wt.clone() for _ in range(nw - 1)]
        wi = [0]
        bias = torch.randn(Nn, device="cuda").to(torch.bfloat16)
        res = torch.randn(M, Nn, device="cuda").to(torch.bfloat16)
        out = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16)
        flops = 2.0 * M * Nn * K * (2 if epi == 7 else 1)

        def run(st=None):
            w = Ws[wi[0] % nw]
            wi[0] += 1
            N.check(lib.pgmi_op_gemm(e.ctx, A.data_ptr(), w.data_ptr(), M, Nn, K, epi, bias.data_ptr(),
                                     res.data_ptr(), out.data_ptr(), st or s))

        N.check(lib.pgmi_tune_gemm(4 if M > 288 else 5, 1))
        run()
        ref = out.float().clone()
        rows = []
        for cfg in [-1] + cfgs:
            for split in ([0] if cfg < 0 else splits):
                if epi == 7 and split > 1:
                    continue
                N.check(lib.pgmi_tune_gemm(cfg, split))
                out.zero_()
                run()
                torch.cuda.synchronize()
                err = float((out.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-6))
                for _ in range(3):
                    run()
                torch.cuda.synchronize()
                # GPU time only: the calls are replayed from a captured graph (host launch cost,
                # ~10 us through ctypes, would otherwise floor every small GEMM)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    cs = torch.cuda.current_stream().cuda_stream
                    for _ in range(max(args.iters, nw)):
                        run(cs)
                g.replay()
                torch.cuda.synchronize()
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0.record()
                g.replay()
                t1.record()
                t1.synchronize()
                us = t0.elapsed_time(t1) * 1e3 / max(args.iters, nw)
                del g
                rows.append((us, cfg, split, err))
        N.check(lib.pgmi_tune_gemm(-1, 0))
        auto = rows[0]
        best = sorted(rows[1:])[:5]
        print(f"{name:12s} M={M} N={Nn} K={K}: auto {auto[0]:7.1f} us ({flops / auto[0] / 1e6:6.0f} TF) | " +
              ", ".join(f"c{c}/s{sp}: {t:6.1f} ({flops / t / 1e6:4.0f} TF, err {er:.1e})" for t, c, sp, er in best),
              flush=True)
        if args.all:
            for t, c, sp, er in sorted(rows[1:]):
                print(f"   {name} c{c}/s{sp}: {t:7.1f} us ({flops / t / 1e6:5.0f} TF, err {er:.1e})", flush=True)
        bad = [(c, sp, er) for _, c, sp, er in rows if er > 2e-2]
        if bad:
            print(f"   MISMATCH {name}: {bad}", flush=True)


if __name__ == "__main__":
    main()
