"""Probe: do the prefill GEMMs depend on the operands' row pitch?  Every shape runs its default plan
(pgmi_op_gemm_strided) with A and W stored at row strides K + pad elements, pad in {0, 8, 64}, the
weights rotated over copies larger than the Infinity Cache (each call reads them from HBM, as a layer
loop does); the calls are replayed from a captured graph, variants interleaved over rounds.  The outputs
must be bit-identical across pitches (same tiles, same order).

    python tools/probes/stride_probe.py [shape ...] [--rounds 3] [--iters 20]
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"))
sys.path.insert(0, REPO)
from oracle import weights as W  # noqa: E402
from pgmi import Engine, _native as N  # noqa: E402

SHAPES = {  # name: (M, N, K, epi)
    "t_gateup": (288, 16384, 2048, 7), "t_down": (288, 2048, 16384, 4), "t_qkv": (288, 2560, 2048, 0),
    "t_o": (288, 2048, 2048, 4), "v_qkv": (256, 3456, 1152, 1), "v_out": (256, 1152, 1152, 3),
    "v_fc1": (256, 4304, 1152, 2), "v_fc2": (256, 1152, 4304, 3), "t448_gateup": (1056, 16384, 2048, 7),
}
PADS = [(0, 0), (64, 0), (0, 64), (64, 64), (8, 8)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shapes", nargs="*")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    e = Engine(W.small_config(1, 1, 1024), max_batch=1, max_seq=320, max_kv=512)
    e.fill_synthetic(1, W.init_policy)
    e.prepare()
    lib = e.lib
    torch.manual_seed(0)
    for name in (a.shapes or SHAPES):
        M, Nn, K, epi = SHAPES[name]
        rows_w = Nn * (2 if epi == 7 else 1)
        A0 = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        W0 = ((torch.rand(rows_w, K, device="cuda") * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        bias = torch.randn(Nn, device="cuda").to(torch.bfloat16)
        res = torch.randn(M, Nn, device="cuda").to(torch.bfloat16)
        flops = 2.0 * M * Nn * K * (2 if epi == 7 else 1)
        variants = []
        for pa, pw in PADS:
            A = torch.zeros(M, K + pa, device="cuda", dtype=torch.bfloat16)
            A[:, :K] = A0
            nw = max(1, -(-(320 << 20) // (rows_w * (K + pw) * 2)))
            Ws = []
            for _ in range(nw):
                Wp = torch.zeros(rows_w, K + pw, device="cuda", dtype=torch.bfloat16)
                Wp[:, :K] = W0
                Ws.append(Wp)
            out = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16)
            variants.append(dict(pa=pa, pw=pw, A=A, Ws=Ws, out=out, nw=nw))

        def call(v, w, st):
            N.check(lib.pgmi_op_gemm_strided(e.ctx, v["A"].data_ptr(), v["A"].shape[1], w.data_ptr(), w.shape[1], M,
                                             Nn, K, epi, bias.data_ptr(), res.data_ptr(), v["out"].data_ptr(), st))

        for v in variants:
            call(v, v["Ws"][0], torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        same = all(torch.equal(v["out"], variants[0]["out"]) for v in variants)
        for v in variants:
            for _ in range(2):
                call(v, v["Ws"][0], torch.cuda.current_stream().cuda_stream)
            g = torch.cuda.CUDAGraph()
            n = max(a.iters, v["nw"])
            with torch.cuda.graph(g):
                cs = torch.cuda.current_stream().cuda_stream
                for i in range(n):
                    call(v, v["Ws"][i % v["nw"]], cs)
            v["g"], v["n"] = g, n
        times = {(v["pa"], v["pw"]): [] for v in variants}
        for _ in range(a.rounds):
            for v in variants:
                v["g"].replay()
                torch.cuda.synchronize()
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0.record()
                v["g"].replay()
                t1.record()
                t1.synchronize()
                times[(v["pa"], v["pw"])].append(t0.elapsed_time(t1) * 1e3 / v["n"])
        print(f"{name} M={M} N={Nn} K={K} (outputs identical across pitches: {same}): " + ", ".join(
            f"pad A {pa} W {pw}: {min(ts):.1f} us ({flops / min(ts) / 1e6:.0f} TF)" for (pa, pw), ts in times.items()),
            flush=True)
        del variants
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
