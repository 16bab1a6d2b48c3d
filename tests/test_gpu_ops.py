"""Kernel-level parity: each libpgmi op (through the C ABI) vs the CPU restatement in
oracle/paligemma_np.py on the same seeded inputs.

Tolerances: elementwise ops within 2 bf16 ulp; GEMM / attention rel-L2
<= 1e-2 (in practice ~1e-3: both sides accumulate in fp32, only the order differs)."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import paligemma_np as O
from oracle import weights as W

pytestmark = pytest.mark.gpu


def bf(x_np):
    """numpy float32 (bf16-valued) -> cuda bf16 tensor."""
    return torch.from_numpy(O.bf16(x_np)).to(torch.bfloat16).cuda()


def np32(t):
    return t.detach().float().cpu().numpy()


def rand(rng, *shape, scale=1.0):
    return O.bf16(rng.standard_normal(shape).astype(np.float32) * np.float32(scale))


def rel_l2(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def ulp_frac(a, b, ulps=1):
    """fraction of elements within `ulps` bf16 ulps of each other"""
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    sp = np.abs(b) * np.float32(2.0 ** -7) + np.float32(1e-30)
    return float((np.abs(a - b) <= ulps * sp).mean())


@pytest.fixture(scope="module")
def eng():
    from pgmi import Engine
    cfg = W.small_config(vision_layers=1, text_layers=1, vocab=1024)
    e = Engine(cfg, max_batch=2, max_seq=320, max_kv=1024)
    e.fill_synthetic(1234, W.init_policy)
    e.prepare()
    return e


def _gemm(eng, A, Wt, epi, bias=None, res=None, out_f32=False, geglu=False):
    M, K = A.shape
    N = Wt.shape[0] // (2 if geglu else 1)
    out = torch.empty((M, N), dtype=torch.float32 if out_f32 else torch.bfloat16, device="cuda")
    from pgmi import _native as NN
    NN.check(eng.lib.pgmi_op_gemm(eng.ctx, A.data_ptr(), Wt.data_ptr(), M, N, K, epi,
                                  NN.ptr(bias), NN.ptr(res), out.data_ptr(), NN.stream_handle()))
    torch.cuda.synchronize()
    return np32(out)


@pytest.mark.parametrize("M,N,K", [(288, 2560, 2048), (256, 4304, 1152), (256, 1152, 4304), (288, 2048, 16384),
                                   (37, 200, 64), (1, 128, 2048), (256, 1152, 640)])
def test_gemm_store(eng, M, N, K):
    rng = np.random.default_rng(M * 7 + N + K)
    A, Wt = rand(rng, M, K), rand(rng, N, K, scale=1 / np.sqrt(K))
    got = _gemm(eng, bf(A), bf(Wt), 0)
    ref = O.bf16(A @ Wt.T)
    assert rel_l2(got, ref) < 2e-3
    assert ulp_frac(got, ref, 1) > 0.99


@pytest.mark.parametrize("epi", ["bias", "bias_gelu", "bias_res", "res", "f32"])
def test_gemm_epilogues(eng, epi):
    from pgmi._native import EPI
    rng = np.random.default_rng(5)
    M, N, K = 256, 1152, 1152
    A, Wt = rand(rng, M, K), rand(rng, N, K, scale=1 / np.sqrt(K))
    b, r = rand(rng, N, scale=0.1), rand(rng, M, N)
    acc = A @ Wt.T
    if epi == "bias":
        ref = O.bf16(acc + b)
    elif epi == "bias_gelu":
        ref = O.gelu_tanh(O.bf16(acc + b))
    elif epi == "bias_res":
        ref = O.bf16(O.bf16(acc + b) + r)
    elif epi == "res":
        ref = O.bf16(O.bf16(acc) + r)
    else:
        ref = O.bf16(acc)
    got = _gemm(eng, bf(A), bf(Wt), EPI[epi], bias=bf(b), res=bf(r), out_f32=(epi == "f32"))
    assert rel_l2(got, ref) < 3e-3
    assert ulp_frac(got, ref, 1) > 0.98


def test_gemm_geglu(eng):
    rng = np.random.default_rng(9)
    M, N, K = 288, 512, 2048
    A = rand(rng, M, K)
    Wg, Wu = rand(rng, N, K, scale=2 / np.sqrt(K)), rand(rng, N, K, scale=2 / np.sqrt(K))
    got = _gemm(eng, bf(A), bf(np.concatenate([Wg, Wu])), 7, geglu=True)
    ref = O.bf16(O.gelu_tanh(O.bf16(A @ Wg.T)) * O.bf16(A @ Wu.T))
    assert rel_l2(got, ref) < 5e-3


@pytest.mark.parametrize("M,N,K,epi,pa,pw", [(288, 2560, 2048, 0, 64, 0), (256, 1152, 1152, 3, 8, 64),
                                              (288, 512, 2048, 7, 64, 64), (288, 2048, 16384, 4, 0, 8)])
def test_gemm_strided_matches_contiguous(eng, M, N, K, epi, pa, pw):
    """pgmi_op_gemm_strided (the row-pitch probe's entry): A and W at row strides K + pa / K + pw give the
    contiguous call's output bit for bit (same plan, same tiles, same order), and the pad columns are never
    read (they hold NaN here)."""
    from pgmi import _native as NN
    rng = np.random.default_rng(M + N + K + epi)
    rows_w = N * (2 if epi == 7 else 1)
    A, Wt = bf(rand(rng, M, K)), bf(rand(rng, rows_w, K, scale=1 / np.sqrt(K)))
    b, r = bf(rand(rng, N, scale=0.1)), bf(rand(rng, M, N))
    Ap = torch.full((M, K + pa), float("nan"), dtype=torch.bfloat16, device="cuda")
    Ap[:, :K] = A
    Wp = torch.full((rows_w, K + pw), float("nan"), dtype=torch.bfloat16, device="cuda")
    Wp[:, :K] = Wt
    out0 = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
    out1 = torch.empty_like(out0)
    s = NN.stream_handle()
    NN.check(eng.lib.pgmi_op_gemm(eng.ctx, A.data_ptr(), Wt.data_ptr(), M, N, K, epi, b.data_ptr(), r.data_ptr(),
                                  out0.data_ptr(), s))
    NN.check(eng.lib.pgmi_op_gemm_strided(eng.ctx, Ap.data_ptr(), K + pa, Wp.data_ptr(), K + pw, M, N, K, epi,
                                          b.data_ptr(), r.data_ptr(), out1.data_ptr(), s))
    torch.cuda.synchronize()
    assert torch.equal(out0, out1)
    with pytest.raises(ValueError):  # a pitch below K
        NN.check(eng.lib.pgmi_op_gemm_strided(eng.ctx, Ap.data_ptr(), K - 8, Wp.data_ptr(), K + pw, M, N, K, epi,
                                              b.data_ptr(), r.data_ptr(), out1.data_ptr(), s))


def test_rmsnorm(eng):
    from pgmi import _native as NN
    rng = np.random.default_rng(3)
    x, w = rand(rng, 300, 2048, scale=3.0), rand(rng, 2048, scale=0.1)
    out = torch.empty((300, 2048), dtype=torch.bfloat16, device="cuda")
    xt, wt = bf(x), bf(w)  # keep the inputs alive across the call
    NN.check(eng.lib.pgmi_op_rmsnorm(eng.ctx, xt.data_ptr(), wt.data_ptr(), 300, 2048, 1e-6, out.data_ptr(),
                                     NN.stream_handle()))
    torch.cuda.synchronize()
    ref = O.rms_norm(x, w, 1e-6)
    assert ulp_frac(np32(out), ref, 2) == 1.0


def test_layernorm(eng):
    from pgmi import _native as NN
    rng = np.random.default_rng(4)
    x, w, b = rand(rng, 256, 1152, scale=2.0), O.bf16(1 + rand(rng, 1152, scale=0.1)), rand(rng, 1152, scale=0.05)
    out = torch.empty((256, 1152), dtype=torch.bfloat16, device="cuda")
    xt, wt, bt = bf(x), bf(w), bf(b)
    NN.check(eng.lib.pgmi_op_layernorm(eng.ctx, xt.data_ptr(), wt.data_ptr(), bt.data_ptr(), 256, 1152,
                                       1e-6, out.data_ptr(), NN.stream_handle()))
    torch.cuda.synchronize()
    ref = O.layer_norm(x, w, b, 1e-6)
    assert ulp_frac(np32(out), ref, 2) > 0.999


def _attn_ref(q, k, v, scale):
    # q (B,Lq,H,d), k/v (B,Lk,Hkv,d)
    H, Hkv = q.shape[2], k.shape[2]
    qh = q.transpose(0, 2, 1, 3)
    kh = np.repeat(k.transpose(0, 2, 1, 3), H // Hkv, axis=1)
    vh = np.repeat(v.transpose(0, 2, 1, 3), H // Hkv, axis=1)
    s = O.bf16(O.bf16(qh @ kh.transpose(0, 1, 3, 2)) * np.float32(scale))
    p = O.bf16(O.softmax_f32(s))
    return O.bf16(p @ vh).transpose(0, 2, 1, 3)


@pytest.mark.parametrize("B,Lq,Lk,H,Hkv,d,scale", [
    (1, 256, 256, 16, 16, 72, 72 ** -0.5),     # SigLIP 224
    (2, 100, 100, 16, 16, 72, 72 ** -0.5),
    (1, 288, 288, 8, 1, 256, 1 / 16),          # Gemma prefill (MQA)
    (2, 33, 70, 8, 1, 256, 1 / 16),            # ragged, keys beyond queries (cache)
    (1, 1, 290, 8, 1, 256, 1 / 16),            # one query position
    (1, 1024, 1024, 16, 16, 72, 72 ** -0.5),   # SigLIP 448
    (1, 1056, 1056, 8, 1, 256, 1 / 16),        # Gemma 448 prefill
    (1, 40, 2100, 8, 1, 256, 1 / 16),          # keys past the old LDS-resident score limit
    (3, 17, 5, 16, 16, 72, 72 ** -0.5),        # fewer keys than one tile
])
def test_attention_prefill(eng, B, Lq, Lk, H, Hkv, d, scale):
    from pgmi import _native as NN
    rng = np.random.default_rng(Lq + Lk + d)
    q, k, v = rand(rng, B, Lq, H, d, scale=2.0), rand(rng, B, Lk, Hkv, d, scale=2.0), rand(rng, B, Lk, Hkv, d)
    o = torch.empty((B, Lq, H, d), dtype=torch.bfloat16, device="cuda")
    qt, kt, vt = bf(q), bf(k), bf(v)
    NN.check(eng.lib.pgmi_op_attention(eng.ctx, qt.data_ptr(), kt.data_ptr(), vt.data_ptr(), o.data_ptr(),
                                       B, Lq, Lk, H, Hkv, d, scale, NN.stream_handle()))
    torch.cuda.synchronize()
    ref = _attn_ref(q, k, v, scale)
    assert rel_l2(np32(o), ref) < 1e-2


@pytest.mark.parametrize("B,K,N", [(1, 2048, 2048), (3, 2048, 2048), (1, 16384, 2048), (4, 16384, 2048),
                                   (8, 2048, 1000), (6, 16384, 512)])
def test_gemv_res(eng, B, K, N):
    from pgmi import _native as NN
    rng = np.random.default_rng(B * K + N)
    x, Wt, h = rand(rng, B, K), rand(rng, N, K, scale=1 / np.sqrt(K)), rand(rng, B, N)
    ht, xt, wt = bf(h), bf(x), bf(Wt)
    NN.check(eng.lib.pgmi_op_gemv_res(eng.ctx, xt.data_ptr(), wt.data_ptr(), B, N, K, ht.data_ptr(),
                                      NN.stream_handle()))
    torch.cuda.synchronize()
    ref = O.bf16(O.bf16(x @ Wt.T) + h)
    assert rel_l2(np32(ht), ref) < 2e-3
    assert ulp_frac(np32(ht), ref, 1) > 0.99


def test_synthetic_fill_matches_oracle(eng):
    """device generator (csrc/kernels_misc.hip) == oracle/wgen.c, bit for bit"""
    for name, view in list(eng.views.items())[:12] + list(eng.views.items())[-6:]:
        ref = W.gen_bf16(name, tuple(view.shape), 1234)
        got = view.contiguous().view(torch.int16).cpu().numpy().view(np.uint16)
        assert np.array_equal(got, ref), name


@pytest.mark.parametrize("rows,V", [(1, 257216), (2, 257216), (3, 1001), (1, 7), (40, 16384), (1500, 300)])
def test_argmax_rows(eng, rows, V):
    """pgmi_argmax == torch.argmax (first maximum wins), with planted ties."""
    g = torch.Generator().manual_seed(rows * 7 + V)
    x = torch.randn(rows, V, generator=g)
    # plant ties of the row maximum at two positions; the earlier must win
    for r in range(rows):
        m = float(x[r].max()) + 1.0
        i, j = sorted(torch.randint(0, V, (2,), generator=g).tolist())
        x[r, j] = m
        x[r, i] = m
    xd = x.cuda()
    got = eng.argmax(xd).cpu()
    assert torch.equal(got, x.argmax(-1))
    # unaligned view (offset by one float): exercises the scalar path
    if V > 8:
        y = torch.randn(rows * V + 1, generator=g)
        yd = y.cuda()[1:].view(rows, V)
        got = torch.empty(rows, dtype=torch.int64, device="cuda")
        from pgmi import _native as N
        N.check(eng.lib.pgmi_argmax(eng.ctx, yd.data_ptr(), rows, V, got.data_ptr(), N.stream_handle()))
        torch.cuda.synchronize()
        assert torch.equal(got.cpu(), y[1:].view(rows, V).argmax(-1))


@pytest.mark.parametrize("variant", [0, 7, 8, 41, 42, 21, 22, 44, 24, 9, 91, 92, 94, 81, 82])
@pytest.mark.parametrize("B,Lq,Lk,H,Hkv,d,scale", [
    (1, 256, 256, 16, 16, 72, 72 ** -0.5),     # SigLIP 224
    (3, 17, 5, 16, 16, 72, 72 ** -0.5),        # fewer keys than one tile
    (2, 100, 200, 16, 16, 72, 72 ** -0.5),     # ragged key count inside a wave's range
    (8, 256, 256, 16, 16, 72, 72 ** -0.5),     # 8 images (configs[3] per GPU)
    (1, 288, 288, 8, 1, 256, 1 / 16),          # Gemma prefill (MQA)
    (2, 33, 70, 8, 1, 256, 1 / 16),            # ragged, keys beyond queries (cache)
    (1, 288, 576, 8, 1, 256, 1 / 16),          # the ablation's step-0 re-feed: 2L keys
    (1, 1056, 1056, 8, 1, 256, 1 / 16),        # Gemma 448 prefill
    (1, 1024, 1024, 16, 16, 72, 72 ** -0.5),   # SigLIP 448
    (2, 300, 1000, 8, 1, 256, 1 / 16),         # ragged key ranges (a last range shorter than the others)
])
def test_attention_forced_variant(eng, variant, B, Lq, Lk, H, Hkv, d, scale):
    """Every prefill attention kernel the tuning hook (pgmi_tune_attention) can force, against the
    oracle restatement (variants a head dim does not have fall back to the default tiled kernel)."""
    from pgmi import _native as NN
    rng = np.random.default_rng(Lq * 3 + Lk + d + variant)
    q, k, v = rand(rng, B, Lq, H, d, scale=2.0), rand(rng, B, Lk, Hkv, d, scale=2.0), rand(rng, B, Lk, Hkv, d)
    o = torch.empty((B, Lq, H, d), dtype=torch.bfloat16, device="cuda")
    qt, kt, vt = bf(q), bf(k), bf(v)
    NN.check(eng.lib.pgmi_tune_attention(variant))
    try:
        NN.check(eng.lib.pgmi_op_attention(eng.ctx, qt.data_ptr(), kt.data_ptr(), vt.data_ptr(), o.data_ptr(),
                                           B, Lq, Lk, H, Hkv, d, scale, NN.stream_handle()))
        torch.cuda.synchronize()
    finally:
        NN.check(eng.lib.pgmi_tune_attention(-1))
    assert rel_l2(np32(o), _attn_ref(q, k, v, scale)) < 1e-2


@pytest.mark.parametrize("cfg", [36, 37])
@pytest.mark.parametrize("M,N,K,epi,split", [
    (1056, 512, 2048, "geglu", 1),     # 448 px gate|up shape (rows past 1056: clamped, never stored)
    (300, 384, 1024, "store", 1),      # ragged M, N not a multiple of the tile
    (520, 256, 2048, "res", 3),        # split-K partials + the fixed-order epilogue reduction
    (256, 512, 192, "store", 1),       # 3 K-tiles: an odd tile count (the last iteration's second half idle)
])
def test_gemm_8phase(eng, cfg, M, N, K, epi, split):
    """The 8-phase large-M GEMM (k_gemm_8p, plans E256 / E192) forced through the tuning hook."""
    from pgmi import _native as NN
    from pgmi._native import EPI
    rng = np.random.default_rng(M + N + K + cfg)
    A = rand(rng, M, K)
    NN.check(eng.lib.pgmi_tune_gemm(cfg, split))
    try:
        if epi == "geglu":
            Wg, Wu = rand(rng, N, K, scale=2 / np.sqrt(K)), rand(rng, N, K, scale=2 / np.sqrt(K))
            got = _gemm(eng, bf(A), bf(np.concatenate([Wg, Wu])), 7, geglu=True)
            ref = O.bf16(O.gelu_tanh(O.bf16(A @ Wg.T)) * O.bf16(A @ Wu.T))
            tol = 5e-3
        else:
            Wt = rand(rng, N, K, scale=1 / np.sqrt(K))
            r = rand(rng, M, N)
            got = _gemm(eng, bf(A), bf(Wt), EPI[epi], res=bf(r))
            ref = O.bf16(O.bf16(A @ Wt.T) + r) if epi == "res" else O.bf16(A @ Wt.T)
            tol = 3e-3
    finally:
        NN.check(eng.lib.pgmi_tune_gemm(-1, 0))
    assert rel_l2(got, ref) < tol
