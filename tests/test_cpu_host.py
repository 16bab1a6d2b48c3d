"""Host-side logic and the C ABI surface, CPU only (no compute calls without a GPU)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from tests_helpers import pixels_from_u8

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(REPO, "include", "pgmi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pgmi_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from pgmi import _native as N
    lib = N.lib()
    declared = header_functions()
    assert len(declared) >= 25
    for name in declared:
        assert hasattr(lib, name), name
    # the ctypes binding covers the whole header
    assert set(declared) == set(N.SIGNATURES), set(declared) ^ set(N.SIGNATURES)
    assert lib.pgmi_version().startswith(b"pgmi")


@pytest.mark.parametrize("n_mt,n_nt,S,BM,BN,K,blocked", [
    (8, 16, 2, 288, 128, 16384, True),     # 8-image text down (W288w split 2): the XCD block raster
    (8, 9, 2, 288, 128, 4304, None),       # 8-image vision fc2
    (9, 128, 1, 256, 256, 2048, None),     # 8-image gate|up (E256, dual)
    (6, 8, 5, 192, 256, 16384, False),     # 448 px down (E192 split 5): below the 2,048-row panel bound
    (1, 128, 1, 288, 128, 2048, False),    # 224 px gate|up (W288n, one row tile)
    (3, 16, 4, 128, 128, 16384, False),    # 224 px down (W128x128 split 4)
    (4, 18, 1, 64, 64, 1152, False),       # vision out_proj (P64x64s4)
    (2048, 3, 1, 128, 128, 2048, False),   # M = 262,144 rows: n_mt past the old 10-bit packing
    (7, 5, 3, 64, 64, 640, False),         # a grid that is not a multiple of 8
])
def test_gemm_tile_order_is_a_permutation(n_mt, n_nt, S, BM, BN, K, blocked):
    """Every workgroup of a panel / 8-phase GEMM grid gets a distinct (row tile, column tile, K slice)
    (kernels_gemm.hip xcd_tile, its host replica): the XCD block raster and the run order are both
    permutations of the tile set, at every row-tile count (the block code travels in its own argument)."""
    from pgmi import _native as N
    lib = N.lib()
    G = n_mt * n_nt * S
    mt, nt, z = (np.zeros(G, np.int32) for _ in range(3))
    code = lib.pgmi_debug_gemm_tiles(n_mt, n_nt, S, BM, BN, K, mt.ctypes.data, nt.ctypes.data, z.ctypes.data)
    assert code >= 0
    if blocked is not None:
        assert (code != 0) == blocked, code
    assert mt.min() >= 0 and mt.max() < n_mt and nt.min() >= 0 and nt.max() < n_nt and z.min() >= 0 and z.max() < S
    flat = (mt.astype(np.int64) * n_nt + nt) * S + z
    assert np.array_equal(np.sort(flat), np.arange(G))


def test_create_validates_config_without_gpu():
    """pgmi_create only builds the weight layout (no device memory): it runs here."""
    from pgmi import _native as N
    from pgmi.engine import config_dict
    from pgmi.synthetic import paligemma_3b_config
    lib = N.lib()
    cd = config_dict(paligemma_3b_config())
    c = N.PgmiConfig()
    for k, _ in N.PgmiConfig._fields_:
        if k not in ("max_batch", "max_seq", "max_kv"):
            setattr(c, k, cd[k])
    c.max_batch, c.max_seq, c.max_kv = 1, 288, 1024
    h = ctypes.c_void_p()
    assert lib.pgmi_create(0, ctypes.byref(c), ctypes.byref(h)) == 0
    # slab: every reference parameter of PaliGemma-3B (lm_head tied), 256-B aligned, 2,923,466,480 params
    n = lib.pgmi_weight_count(h)
    total = 0
    for i in range(n):
        name, off, shape, nd = ctypes.c_char_p(), ctypes.c_int64(), (ctypes.c_int64 * 4)(), ctypes.c_int()
        assert lib.pgmi_weight_info(h, i, ctypes.byref(name), ctypes.byref(off), ctypes.byref(shape), ctypes.byref(nd)) == 0
        assert off.value % 256 == 0
        total += int(np.prod([shape[j] for j in range(nd.value)]))
    assert total == 2_923_466_480  # SURVEY.md sec.3.5 (the tied lm_head counted once)
    assert lib.pgmi_weights_bytes(h) >= 2 * total
    assert lib.pgmi_kv_bytes(h, 1, 1024) == 18 * 2 * 1024 * 256 * 2
    lib.pgmi_destroy(h)
    # invalid configs are rejected with PGMI_E_ARG and a message
    c.t_kv_heads = 2
    assert lib.pgmi_create(0, ctypes.byref(c), ctypes.byref(h)) == N.PGMI_E_ARG
    assert b"MQA" in lib.pgmi_last_error()


def test_fused_layout_adjacency():
    """q|k|v (and gate|up) are adjacent in the slab so one GEMM/GEMV covers them."""
    from pgmi import _native as N
    from pgmi.engine import config_dict
    from pgmi.synthetic import paligemma_3b_config
    lib = N.lib()
    cd = config_dict(paligemma_3b_config())
    c = N.PgmiConfig()
    for k, _ in N.PgmiConfig._fields_:
        if k not in ("max_batch", "max_seq", "max_kv"):
            setattr(c, k, cd[k])
    c.max_batch, c.max_seq, c.max_kv = 1, 288, 1024
    h = ctypes.c_void_p()
    assert lib.pgmi_create(0, ctypes.byref(c), ctypes.byref(h)) == 0
    info = {}
    for i in range(lib.pgmi_weight_count(h)):
        name, off, shape, nd = ctypes.c_char_p(), ctypes.c_int64(), (ctypes.c_int64 * 4)(), ctypes.c_int()
        lib.pgmi_weight_info(h, i, ctypes.byref(name), ctypes.byref(off), ctypes.byref(shape), ctypes.byref(nd))
        info[name.value.decode()] = (off.value, int(np.prod([shape[j] for j in range(nd.value)])) * 2)
    lib.pgmi_destroy(h)
    for p in ("language_model.model.layers.5.self_attn.", "vision_tower.vision_model.encoder.layers.3.self_attn."):
        q, k, v = (info[p + f"{n}_proj.weight"] for n in "qkv")
        assert q[0] + q[1] == k[0] and k[0] + k[1] == v[0]
    g, u = info["language_model.model.layers.7.mlp.gate_proj.weight"], info["language_model.model.layers.7.mlp.up_proj.weight"]
    assert g[0] + g[1] == u[0]


def test_synthetic_policy_matches_oracle():
    from oracle import weights as OW
    from pgmi import synthetic as S
    for image in (224, 448):
        cfg = OW.full_config(image)
        for name, shape in OW.param_shapes(cfg).items():
            assert S.init_policy(name, shape) == OW.init_policy(name, shape), name
    assert S.paligemma_3b_config(448) == OW.full_config(448)
    ids = S.prompt_ids(257152, 256, 257216)
    assert ids.shape == (1, 288) and ids[0, 256] == 2 and ids[0, -1] == 108


def test_kvcache_reference_semantics():
    """KVCache driven through update() behaves as modeling_gemma.py:10-36."""
    import modeling_gemma as MG
    kv = MG.KVCache()
    assert kv.num_items() == 0
    k = torch.randn(1, 1, 5, 256)
    kv.update(k, k, 0)
    kv.update(k, k, 1)
    kk, vv = kv.update(torch.randn(1, 1, 1, 256), torch.randn(1, 1, 1, 256), 0)
    assert kk.shape == (1, 1, 6, 256) and kv.num_items() == 6
    assert len(kv.key_cache) == 2


def test_positions_helper():
    import modeling_gemma as MG
    p = MG._positions_2d(torch.tensor([[289.0]]), 1, 1)
    assert p.dtype == torch.int64 and p.tolist() == [[289]]
    p = MG._positions_2d(torch.arange(5), 2, 5)
    assert p.shape == (2, 5) and p[1].tolist() == [0, 1, 2, 3, 4]
    p = MG._positions_2d(torch.tensor([[7.0], [7.0]]), 2, 3)  # patched merge, q_len > 1
    assert p.tolist() == [[7, 7, 7], [7, 7, 7]]


def test_configs_and_module_tree():
    import modeling_gemma as MG
    from pgmi.synthetic import paligemma_3b_config
    cfg = MG.PaliGemmaConfig(**{k: v for k, v in paligemma_3b_config().items() if k not in ("bos_token_id", "eos_token_id")})
    assert cfg.vision_config.num_image_tokens is None and cfg.text_config.num_image_tokens == 256
    assert cfg.vision_config.projection_dim == 2048 and cfg.vocab_size == 257216
    with torch.device("meta"):
        m = MG.PaliGemmaForConditionalGeneration(cfg)
    m.tie_weights()
    n = sum(p.numel() for p in m.parameters())
    assert n == 2_923_466_480
    # no CPU fallback: a model that is not on the GPU refuses to run
    with pytest.raises(RuntimeError):
        m(input_ids=torch.zeros(1, 4, dtype=torch.long), attention_mask=torch.ones(1, 4, dtype=torch.long))


def test_processing_matches_reference_arithmetic(golden_dir):
    import processing_paligemma as P
    d = np.load(os.path.join(golden_dir, "pixels.npz"))
    u8 = d["u8_1_224"]
    ours = P.normalize(P.rescale(u8, 1 / 255.0), P.IMAGENET_STANDARD_MEAN, P.IMAGENET_STANDARD_STD).transpose(2, 0, 1)
    assert np.array_equal(ours, pixels_from_u8(u8))
    from PIL import Image
    img = Image.fromarray(d["u8_0_448"])
    out = P.process_images([img], size=(224, 224), resample=Image.Resampling.BICUBIC, rescale_factor=1 / 255.0,
                           image_mean=P.IMAGENET_STANDARD_MEAN, image_std=P.IMAGENET_STANDARD_STD)
    assert out[0].shape == (3, 224, 224) and out[0].dtype == np.float32
    assert P.add_image_tokens_to_prompt("hi", "<bos>", 3, "<image>") == "<image><image><image><bos>hi\n"


def test_shard_range():
    from pgmi.dist import shard_range
    for n in (1, 7, 64):
        for w in (1, 2, 3, 8):
            got = [shard_range(n, r, w) for r in range(w)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(got[i][1] == got[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in got) - min(h - l for l, h in got) <= 1


def test_merged_positions_and_mask_check():
    """The patched-merge path reads a merge's positions and checks its mask in one host copy; a
    non-zero additive mask is refused (libpgmi attends every cached key, the reference's zero mask)."""
    import modeling_gemma as MG
    m = torch.zeros(1, 1, 1, 577, dtype=torch.bfloat16)
    pos = MG._merged_positions(torch.tensor([[289.0]]), m, 1, 1)          # decode: float cumsum
    assert pos.tolist() == [[289]] and pos.dtype == torch.int64
    pos = MG._merged_positions(torch.tensor([[288]]), torch.zeros(1, 1, 288, 576), 1, 288)  # step-0 re-feed
    assert pos.shape == (1, 288) and bool((pos == 288).all())
    pos = MG._merged_positions(torch.arange(5).unsqueeze(0), torch.zeros(1, 1, 5, 5), 1, 5)
    assert pos.tolist() == [[0, 1, 2, 3, 4]]
    with pytest.raises(NotImplementedError):
        MG._merged_positions(torch.arange(5).unsqueeze(0), torch.full((1, 1, 5, 5), -1e4), 1, 5)


def test_ablation_patches_restated_match_reference_semantics():
    """tests_helpers' restated ablation merge: a filled cache puts every query row at cumsum(mask)[-1]
    and widens the mask to cached + q_len keys (ablation_study_fixed.py:121-133)."""
    import types
    from tests_helpers import ablation_merge
    cfg = types.SimpleNamespace(image_token_index=9, hidden_size=4,
                                text_config=types.SimpleNamespace(max_position_embeddings=8))
    self = types.SimpleNamespace(config=cfg, pad_token_id=0)
    ids = torch.tensor([[9, 9, 5, 0, 6]])
    emb = torch.ones(1, 5, 4)
    img = torch.full((1, 2, 4), 2.0)
    kv = types.SimpleNamespace(num_items=lambda: 5)
    out, mask, pos = ablation_merge(self, img, emb, ids, torch.ones(1, 5, dtype=torch.long), kv)
    assert mask.shape == (1, 1, 5, 10) and pos.tolist() == [[5]]
    assert torch.equal(out[0, :, 0], torch.tensor([1.0, 1.0, 1.0, 0.0, 1.0]))  # 2 / sqrt(4) = 1; pad row zero
    out, mask, pos = ablation_merge(self, img, emb, ids, torch.ones(1, 12, dtype=torch.long)[:, :5], None)
    assert mask.shape == (1, 1, 5, 5) and pos.tolist() == [[0, 1, 2, 3, 4]]


def test_prefill_gemm_shape_labels(tmp_path):
    """tools/prefill_gemm_shapes.py labels the prefill MLP GEMMs of a kernel trace by template (round 6: the
    M = 288 down runs W288n split 8, its own template, and o_proj W128x128 split 4); a W288w split launch is
    the 8-image down only right after the 8-image gate|up -- the per-shape figures bench.py's in-situ
    prefill_gemm_roofline is checked against."""
    import csv
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("pgs", os.path.join(root, "tools", "prefill_gemm_shapes.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    seq = [("k_attn_fs", 5), (m.W128S, 10), ("k_splitk", 3), (m.GU224, 44), (m.DN224, 36), ("k_splitk", 3),
           (m.GU224, 44), (m.DN224, 36), (m.DN224, 38), ("x", 1), (m.GU448, 126), (m.DN448, 72),
           (m.DN8, 50), (m.GU8, 300), (m.DN8, 200)]
    tr = tmp_path / "trace.csv"
    with open(tr, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        t = 0
        for name, us in seq:
            w.writerow([f"void pgmi::{name}(args)", t, t + us * 1000])
            t += us * 1000 + 500
    out = tmp_path / "out.csv"
    m.main(str(tr), str(out))
    rows = {r["label"]: r for r in csv.DictReader(open(out))}
    assert rows["224 o_proj (M=288)"]["launches"] == "1" and float(rows["224 o_proj (M=288)"]["mean_us"]) == 10
    assert rows["224 down (M=288)"]["launches"] == "3" and float(rows["224 down (M=288)"]["median_us"]) == 36
    assert rows["8-image down (M=2304)"]["launches"] == "1" and float(rows["8-image down (M=2304)"]["mean_us"]) == 200
    assert float(rows["448 gate|up + GeGLU (M=1056)"]["mean_us"]) == 126


def test_bench_decode_chunking():
    """bench.py's batched decode legs (configs[3], the N > 1 lines) run the generate driver's steps per graph launch
    (decode_chunk): GEN_CHUNK for 3+ rows, halved until it divides the timed steps and two chunks fit in the warmup
    (the second call with a buffer set is the one that captures its graph); one step per launch for B <= 2 or
    without graphs.  run_decode walks the KV rows and positions in order, chunk by chunk, singles at the tail."""
    import sys
    sys.path.insert(0, REPO)
    import bench
    from pgmi import Engine
    assert Engine.GEN_CHUNK == 8 and Engine.GEN_MIN_BATCH == 3
    assert bench.decode_chunk(1, 20, 16) == 1 and bench.decode_chunk(2, 256, 16) == 1
    assert bench.decode_chunk(8, 256, 16) == 8 and bench.decode_chunk(8, 20, 16) == 4
    assert bench.decode_chunk(8, 20, 5) == 2 and bench.decode_chunk(8, 7, 16) == 1
    assert bench.decode_chunk(8, 256, 16, graph=False) == 1 and bench.decode_chunk(3, 256, 0) == 1

    class FakeEngine:
        def __init__(self):
            self.calls = []

        def decode_steps(self, cur, kv, kv_len, position, n, logits=None, graph=False):
            self.calls.append(("steps", kv_len, position, n))

        def decode(self, cur, kv, kv_len, position, logits=None, next_ids=None, graph=False):
            assert next_ids is cur  # greedy feedback in place
            self.calls.append(("one", kv_len, position, 1))

    e = FakeEngine()
    bench.run_decode(e, "cur", None, 288, 0, 5, 2, None, True)
    bench.run_decode(e, "cur", None, 288, 5, 8, 4, None, True)
    assert e.calls == [("steps", 288, 289, 2), ("steps", 290, 291, 2), ("one", 292, 293, 1),
                       ("steps", 293, 294, 4), ("steps", 297, 298, 4)]
