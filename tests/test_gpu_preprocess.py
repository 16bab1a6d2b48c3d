"""GPU image preprocessing (processing_paligemma.py:13-49) through the
C ABI (pgmi_preprocess) vs PIL's own BICUBIC outputs recorded in tests/golden/preprocess.npz
(tests/golden/make_preprocess.py) and the reference's pixel_values restatement.

Bar: bit-exact -- the uint8 resample is integer arithmetic after double-precision weights, and
the float pixels follow from it by the reference's exact float32 ops."""
import os
import sys

import numpy as np
import pytest
import torch

from oracle import resize_np as R
from oracle import weights as W

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from make_preprocess import SYNTH, synthetic_image  # noqa: E402


@pytest.fixture(scope="module")
def eng():
    from pgmi import Engine
    e = Engine(W.small_config(vision_layers=1, text_layers=1, vocab=1024), max_batch=1, max_seq=320, max_kv=512)
    e.fill_synthetic(7, W.init_policy)
    e.prepare()
    return e


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(HERE, "golden", "preprocess.npz"))


def cases(gold):
    out = [(gold["coco0_src"], s, gold[f"coco0_{s}"]) for s in (224, 448)]
    for seed, h, w, s in SYNTH:
        out.append((synthetic_image(seed, h, w), s, gold[f"syn{seed}_{h}x{w}_{s}"]))
    return out


def test_pixels_bit_exact_vs_pil(eng, gold):
    for src, size, pil_u8 in cases(gold):
        px = eng.preprocess([src], size=size)
        torch.cuda.synchronize()
        want = R.pixels_from_u8(pil_u8)
        got = px[0].cpu().numpy()
        assert got.shape == want.shape
        assert np.array_equal(got, want), (src.shape, size, float(np.abs(got - want).max()))


def test_batch_and_processor_path(eng, gold):
    from PIL import Image
    import processing_paligemma as P
    imgs = [Image.fromarray(gold["coco0_src"]), Image.fromarray(synthetic_image(1, 480, 640))]
    px = P.process_images_gpu(imgs, (224, 224), eng)
    ref = np.stack(P.process_images(imgs, size=(224, 224), resample=Image.Resampling.BICUBIC,
                                    rescale_factor=1 / 255.0, image_mean=P.IMAGENET_STANDARD_MEAN,
                                    image_std=P.IMAGENET_STANDARD_STD))
    assert np.array_equal(px.cpu().numpy(), ref)


def test_rejects_bad_input(eng):
    with pytest.raises(ValueError):
        eng.preprocess([np.zeros((10, 10), np.uint8)])
