"""CPU restatement of the reference's image preprocessing (test infrastructure only).

processing_paligemma.py:13-18 resizes with PIL `Image.resize(size, resample=BICUBIC)`; PIL
(pillow==11.3.0 pinned by the reference, not vendored) implements it in libImaging/Resample.c
as a separable two-pass convolution:
  * precompute_coeffs: for output index xx, center = (xx + 0.5) * scale, filterscale =
    max(scale, 1), support = 2 * filterscale, taps x in [int(center - support + 0.5),
    int(center + support + 0.5)) clipped to the image, weights bicubic((x - center + 0.5) /
    filterscale) with a = -0.5, normalised by their sum (all in double);
  * normalize_coeffs_8bpc: weights to fixed point with PRECISION_BITS = 22, rounding half away
    from zero (int(w * 2^22 +- 0.5));
  * horizontal pass first (rows bounds_vert[0] .. last used row only), to a uint8 image with
    clip8((sum + 2^21) >> 22); then the vertical pass over that image, same arithmetic.
Then :20-29,43-49: x/255 (float64 -> float32), (x - 0.5)/0.5 in float32, HWC -> CHW.
Pinned bit-exact against PIL on tests/golden/preprocess.npz (tests/test_cpu_oracle.py).
"""
import numpy as np

PRECISION_BITS = 32 - 8 - 2


def bicubic(x):
    a = -0.5
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def precompute_coeffs(in_size, out_size):
    """Resample.c precompute_coeffs + normalize_coeffs_8bpc: (bounds [out][2], int32 kk [out][ksize])."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    ksize = int(np.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [bicubic((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for v in w:
            ww += v
        if ww != 0.0:
            w = [v / ww for v in w]
        for x, v in enumerate(w):
            kk[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _clip8(acc):
    return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def resize_bicubic_u8(img, out_h, out_w):
    """PIL BICUBIC resize of a uint8 HWC RGB image (ImagingResampleInner semantics)."""
    in_h, in_w, _ = img.shape
    bh, kh = precompute_coeffs(in_w, out_w)
    bv, kv = precompute_coeffs(in_h, out_h)
    need_h = out_w != in_w
    need_v = out_h != in_h
    cur = img
    if need_h:
        y0 = int(bv[0, 0])
        y1 = int(bv[-1, 0] + bv[-1, 1])
        src = img[y0:y1].astype(np.int64)
        out = np.empty((y1 - y0, out_w, 3), np.uint8)
        for xx in range(out_w):
            xmin, n = bh[xx]
            acc = np.full((y1 - y0, 3), 1 << (PRECISION_BITS - 1), np.int64)
            acc += np.einsum("hxc,x->hc", src[:, xmin:xmin + n], kh[xx, :n])
            out[:, xx] = _clip8(acc)
        cur = out
        bv = bv.copy()
        bv[:, 0] -= y0
    if need_v:
        src = cur.astype(np.int64)
        out = np.empty((out_h, cur.shape[1], 3), np.uint8)
        for yy in range(out_h):
            ymin, n = bv[yy]
            acc = np.full((cur.shape[1], 3), 1 << (PRECISION_BITS - 1), np.int64)
            acc += np.einsum("ywc,y->wc", src[ymin:ymin + n], kv[yy, :n])
            out[yy] = _clip8(acc)
        cur = out
    return cur


def pixels_from_u8(u8):
    """processing_paligemma.py:20-29,47-49 on the resized uint8 image: float32 CHW."""
    px = (u8 * (1 / 255.0)).astype(np.float32)
    return ((px - np.float32(0.5)) / np.float32(0.5)).transpose(2, 0, 1)
