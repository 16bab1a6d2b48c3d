"""Probe: phase timeline of the prefill attention at the Gemma-224 shape from in-kernel stamps
(attention variant 9 = k_attn_full_pre with s_memrealtime stamps, pgmi_debug_stamps): per phase the
median / max over workgroups of (stamp - the workgroup's first stamp), in microseconds.
    python tools/probes/attn_stamps.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"), REPO]
from oracle import weights as W  # noqa: E402
from pgmi import Engine  # noqa: E402
from pgmi import _native as NN  # noqa: E402

eng = Engine(W.small_config(vision_layers=1, text_layers=1, vocab=1024), max_batch=1, max_seq=64, max_kv=64)
L, H, Hkv, d = 288, 8, 1, 256
q = (torch.randn(1, L, H, d, device="cuda") * 2).bfloat16()
k = (torch.randn(1, L, Hkv, d, device="cuda") * 2).bfloat16()
v = torch.randn(1, L, Hkv, d, device="cuda").bfloat16()
o = torch.empty_like(q)
NN.check(eng.lib.pgmi_tune_attention(9))
for _ in range(5):
    NN.check(eng.lib.pgmi_op_attention(eng.ctx, q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                       1, L, L, H, Hkv, d, d ** -0.5, NN.stream_handle()))
torch.cuda.synchronize()
nwg = (L * H + 15) // 16
buf = (ctypes.c_longlong * (nwg * 8 * 64))()
NN.check(eng.lib.pgmi_debug_stamps(0, buf, nwg * 8 * 64))
st = np.frombuffer(buf, dtype=np.int64).reshape(nwg, 8, 64)[:, :, 0].astype(np.float64) / 100.0  # 100 MHz -> us
t0 = st[:, 0].min()
names = ["start", "loads issued", "phase 1 (QK^T) + barrier", "phase 2 (softmax)", "phase 3 (P.V)", "stores"]
print(f"{nwg} workgroups; launch spread of start {st[:, 0].max() - t0:.2f} us")
for p in range(1, 6):
    dt = st[:, p] - st[:, p - 1]
    print(f"{names[p]:28s} median {np.median(dt):7.2f} us  max {dt.max():7.2f} us")
tot = st[:, 5] - st[:, 0]
print(f"{'workgroup total':28s} median {np.median(tot):7.2f} us  max {tot.max():7.2f} us; "
      f"last end - first start {st[:, 5].max() - t0:.2f} us")
