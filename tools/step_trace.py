"""Timeline of one fused decode step (PGMI_STEP_TRACE=1): per phase, when its workgroups were
placed, got their inputs and published, in us from the first placement (s_memrealtime, 100 MHz)."""
import ctypes
import os
import sys

os.environ["PGMI_STEP_TRACE"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-financial-analysis-tool-using-paligemma_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import weights as W  # noqa: E402
from pgmi import Engine  # noqa: E402


def main():
    e = Engine(W.full_config(224), max_batch=1, max_seq=320, max_kv=512)
    e.fill_synthetic(1234, W.init_policy)
    e.prepare()
    kv = e.new_kv(1, 512)
    L = 288
    ids = torch.randint(3, 4000, (1, L), device="cuda")
    e.lm_forward(kv, 0, torch.arange(L)[None], ids=ids, logits_rows=1)
    tok = torch.tensor([5], device="cuda")
    for t in range(6):
        e.decode(tok, kv, L + t, L + t + 1, graph=False)
    torch.cuda.synchronize()
    t0 = __import__("time").perf_counter()
    for t in range(6, 26):
        e.decode(tok, kv, L + t, L + t + 1, graph=False)
    torch.cuda.synchronize()
    print(f"eager fused step (traced) {(__import__('time').perf_counter() - t0) / 20 * 1e6:.1f} us")
    n = 80000
    buf = (ctypes.c_longlong * (4 * n))()
    got = e.lib.pgmi_decode_trace(e.ctx, ctypes.addressof(buf), 4 * n)
    tr = np.frombuffer(buf, dtype=np.int64)[: 4 * got].reshape(got, 4).astype(np.float64)
    base = tr[:, 0].min()
    us = (tr - base) / 100.0  # 100 MHz ticks -> us
    cfg = e.cfgd
    nqkv = (cfg["t_heads"] + 2 * cfg["t_kv_heads"]) * 128 // 4
    nat = (512 + 63) // 64
    # workgroups per phase: kernels_step.hip (kOUpb 32, kGuUpb 64, kDnUpb 8, kLmUpb 1008)
    no, ngu, ndn = -(-cfg["t_hidden"] // 32), -(-cfg["t_intermediate"] // 64), -(-cfg["t_hidden"] // 8)
    nlm = -(-cfg["t_vocab"] // 1008)
    per = nqkv + nat + no + ngu + ndn
    names = ["qkv", "attn", "o", "gu", "dn"]
    sizes = [nqkv, nat, no, ngu, ndn]
    print(f"grid {got} workgroups, step span {us[:, 2].max():.1f} us (entry..last publish)")
    print("phase      placed[first,last]   ready[first,last]   done[last]")
    for l in list(range(3)) + [17]:
        b = 1 + l * per
        for nm, sz in zip(names, sizes):
            seg = us[b:b + sz]
            if nm == "attn":
                seg = seg[:5]
            print(f"L{l:02d} {nm:4s}  {seg[:,0].min():8.1f} {seg[:,0].max():8.1f}   {seg[:,1].min():8.1f} "
                  f"{seg[:,1].max():8.1f}   {seg[:,2].max():8.1f}")
            b += sz
    lm = us[1 + 18 * per: 1 + 18 * per + nlm]
    print(f"lm    {lm[:,0].min():8.1f} {lm[:,0].max():8.1f}   {lm[:,1].min():8.1f} {lm[:,1].max():8.1f}   "
          f"{lm[:,2].max():8.1f}")
    print(f"argmax entry {us[-1,0]:.1f} ready {us[-1,1]:.1f}")
    print("status", e.decode_status())


if __name__ == "__main__":
    main()
