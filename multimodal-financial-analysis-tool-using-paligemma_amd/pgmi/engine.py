"""Engine: one libpgmi context on one GPU (weights slab, KV slabs, forward calls).

Device memory for the weights and the KV caches is torch-allocated (so the Python API can
expose the reference's parameter / cache tensors as views of it); the library owns its
workspaces.  Every compute call goes through libpgmi.so -- nothing here computes on the CPU.
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional

import torch

from . import _native as N


def config_dict(cfg) -> dict:
    """Accept a PaliGemmaConfig (reference or drop-in) or an HF-style config.json dict."""
    if isinstance(cfg, dict):
        v, t = dict(cfg["vision_config"]), dict(cfg["text_config"])
        top = cfg
        get = top.get
    else:
        v = dict(vars(cfg.vision_config))
        t = dict(vars(cfg.text_config))
        top = vars(cfg)
        get = top.get
    pad = get("pad_token_id", None)
    return {
        "v_hidden": v.get("hidden_size", 768), "v_intermediate": v.get("intermediate_size", 3072),
        "v_layers": v.get("num_hidden_layers", 12), "v_heads": v.get("num_attention_heads", 12),
        "v_channels": v.get("num_channels", 3), "v_image": v.get("image_size", 224),
        "v_patch": v.get("patch_size", 16), "v_ln_eps": v.get("layer_norm_eps", 1e-6),
        "t_vocab": t["vocab_size"], "t_hidden": t["hidden_size"], "t_intermediate": t["intermediate_size"],
        "t_layers": t["num_hidden_layers"], "t_heads": t["num_attention_heads"],
        "t_kv_heads": t["num_key_value_heads"], "t_head_dim": t.get("head_dim", 256),
        "t_max_pos": t.get("max_position_embeddings", 8192), "t_rms_eps": t.get("rms_norm_eps", 1e-6),
        "t_rope_theta": t.get("rope_theta", 10000.0),
        "projection_dim": get("projection_dim", 2048), "image_token_index": get("image_token_index", 256000),
        "pad_token_id": -1 if pad is None else int(pad),
        "hidden_size": get("hidden_size", 2048),
    }


class Engine:
    # generate(): greedy steps per hipGraph launch (pgmi_decode_steps) for batches of GEN_MIN_BATCH rows or more.
    # Same box (tools/probes/multistep_probe.py): B = 8 step 1.279 -> 1.271 ms at 8-16 steps per launch, B = 1
    # 1.056 -> 1.060 ms (slower: B <= 2 keeps one launch per step)
    GEN_CHUNK = 8
    GEN_MIN_BATCH = 3

    def __init__(self, cfg, device=None, max_batch: int = 8, max_seq: int = 1472, max_kv: Optional[int] = None):
        self.lib = N.lib()
        self.cfgd = config_dict(cfg)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   torch.device(device).index or 0)
        c = N.PgmiConfig()
        for k, _ in N.PgmiConfig._fields_:
            if k in ("max_batch", "max_seq", "max_kv"):
                continue
            setattr(c, k, self.cfgd[k])
        c.max_batch, c.max_seq = max_batch, max_seq
        c.max_kv = max_kv if max_kv else self.cfgd["t_max_pos"]
        self.max_batch, self.max_seq, self.max_kv = max_batch, max_seq, c.max_kv
        h = ctypes.c_void_p()
        N.check(self.lib.pgmi_create(self.device.index, ctypes.byref(c), ctypes.byref(h)), "pgmi_create")
        self.ctx = h
        nbytes = self.lib.pgmi_weights_bytes(self.ctx)
        self.slab = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        N.check(self.lib.pgmi_bind_weights(self.ctx, self.slab.data_ptr()), "pgmi_bind_weights")
        self.views = {}
        for i in range(self.lib.pgmi_weight_count(self.ctx)):
            name, off, shape, nd = ctypes.c_char_p(), ctypes.c_int64(), (ctypes.c_int64 * 4)(), ctypes.c_int()
            N.check(self.lib.pgmi_weight_info(self.ctx, i, ctypes.byref(name), ctypes.byref(off),
                                              ctypes.byref(shape), ctypes.byref(nd)))
            shp = tuple(shape[j] for j in range(nd.value))
            numel = math.prod(shp)
            self.views[name.value.decode()] = self.slab[off.value: off.value + 2 * numel].view(torch.bfloat16).view(shp)
        self.prepared = False
        self._logits_buf = {}

    def __del__(self):
        try:
            if getattr(self, "ctx", None):
                # a greedy lookahead step (pgmi/lookahead.py) may still run on its side stream in this context's
                # workspace: it ends before the context's memory is released
                la = self.__dict__.get("_lookahead")
                if la is not None and la.last is not None:
                    la.last.synchronize()
                self.lib.pgmi_destroy(self.ctx)
                self.ctx = None
        except Exception:
            pass

    # ------------------------------------------------------------------ weights
    def names(self):
        return list(self.views.keys())

    @torch.no_grad()
    def load_state_dict(self, sd: dict, strict: bool = True):
        missing = [n for n in self.views if n not in sd]
        if strict and missing:
            raise KeyError(f"missing weights: {missing[:5]}{'...' if len(missing) > 5 else ''}")
        for n, view in self.views.items():
            if n in sd:
                t = sd[n]
                if tuple(t.shape) != tuple(view.shape):
                    raise ValueError(f"{n}: shape {tuple(t.shape)} != {tuple(view.shape)}")
                view.copy_(t.to(device=self.device, dtype=torch.bfloat16))
        self.prepared = False

    def load_safetensors(self, path: str, strict: bool = True) -> int:
        """Native safetensors loading into the slab (pgmi_load_safetensors).
        `path` is a *.safetensors file or a directory of shards.  With strict, every slab weight
        must come from the files.  Returns the number of tensors loaded."""
        import glob
        import os
        files = sorted(glob.glob(os.path.join(path, "*.safetensors"))) if os.path.isdir(path) else [path]
        if not files:
            raise FileNotFoundError(f"no *.safetensors under {path}")
        s = N.stream_handle(self.device)
        got = set()
        total = 0
        for f in files:
            nl, ns = ctypes.c_int(), ctypes.c_int()
            N.check(self.lib.pgmi_load_safetensors(self.ctx, f.encode(), ctypes.byref(nl), ctypes.byref(ns), s), f)
            total += nl.value
            got.update(e[0] for e in N.safetensors_index(f) if e[0] in self.views)
        missing = [n for n in self.views if n not in got]
        if strict and missing:
            raise KeyError(f"{len(missing)} weights missing from {path}: {missing[:4]}")
        self.prepared = False
        return total

    def fill_synthetic(self, seed: int, policy):
        """Device-side deterministic init (oracle/wgen.c recipe); policy(name, shape) -> (scale, offset)."""
        s = N.stream_handle(self.device)
        for n, view in self.views.items():
            scale, offset = policy(n, tuple(view.shape))
            key = self.lib.pgmi_synthetic_key(n.encode(), seed)
            N.check(self.lib.pgmi_fill_synthetic(self.ctx, n.encode(), key, scale, offset, s), n)
        self.prepared = False

    def prepare(self, inv_freq: Optional[torch.Tensor] = None, exact_table: bool = True):
        """RoPE tables from the module's inv_freq buffer (the reference's own values) and the
        padded patch matrix.  With exact_table the cos/sin table is computed by torch on the
        CPU exactly as GemmaRotaryEmbedding.forward does (modeling_gemma.py:168-185)."""
        hd, mp = self.cfgd["t_head_dim"], self.cfgd["t_max_pos"]
        if inv_freq is None:
            inv_freq = 1.0 / (self.cfgd["t_rope_theta"] ** (torch.arange(0, hd, 2, dtype=torch.int64).float() / hd))
        inv = inv_freq.detach().float().cpu().contiguous()
        N.check(self.lib.pgmi_set_rope_inv_freq(self.ctx, inv.numpy().ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
        if exact_table:
            pos = torch.arange(mp, dtype=torch.float32)
            freqs = (inv[None, :, None] @ pos[None, None, :]).transpose(1, 2)[0]  # (mp, hd/2) as :178
            cos = freqs.cos().to(torch.bfloat16).contiguous().view(torch.int16)
            sin = freqs.sin().to(torch.bfloat16).contiguous().view(torch.int16)
            N.check(self.lib.pgmi_set_rope_table(self.ctx, cos.data_ptr(), sin.data_ptr(), mp))
        N.check(self.lib.pgmi_prepare(self.ctx), "pgmi_prepare")
        self.prepared = True

    # ------------------------------------------------------------------ caches
    def new_kv(self, batch: int, max_tokens: Optional[int] = None) -> torch.Tensor:
        T = max_tokens or self.max_kv
        t = self.cfgd
        return torch.empty((t["t_layers"], 2, batch, T, t["t_kv_heads"] * t["t_head_dim"]),
                           dtype=torch.bfloat16, device=self.device)

    def scratch_kv(self, batch: int, tokens: int) -> torch.Tensor:
        """Cache for calls without a KVCache (kv_cache=None: the no-KV ablation mode)."""
        cur = getattr(self, "_scratch_kv", None)
        if cur is None or cur.shape[2] < batch or cur.shape[3] < tokens:
            cur = self.new_kv(max(batch, cur.shape[2] if cur is not None else 0),
                              max(tokens, cur.shape[3] if cur is not None else 0))
            self._scratch_kv = cur
        if cur.shape[2] != batch:
            return self.new_kv(batch, tokens)
        return cur

    def logits_buffer(self, batch: int) -> torch.Tensor:
        """Persistent decode logits buffer (a stable pointer lets the decode hipGraph be reused)."""
        buf = self._logits_buf.get(batch)
        if buf is None:
            buf = torch.empty((batch, self.cfgd["t_vocab"]), dtype=torch.float32, device=self.device)
            self._logits_buf[batch] = buf
        return buf

    # ------------------------------------------------------------------ forward pieces
    _stream_guard = None  # pgmi/lookahead.py: makes a call wait for a step still running on its side stream

    def _s(self):
        h = N.stream_handle(self.device)
        if self._stream_guard is not None:
            self._stream_guard(h)
        return h

    def _ready(self):
        if not self.prepared:
            self.prepare()

    def vision(self, pixel_values: torch.Tensor) -> torch.Tensor:
        self._ready()
        px = pixel_values.to(self.device)
        if px.dtype not in (torch.float32, torch.bfloat16):
            px = px.float()
        px = px.contiguous()
        B = px.shape[0]
        c = self.cfgd
        n = (c["v_image"] // c["v_patch"]) ** 2
        if tuple(px.shape[1:]) != (c["v_channels"], c["v_image"], c["v_image"]):
            raise ValueError(f"pixel_values shape {tuple(px.shape)} does not match the vision config")
        out = torch.empty((B, n, c["v_hidden"]), dtype=torch.bfloat16, device=self.device)
        dt = N.DTYPE_F32 if px.dtype == torch.float32 else N.DTYPE_BF16
        N.check(self.lib.pgmi_vision(self.ctx, px.data_ptr(), dt, B, out.data_ptr(), self._s()), "pgmi_vision")
        return out

    def preprocess(self, images, size: Optional[int] = None) -> torch.Tensor:
        """process_images (processing_paligemma.py:31-50) on the GPU: PIL-exact BICUBIC resize
        of each decoded RGB image (PIL image or uint8 HWC array), x/255, (x-0.5)/0.5, CHW.
        Returns pixel_values (B, 3, size, size) float32 on the device."""
        import numpy as np
        S = int(size or self.cfgd["v_image"])
        out = torch.empty((len(images), 3, S, S), dtype=torch.float32, device=self.device)
        for i, im in enumerate(images):
            arr = np.asarray(im.convert("RGB") if hasattr(im, "convert") else im, dtype=np.uint8)
            if arr.ndim != 3 or arr.shape[2] != 3:
                raise ValueError(f"expected an RGB image (H, W, 3), got {arr.shape}")
            src = torch.from_numpy(np.array(arr, dtype=np.uint8, order="C")).to(self.device)
            N.check(self.lib.pgmi_preprocess(self.ctx, src.data_ptr(), arr.shape[0], arr.shape[1], S, S,
                                             out[i].data_ptr(), self._s()), "pgmi_preprocess")
        return out

    def project(self, feats: torch.Tensor) -> torch.Tensor:
        self._ready()
        f = feats.to(self.device, torch.bfloat16).contiguous()
        rows = f.numel() // f.shape[-1]
        out = torch.empty(f.shape[:-1] + (self.cfgd["projection_dim"],), dtype=torch.bfloat16, device=self.device)
        N.check(self.lib.pgmi_project(self.ctx, f.data_ptr(), rows, out.data_ptr(), self._s()), "pgmi_project")
        return out

    def embed(self, ids: torch.Tensor) -> torch.Tensor:
        self._ready()
        i = ids.to(self.device, torch.int64).contiguous()
        out = torch.empty(tuple(i.shape) + (self.cfgd["t_hidden"],), dtype=torch.bfloat16, device=self.device)
        # (a plain lookup into a fresh tensor: no engine workspace, so no wait for a lookahead in flight)
        N.check(self.lib.pgmi_embed(self.ctx, i.data_ptr(), i.numel(), out.data_ptr(), N.stream_handle(self.device)),
                "pgmi_embed")
        return out

    def lm_forward(self, kv: torch.Tensor, kv_start: int, positions, ids=None, image_feats=None, embeds=None,
                   logits_rows: int = 0) -> torch.Tensor:
        """GemmaForCausalLM.forward over merged embeddings (see pgmi.h).  Returns fp32 logits
        (B, L, V) (logits_rows 0) or (B, 1, V): logits_rows 1 keeps every row's final hidden state
        for final_hidden / lazy all-row logits; 2 needs only the last row's, so the last layer's
        post-attention work runs for the last row alone (the KV cache is written for every row)."""
        self._ready()
        if embeds is not None:
            e = embeds.to(self.device, torch.bfloat16).contiguous()
            B, L = e.shape[0], e.shape[1]
            idp, imgp, nimg = None, None, 0
        else:
            ids = ids.to(self.device, torch.int64).contiguous()
            B, L = ids.shape
            e = None
            idp = ids.data_ptr()
            if image_feats is not None:
                image_feats = image_feats.to(self.device, torch.bfloat16).contiguous()
                imgp, nimg = image_feats.data_ptr(), image_feats.numel() // image_feats.shape[-1]
            else:
                imgp, nimg = None, 0
        pos = torch.as_tensor(positions, dtype=torch.int64).cpu()
        pos = torch.broadcast_to(pos.reshape(pos.shape[0] if pos.dim() > 1 else 1, -1), (B, L)).contiguous()
        V = self.cfgd["t_vocab"]
        out = torch.empty((B, L if logits_rows == 0 else 1, V), dtype=torch.float32, device=self.device)
        N.check(self.lib.pgmi_lm_forward(self.ctx, idp, imgp, nimg, N.ptr(e), B, L, pos.data_ptr(), kv.data_ptr(),
                                         kv.shape[2], kv.shape[3], kv_start, out.data_ptr(), logits_rows, self._s()),
                "pgmi_lm_forward")
        return out

    def final_hidden(self, rows: int) -> torch.Tensor:
        """The final RMSNorm output of the last lm_forward's rows (B*L, hidden) bf16 (a copy)."""
        out = torch.empty((rows, self.cfgd["t_hidden"]), dtype=torch.bfloat16, device=self.device)
        N.check(self.lib.pgmi_lm_final_hidden(self.ctx, out.data_ptr(), rows, self._s()), "pgmi_lm_final_hidden")
        return out

    def lm_head(self, normed: torch.Tensor) -> torch.Tensor:
        """lm_head + .float() (modeling_gemma.py:417-418) over final-normed rows -> (rows, V) fp32."""
        self._ready()
        x = normed.to(self.device, torch.bfloat16).reshape(-1, normed.shape[-1]).contiguous()
        out = torch.empty((x.shape[0], self.cfgd["t_vocab"]), dtype=torch.float32, device=self.device)
        N.check(self.lib.pgmi_lm_head(self.ctx, x.data_ptr(), x.shape[0], out.data_ptr(), self._s()), "pgmi_lm_head")
        return out

    def decode(self, ids: torch.Tensor, kv: torch.Tensor, kv_len: int, position: int, logits: torch.Tensor = None,
               next_ids: torch.Tensor = None, graph: bool = False) -> torch.Tensor:
        """One KV-cached decode step for B sequences; returns logits (B, V) fp32."""
        self._ready()
        if ids.dtype is not torch.int64 or ids.device != self.device or not ids.is_contiguous():
            ids = ids.to(self.device, torch.int64).contiguous()
        ids = ids.view(-1)
        B = ids.numel()
        if logits is None:
            logits = torch.empty((B, self.cfgd["t_vocab"]), dtype=torch.float32, device=self.device)
        N.check(self.lib.pgmi_decode(self.ctx, ids.data_ptr(), B, kv.data_ptr(), kv.shape[2], kv.shape[3], kv_len,
                                     position, logits.data_ptr(), N.ptr(next_ids), int(graph), self._s()),
                "pgmi_decode")
        return logits

    def decode_steps(self, ids: torch.Tensor, kv: torch.Tensor, kv_len: int, position: int, n_steps: int,
                     logits: torch.Tensor = None, tokens: torch.Tensor = None, graph: bool = False) -> torch.Tensor:
        """n_steps greedy decode steps back to back (pgmi_decode_steps): ids (device int64, B) is read by the
        first step and receives every step's argmax in place; tokens (int64 (n_steps, B), optional) records
        them.  Returns the last step's logits (B, V) fp32."""
        self._ready()
        if ids.dtype is not torch.int64 or ids.device != self.device or not ids.is_contiguous():
            raise ValueError("decode_steps: ids must be a contiguous int64 tensor on the engine's device (updated in place)")
        B = ids.numel()
        if logits is None:
            logits = torch.empty((B, self.cfgd["t_vocab"]), dtype=torch.float32, device=self.device)
        if tokens is not None and (tokens.dtype is not torch.int64 or tokens.device != self.device
                                   or not tokens.is_contiguous() or tokens.numel() < n_steps * B):
            raise ValueError("decode_steps: tokens must be a contiguous int64 (n_steps, B) tensor on the device")
        N.check(self.lib.pgmi_decode_steps(self.ctx, ids.data_ptr(), B, kv.data_ptr(), kv.shape[2], kv.shape[3], kv_len,
                                           position, int(n_steps), logits.data_ptr(), N.ptr(tokens), int(graph),
                                           self._s()), "pgmi_decode_steps")
        return logits

    def decode_embeds(self, embeds: torch.Tensor, kv: torch.Tensor, kv_len: int, position: int,
                      logits: torch.Tensor = None, graph: bool = False) -> torch.Tensor:
        """The decode step over already-merged input rows (B, hidden) bf16 -- a caller's merge for
        a q_len == 1 step (pgmi_decode_embeds); returns logits (B, V) fp32."""
        self._ready()
        e = embeds.to(self.device, torch.bfloat16).reshape(-1, self.cfgd["t_hidden"]).contiguous()
        B = e.shape[0]
        if logits is None:
            logits = torch.empty((B, self.cfgd["t_vocab"]), dtype=torch.float32, device=self.device)
        N.check(self.lib.pgmi_decode_embeds(self.ctx, e.data_ptr(), B, kv.data_ptr(), kv.shape[2], kv.shape[3], kv_len,
                                            position, logits.data_ptr(), None, int(graph), self._s()),
                "pgmi_decode_embeds")
        return logits

    _POS_DTYPES = {torch.bfloat16: 0, torch.float32: 2, torch.int64: 10, torch.int32: 11, torch.float64: 12}

    def decode_embeds_dev(self, embeds: torch.Tensor, kv: torch.Tensor, kv_len: int, position: torch.Tensor,
                          mask: torch.Tensor = None, logits: torch.Tensor = None, graph: bool = False,
                          next_ids: torch.Tensor = None) -> torch.Tensor:
        """decode_embeds for one sequence with its rotary position and additive mask left on the device
        (a merge's outputs, read by the step itself: no host sync).  position: one element; mask:
        kv_len + 1 additive values (bf16 or fp32; other float dtypes are promoted to fp32)."""
        self._ready()
        e = embeds.to(self.device, torch.bfloat16).reshape(-1, self.cfgd["t_hidden"]).contiguous()
        if e.shape[0] != 1:
            raise ValueError("decode_embeds_dev: one sequence per step")
        p = position.to(self.device).reshape(-1)[:1]
        if p.dtype not in self._POS_DTYPES:
            p = p.to(torch.float64)
        p = p.contiguous()
        mp, mdt = None, N.DTYPE_BF16
        if mask is not None:
            m = mask.to(self.device).reshape(-1)
            if m.numel() != kv_len + 1:
                raise ValueError(f"mask has {m.numel()} keys, the step attends {kv_len + 1}")
            if m.dtype not in (torch.bfloat16, torch.float32):
                m = m.float()
            mp = m.contiguous()
            mdt = N.DTYPE_F32 if mp.dtype == torch.float32 else N.DTYPE_BF16
        if logits is None:
            logits = torch.empty((1, self.cfgd["t_vocab"]), dtype=torch.float32, device=self.device)
        N.check(self.lib.pgmi_decode_embeds_dev(self.ctx, e.data_ptr(), 1, kv.data_ptr(), kv.shape[2], kv.shape[3],
                                                kv_len, p.data_ptr(), self._POS_DTYPES[p.dtype], N.ptr(mp), mdt,
                                                mp.numel() if mp is not None else 0, logits.data_ptr(),
                                                N.ptr(next_ids), int(graph), self._s()),
                "pgmi_decode_embeds_dev")
        return logits

    def set_prefill_graph(self, on: bool) -> None:
        """Replay captured hipGraphs for repeated vision / language-model calls with the same buffers."""
        N.check(self.lib.pgmi_set_prefill_graph(self.ctx, int(bool(on))), "pgmi_set_prefill_graph")

    def set_decode_staged_norm(self, on: int) -> None:
        """Batched decode RMSNorm form: 0 once per row (default), 1 staged per projection, -1 default."""
        N.check(self.lib.pgmi_set_decode_staged_norm(self.ctx, int(on)), "pgmi_set_decode_staged_norm")

    def argmax(self, logits: torch.Tensor) -> torch.Tensor:
        l2 = logits.reshape(-1, logits.shape[-1]).contiguous()
        out = torch.empty(l2.shape[0], dtype=torch.int64, device=self.device)
        N.check(self.lib.pgmi_argmax(self.ctx, l2.data_ptr(), l2.shape[0], l2.shape[1], out.data_ptr(), self._s()))
        return out

    def sample_top_p(self, x: torch.Tensor, top_p: float, temperature: Optional[float] = None,
                     u: Optional[torch.Tensor] = None, generator: Optional[torch.Generator] = None,
                     return_kept_mass: bool = False):
        """Nucleus sampling on the device (inference.py:15-24).
        x (..., V) fp32: logits when `temperature` > 0 (softmax(x / T) of inference.py:65 is
        fused), else probabilities (the reference _sample_top_p's input).  u: uniforms in [0, 1)
        per row (default: torch.rand on the device with `generator`).  Returns int64 (rows,)."""
        x2 = x.reshape(-1, x.shape[-1]).to(self.device, torch.float32).contiguous()
        rows, V = x2.shape
        if u is None:
            u = torch.rand(rows, device=self.device, generator=generator)
        u = u.to(self.device, torch.float32).reshape(-1).contiguous()
        if u.numel() != rows:
            raise ValueError(f"need one uniform per row: {u.numel()} != {rows}")
        out = torch.empty(rows, dtype=torch.int64, device=self.device)
        kept = torch.empty(rows, dtype=torch.float32, device=self.device) if return_kept_mass else None
        T = float(temperature) if temperature is not None and temperature > 0 else 0.0
        N.check(self.lib.pgmi_sample_top_p(self.ctx, x2.data_ptr(), rows, V, T, float(top_p), u.data_ptr(),
                                           out.data_ptr(), N.ptr(kept), self._s()), "pgmi_sample_top_p")
        return (out, kept) if return_kept_mass else out

    # ------------------------------------------------------------------ batched greedy driver
    @torch.no_grad()
    def generate(self, input_ids: torch.Tensor, pixel_values: torch.Tensor, n_tokens: int, graph: bool = True,
                 kv: torch.Tensor = None, do_sample: bool = False, temperature: float = 0.8, top_p: float = 0.9,
                 generator: Optional[torch.Generator] = None, eos_token_id: Optional[int] = None,
                 pad_token_id: Optional[int] = None, sync_every: int = 16, return_lengths: bool = False):
        """Batched generation: prefill, then n_tokens-1 decode steps
        with the next token picked on the device -- greedy argmax, or with do_sample the
        temperature + top-p draw of inference.py:64-66 -- and no host sync per token.
        Positions follow inference.py's semantics (first decode position = L + 1,
        modeling_gemma.py:526).

        eos_token_id: the stop token of inference.py:51,70-71, applied per row on the device
        (pgmi_eos_update): a row keeps its eos and emits pad_token_id (default: eos) after it.
        The loop ends early once every row has stopped, checked every `sync_every` steps (one
        host read per check instead of the reference's `.item()` per token); the result is
        trimmed to the longest row.  return_lengths: also return int64 (B,) tokens per row up
        to and including its eos (the length of the reference's generated_tokens)."""
        ids = input_ids.to(self.device, torch.int64)
        B, L = ids.shape
        if kv is None:
            kv = self.new_kv(B, L + n_tokens + 1)
        feats = self.project(self.vision(pixel_values))
        logits = self.lm_forward(kv, 0, torch.arange(L).expand(B, L), ids=ids, image_feats=feats, logits_rows=2)
        toks = torch.empty((B, n_tokens), dtype=torch.int64, device=self.device)
        if do_sample:
            us = torch.rand((n_tokens, B), device=self.device, generator=generator)
            toks[:, 0] = self.sample_top_p(logits[:, 0], top_p, temperature, u=us[0])
        else:
            toks[:, 0] = self.argmax(logits[:, 0])
        step_logits = torch.empty((B, self.cfgd["t_vocab"]), dtype=torch.float32, device=self.device)
        nxt = torch.empty(B, dtype=torch.int64, device=self.device)
        cur = toks[:, 0].clone()
        stop = eos_token_id is not None
        if stop:
            pad = int(eos_token_id if pad_token_id is None else pad_token_id)
            finished = torch.zeros(B, dtype=torch.int32, device=self.device)
            alive = torch.empty(1, dtype=torch.int32, device=self.device)
            self._eos_update(cur, finished, int(eos_token_id), pad, alive)
            toks[:, 0] = cur
        n_done = n_tokens
        if not do_sample and not stop and graph and n_tokens > 1 and B >= self.GEN_MIN_BATCH:
            # greedy without a stop token: GEN_CHUNK steps per hipGraph launch (pgmi_decode_steps), the
            # argmax fed back in place and every step's token kept in a device record
            rec = torch.empty((self.GEN_CHUNK, B), dtype=torch.int64, device=self.device)
            t = 1
            while t < n_tokens:
                n = min(self.GEN_CHUNK, n_tokens - t)
                self.decode_steps(cur, kv, L + t - 1, L + t, n, logits=step_logits, tokens=rec, graph=graph)
                toks[:, t:t + n] = rec[:n].t()
                t += n
            return (toks, torch.full((B,), n_tokens, dtype=torch.int64, device=self.device)) if return_lengths else toks
        for t in range(1, n_tokens):
            if stop and (t - 1) % max(1, sync_every) == 0 and int(alive.item()) == 0:
                n_done = t
                break
            if do_sample:
                self.decode(cur, kv, L + t - 1, L + t, logits=step_logits, next_ids=nxt, graph=graph)
                cur.copy_(self.sample_top_p(step_logits, top_p, temperature, u=us[t]))
            else:  # greedy: the argmax is fed back in place (pgmi_decode with next_ids == ids)
                self.decode(cur, kv, L + t - 1, L + t, logits=step_logits, next_ids=cur, graph=graph)
            if stop:
                self._eos_update(cur, finished, int(eos_token_id), pad, alive)
            toks[:, t] = cur
        if not stop:
            return (toks, torch.full((B,), n_tokens, dtype=torch.int64, device=self.device)) if return_lengths else toks
        toks = toks[:, :n_done]
        hit = toks == int(eos_token_id)
        first = torch.where(hit.any(1), hit.int().argmax(1) + 1, torch.full_like(hit[:, 0], n_done, dtype=torch.int64))
        toks = toks[:, :int(first.max().item())].contiguous()
        return (toks, first.to(torch.int64)) if return_lengths else toks

    def _eos_update(self, next_ids: torch.Tensor, finished: torch.Tensor, eos: int, pad: int,
                    n_alive: Optional[torch.Tensor]) -> None:
        N.check(self.lib.pgmi_eos_update(self.ctx, next_ids.data_ptr(), finished.data_ptr(), next_ids.numel(), eos, pad,
                                         n_alive.data_ptr() if n_alive is not None else None, self._s()),
                "pgmi_eos_update")
