"""ctypes binding of libpgmi.so (include/pgmi.h).

torch is imported first so that its bundled HIP runtime (libamdhip64.so.7) is the one the
library binds to -- one HIP runtime per process.  There is no fallback: if the shared
library is missing or fails to load, every product entry point raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the library load: shared HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
# PGMI_LIB_PATH: an alternative build of the same library, for same-box A/B measurements only
LIB_PATH = os.environ.get("PGMI_LIB_PATH") or os.path.join(_HERE, "libpgmi.so")

PGMI_OK, PGMI_E_ARG, PGMI_E_STATE, PGMI_E_HIP, PGMI_E_NOMEM = 0, -1, -2, -3, -4
DTYPE_BF16, DTYPE_F16, DTYPE_F32 = 0, 1, 2

EPI = {"store": 0, "bias": 1, "bias_gelu": 2, "bias_res": 3, "res": 4, "bias_pos": 5, "f32": 6, "geglu": 7}


class PgmiConfig(ctypes.Structure):
    _fields_ = [
        ("v_hidden", ctypes.c_int), ("v_intermediate", ctypes.c_int), ("v_layers", ctypes.c_int),
        ("v_heads", ctypes.c_int), ("v_channels", ctypes.c_int), ("v_image", ctypes.c_int),
        ("v_patch", ctypes.c_int), ("v_ln_eps", ctypes.c_float),
        ("t_vocab", ctypes.c_int), ("t_hidden", ctypes.c_int), ("t_intermediate", ctypes.c_int),
        ("t_layers", ctypes.c_int), ("t_heads", ctypes.c_int), ("t_kv_heads", ctypes.c_int),
        ("t_head_dim", ctypes.c_int), ("t_max_pos", ctypes.c_int), ("t_rms_eps", ctypes.c_float),
        ("t_rope_theta", ctypes.c_float), ("projection_dim", ctypes.c_int),
        ("image_token_index", ctypes.c_int64), ("pad_token_id", ctypes.c_int64),
        ("max_batch", ctypes.c_int), ("max_seq", ctypes.c_int), ("max_kv", ctypes.c_int),
    ]


vp, i32, i64, f32, u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_uint64

# name -> (restype, argtypes); the exported surface of include/pgmi.h
SIGNATURES = {
    "pgmi_last_error": (ctypes.c_char_p, []),
    "pgmi_version": (ctypes.c_char_p, []),
    "pgmi_create": (i32, [i32, ctypes.POINTER(PgmiConfig), ctypes.POINTER(vp)]),
    "pgmi_destroy": (i32, [vp]),
    "pgmi_weights_bytes": (i64, [vp]),
    "pgmi_weight_count": (i32, [vp]),
    "pgmi_weight_info": (i32, [vp, i32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(i64),
                               ctypes.POINTER(i64 * 4), ctypes.POINTER(i32)]),
    "pgmi_bind_weights": (i32, [vp, vp]),
    "pgmi_load_weight": (i32, [vp, ctypes.c_char_p, vp, i32, i32, vp]),
    "pgmi_fill_synthetic": (i32, [vp, ctypes.c_char_p, u64, f32, f32, vp]),
    "pgmi_load_safetensors": (i32, [vp, ctypes.c_char_p, ctypes.POINTER(i32), ctypes.POINTER(i32), vp]),
    "pgmi_safetensors_count": (i32, [ctypes.c_char_p, ctypes.POINTER(i32)]),
    "pgmi_safetensors_entry": (i32, [ctypes.c_char_p, i32, ctypes.c_char_p, i32, ctypes.POINTER(i32),
                                     ctypes.POINTER(i64 * 4), ctypes.POINTER(i32), ctypes.POINTER(i64),
                                     ctypes.POINTER(i64)]),
    "pgmi_synthetic_key": (u64, [ctypes.c_char_p, u64]),
    "pgmi_set_rope_inv_freq": (i32, [vp, ctypes.POINTER(f32)]),
    "pgmi_set_rope_table": (i32, [vp, vp, vp, i32]),
    "pgmi_prepare": (i32, [vp]),
    "pgmi_kv_bytes": (i64, [vp, i32, i32]),
    "pgmi_vision": (i32, [vp, vp, i32, i32, vp, vp]),
    "pgmi_project": (i32, [vp, vp, i32, vp, vp]),
    "pgmi_embed": (i32, [vp, vp, i32, vp, vp]),
    "pgmi_lm_forward": (i32, [vp, vp, vp, i32, vp, i32, i32, vp, vp, i32, i32, i32, vp, i32, vp]),
    "pgmi_decode": (i32, [vp, vp, i32, vp, i32, i32, i32, i32, vp, vp, i32, vp]),
    "pgmi_decode_steps": (i32, [vp, vp, i32, vp, i32, i32, i32, i32, i32, vp, vp, i32, vp]),
    "pgmi_decode_embeds": (i32, [vp, vp, i32, vp, i32, i32, i32, i32, vp, vp, i32, vp]),
    "pgmi_decode_embeds_dev": (i32, [vp, vp, i32, vp, i32, i32, i32, vp, i32, vp, i32, i64, vp, vp, i32, vp]),
    "pgmi_set_prefill_graph": (i32, [vp, i32]),
    "pgmi_set_decode_staged_norm": (i32, [vp, i32]),
    "pgmi_prefill_kernel": (i32, [vp, i32, i32, i32, vp]),
    "pgmi_debug_gemm_tiles": (i32, [i32, i32, i32, i32, i32, i32, vp, vp, vp]),
    "pgmi_prefill_probe": (i32, [vp, i32]),
    "pgmi_prefill_probe_times": (i32, [vp, ctypes.POINTER(f32), i32]),
    "pgmi_preprocess": (i32, [vp, vp, i32, i32, i32, i32, vp, vp]),
    "pgmi_argmax": (i32, [vp, vp, i32, i32, vp, vp]),
    "pgmi_lm_head": (i32, [vp, vp, i32, vp, vp]),
    "pgmi_lm_final_hidden": (i32, [vp, vp, i32, vp]),
    "pgmi_comm_unique_id": (i32, [vp]),
    "pgmi_comm_init": (i32, [i32, i32, i32, vp, ctypes.POINTER(vp)]),
    "pgmi_comm_destroy": (i32, [vp]),
    "pgmi_broadcast_weights": (i32, [vp, vp, i32, vp]),
    "pgmi_eos_update": (i32, [vp, vp, vp, i32, i64, i64, vp, vp]),
    "pgmi_decode_kernel": (i32, [vp, i32, i32, i32, vp]),
    "pgmi_tune_gemm": (i32, [i32, i32]),
    "pgmi_tune_gemm_shape": (i32, [i32, i32, i32, i32, i32, i32]),
    "pgmi_tune_attention": (i32, [i32]),
    "pgmi_sample_top_p": (i32, [vp, vp, i32, i32, f32, f32, vp, vp, vp, vp]),
    "pgmi_op_gemm": (i32, [vp, vp, vp, i32, i32, i32, i32, vp, vp, vp, vp]),
    "pgmi_op_gemm_strided": (i32, [vp, vp, i32, vp, i32, i32, i32, i32, i32, vp, vp, vp, vp]),
    "pgmi_op_rmsnorm": (i32, [vp, vp, vp, i32, i32, f32, vp, vp]),
    "pgmi_op_layernorm": (i32, [vp, vp, vp, vp, i32, i32, f32, vp, vp]),
    "pgmi_op_attention": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, f32, vp]),
    "pgmi_op_add": (i32, [vp, vp, vp, i64, vp, vp]),
    "pgmi_op_patch_embed": (i32, [vp, vp, i32, i32, i32, i32, i32, vp, vp, vp, i32, vp, vp]),
    "pgmi_op_gemv_res": (i32, [vp, vp, vp, i32, i32, i32, vp, vp]),
    "pgmi_op_attention_ex": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, f32, i32, vp, i32, i64, i64,
                                   i64, vp, vp]),
    "pgmi_op_rope": (i32, [vp, vp, vp, vp, i64, i32, i32, vp, vp]),
    "pgmi_op_scale": (i32, [vp, vp, f32, i64, vp, vp]),
}

_lib = None


class NativeError(RuntimeError):
    pass


def lib():
    """Load libpgmi.so (once).  Raises if it is missing: there is no CPU fallback."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(f"{LIB_PATH} not built: run `make -C csrc` or __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str = ""):
    if rc == PGMI_OK:
        return
    msg = lib().pgmi_last_error().decode(errors="replace")
    text = f"{what}: {msg}" if what else msg
    if rc == PGMI_E_ARG:
        raise ValueError(text)
    if rc == PGMI_E_STATE:
        raise AssertionError(text)
    if rc == PGMI_E_NOMEM:
        raise MemoryError(text)
    raise NativeError(text)


def ptr(t) -> "int | None":
    return None if t is None else t.data_ptr()


def safetensors_index(path: str):
    """[(name, dtype code, shape, begin, end)] of a safetensors file, parsed by libpgmi (no GPU)."""
    L = lib()
    n = ctypes.c_int()
    check(L.pgmi_safetensors_count(path.encode(), ctypes.byref(n)), path)
    out = []
    for i in range(n.value):
        name = ctypes.create_string_buffer(1024)
        dt, nd = ctypes.c_int(), ctypes.c_int()
        shape, b, e = (i64 * 4)(), ctypes.c_int64(), ctypes.c_int64()
        check(L.pgmi_safetensors_entry(path.encode(), i, name, 1024, ctypes.byref(dt), ctypes.byref(shape),
                                       ctypes.byref(nd), ctypes.byref(b), ctypes.byref(e)), path)
        out.append((name.value.decode(), dt.value, tuple(shape[j] for j in range(nd.value)), b.value, e.value))
    return out


def stream_handle(device=None) -> int:
    """The caller's current HIP stream on `device` (the raw handle, read without building a Stream object:
    this runs once per engine call, on the decode loop's host path)."""
    if isinstance(device, torch.device) and device.index is not None:
        return torch._C._cuda_getCurrentRawStream(device.index)
    return torch.cuda.current_stream(device).cuda_stream
