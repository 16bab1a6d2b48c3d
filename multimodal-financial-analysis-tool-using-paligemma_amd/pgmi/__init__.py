"""pgmi -- MI355X-native (gfx950) PaliGemma-3B inference path.

Host-side Python over libpgmi.so (C ABI: include/pgmi.h).  The drop-in reference API
(modeling_gemma / modeling_siglip / processing_paligemma / utils) lives beside this package.
"""
from ._native import NativeError, lib  # noqa: F401
from .engine import Engine, config_dict  # noqa: F401

__version__ = "0.1.0"
