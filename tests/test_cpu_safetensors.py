"""libpgmi's safetensors header reader (csrc/safetensors_hdr.h) vs the safetensors library, on
files written here by safetensors itself -- no GPU: pgmi_safetensors_count / _entry only parse."""
import json
import os
import struct

import numpy as np
import pytest
from safetensors.numpy import save_file

from pgmi import _native as N


def _header(path):
    with open(path, "rb") as f:
        n = struct.unpack("<Q", f.read(8))[0]
        return json.loads(f.read(n))


def test_index_matches_the_safetensors_library(tmp_path):
    rng = np.random.default_rng(0)
    tensors = {
        "language_model.model.layers.0.mlp.gate_proj.weight": rng.standard_normal((32, 16)).astype(np.float32),
        "vision_tower.vision_model.post_layernorm.bias": rng.standard_normal(16).astype(np.float16),
        "multi_modal_projector.linear.weight": rng.standard_normal((2, 3, 4)).astype(np.float32),
        "scalar_like": np.array([1.0], np.float32),
        "i32_tensor": np.arange(6, dtype=np.int32),
    }
    p = str(tmp_path / "a.safetensors")
    save_file(tensors, p, metadata={"format": "pt", "note": "has \"quotes\" and , commas"})
    hdr = _header(p)
    idx = N.safetensors_index(p)
    assert len(idx) == len(tensors)
    codes = {"F32": N.DTYPE_F32, "F16": N.DTYPE_F16, "BF16": N.DTYPE_BF16}
    for name, dt, shape, b, e in idx:
        h = hdr[name]
        assert list(shape) == h["shape"]
        assert [b, e] == h["data_offsets"]
        assert dt == codes.get(h["dtype"], -1)


@pytest.mark.parametrize("blob", [b"", b"\x05\x00\x00\x00\x00\x00\x00\x00{}", b"\x02\x00\x00\x00\x00\x00\x00\x00[]",
                                  b"\x20\x00\x00\x00\x00\x00\x00\x00" + b'{"x": {"dtype": "F32", "shape": [1]}}   '])
def test_malformed_headers_raise_value_error(tmp_path, blob):
    p = str(tmp_path / "bad.safetensors")
    with open(p, "wb") as f:
        f.write(blob)
    with pytest.raises(ValueError):
        N.safetensors_index(p)


def test_out_of_range_offsets_raise(tmp_path):
    hdr = json.dumps({"w": {"dtype": "F32", "shape": [4], "data_offsets": [0, 1 << 20]}}).encode()
    p = str(tmp_path / "oob.safetensors")
    with open(p, "wb") as f:
        f.write(struct.pack("<Q", len(hdr)) + hdr + b"\x00" * 16)
    with pytest.raises(ValueError):
        N.safetensors_index(p)


def test_missing_file_raises():
    with pytest.raises(ValueError):
        N.safetensors_index(os.path.join("/nonexistent", "x.safetensors"))
