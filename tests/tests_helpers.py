"""Shared test helpers (no reference code: restatements of its preprocessing arithmetic)."""
import numpy as np


def pixels_from_u8(u8):
    """processing_paligemma.py:20-29,47-49 on the resized uint8 image: x/255 (float64 -> float32),
    (x - 0.5)/0.5 in float32, HWC -> CHW."""
    px = (u8 * (1 / 255.0)).astype(np.float32)
    return ((px - np.float32(0.5)) / np.float32(0.5)).transpose(2, 0, 1)
