"""Drop-in for the reference's processing_paligemma.py (image preprocessing + prompt glue).

Same functions, constants and PaliGemmaProcessor API as /root/reference/processing_paligemma.py
(:1-117): BICUBIC resize (PIL), x/255, (x - 0.5)/0.5, HWC -> CHW, and the
"<image>" * N + bos + prompt + "\\n" prompt layout; tests/test_cpu_host.py pins it to the
reference's own outputs on the committed COCO images.  `process_images_gpu` (and
PaliGemmaProcessor(..., engine=...)) runs the same steps on the MI355X through libpgmi
(pgmi_preprocess: PIL-exact resample; tests/test_gpu_preprocess.py).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Tuple, Union

import numpy as np
import torch
from PIL import Image

IMAGENET_STANDARD_MEAN = [0.5, 0.5, 0.5]
IMAGENET_STANDARD_STD = [0.5, 0.5, 0.5]


def add_image_tokens_to_prompt(prefix_prompt, bos_token, image_seq_len, image_token):
    """processing_paligemma.py:10-11."""
    return f"{image_token * image_seq_len}{bos_token}{prefix_prompt}\n"


def resize(image: Image.Image, size: Tuple[int, int], resample=None, reducing_gap: Optional[int] = None):
    """processing_paligemma.py:13-18 (PIL takes (width, height))."""
    height, width = size
    return image.resize((width, height), resample=resample, reducing_gap=reducing_gap)


def rescale(image: np.ndarray, scale: float, dtype: np.dtype = np.float32) -> np.ndarray:
    """processing_paligemma.py:20-23: multiply (float64 for a uint8 input) then cast."""
    return (image * scale).astype(dtype)


def normalize(image: np.ndarray, mean: Union[float, Iterable[float]], std: Union[float, Iterable[float]]) -> np.ndarray:
    """processing_paligemma.py:25-29, in the image's dtype."""
    mean = np.array(mean, dtype=image.dtype)
    std = np.array(std, dtype=image.dtype)
    return (image - mean) / std


def process_images(images: List[Image.Image], size: Dict[str, int] = None, resample=None,
                   rescale_factor: float = None, image_mean=None, image_std=None) -> List[np.ndarray]:
    """processing_paligemma.py:31-50: resize -> array -> rescale -> normalize -> CHW."""
    height, width = size[0], size[1]
    out = []
    for image in images:
        arr = np.array(resize(image=image, size=(height, width), resample=resample))
        arr = normalize(rescale(arr, scale=rescale_factor), mean=image_mean, std=image_std)
        out.append(arr.transpose(2, 0, 1))
    return out


def process_images_gpu(images: List[Image.Image], size: Tuple[int, int], engine) -> torch.Tensor:
    """process_images with BICUBIC / 1/255 / IMAGENET_STANDARD mean+std on the GPU (the
    reference's only configuration, processing_paligemma.py:82-89): (B, 3, H, W) float32 on
    the engine's device, bit-identical to torch.tensor(np.stack(process_images(...)))."""
    if size[0] != size[1]:
        raise ValueError("square outputs only (PaliGemma image_size)")
    return engine.preprocess(images, size=size[0])


class PaliGemmaProcessor:
    """processing_paligemma.py:52-117.  engine (optional, not in the reference): a pgmi.Engine
    whose GPU preprocessing produces pixel_values (on the device) instead of PIL + numpy."""

    IMAGE_TOKEN = "<image>"

    def __init__(self, tokenizer, num_image_tokens: int, image_size: int, engine=None):
        super().__init__()
        self.engine = engine
        self.image_seq_length = num_image_tokens
        self.image_size = image_size
        tokenizer.add_special_tokens({"additional_special_tokens": [self.IMAGE_TOKEN]})
        extra = [f"<loc{i:04d}>" for i in range(1024)] + [f"<seg{i:03d}>" for i in range(128)]
        tokenizer.add_tokens(extra)
        self.image_token_id = tokenizer.convert_tokens_to_ids(self.IMAGE_TOKEN)
        tokenizer.add_bos_token = False
        tokenizer.add_eos_token = False
        self.tokenizer = tokenizer

    def __call__(self, text: List[str], images: List[Image.Image], padding: str = "longest",
                 truncation: bool = True) -> dict:
        assert len(images) == 1 and len(text) == 1, f"Received {len(images)} images for {len(text)} prompts."
        if self.engine is not None:
            pixel_values = process_images_gpu(images, (self.image_size, self.image_size), self.engine)
        else:
            pixel_values = process_images(images, size=(self.image_size, self.image_size),
                                          resample=Image.Resampling.BICUBIC, rescale_factor=1 / 255.0,
                                          image_mean=IMAGENET_STANDARD_MEAN, image_std=IMAGENET_STANDARD_STD)
            pixel_values = torch.tensor(np.stack(pixel_values, axis=0))
        input_strings = [add_image_tokens_to_prompt(prefix_prompt=p, bos_token=self.tokenizer.bos_token,
                                                    image_seq_len=self.image_seq_length, image_token=self.IMAGE_TOKEN)
                         for p in text]
        inputs = self.tokenizer(input_strings, return_tensors="pt", padding=padding, truncation=truncation)
        return {"pixel_values": pixel_values, **inputs}
