"""Host preprocessing that feeds the GPU path: CLIP's ``_transform(n_px)`` [3p]
(Resize(n_px, BICUBIC) -> CenterCrop(n_px) -> RGB -> ToTensor -> Normalize), as used at
main.py:201, main.py:438 and main.py:489. torchvision is not installed here, so the transform
is implemented with PIL + numpy (same PIL resampling call torchvision makes for PIL images).
Outside the timed metric (BASELINE.json measures synthetic, already-normalised pixels).
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch
from PIL import Image

MEAN = np.array([0.48145466, 0.4578275, 0.40821073], dtype=np.float32)
STD = np.array([0.26862954, 0.26130258, 0.27577711], dtype=np.float32)


def resize_size(w: int, h: int, n_px: int) -> tuple[int, int]:
    """torchvision Resize(int) on a PIL image: short side -> n_px, long side truncated."""
    if w <= h:
        return n_px, int(n_px * h / w)
    return int(n_px * w / h), n_px


def to_pixels(img: Image.Image, n_px: int = 224) -> np.ndarray:
    """PIL image -> CLIP-normalised float32 [3, n_px, n_px]."""
    nw, nh = resize_size(img.size[0], img.size[1], n_px)
    img = img.resize((nw, nh), Image.BICUBIC)
    top, left = int(round((nh - n_px) / 2.0)), int(round((nw - n_px) / 2.0))
    img = img.crop((left, top, left + n_px, top + n_px)).convert("RGB")
    a = np.asarray(img, dtype=np.float32) / 255.0  # ToTensor: div(255), then Normalize
    a = (a - MEAN) / STD
    return np.ascontiguousarray(a.transpose(2, 0, 1))


def preprocess(img: Image.Image, n_px: int = 224) -> torch.Tensor:
    return torch.from_numpy(to_pixels(img, n_px))


def preprocess_batch(images, n_px: int = 224, workers: int = 8, pin: bool = True) -> torch.Tensor:
    """Preprocess a list of PIL images in a thread pool (PIL releases the GIL in resize) into
    one pinned host tensor, ready for a non-blocking H2D copy."""
    with ThreadPoolExecutor(max_workers=max(1, workers)) as ex:
        arrs = list(ex.map(lambda im: to_pixels(im, n_px), images))
    out = torch.from_numpy(np.stack(arrs)) if arrs else torch.empty((0, 3, n_px, n_px))
    return out.pin_memory() if pin and torch.cuda.is_available() and len(arrs) else out


def load_image(path_or_url: str, timeout: int = 30):
    """main.py:119-128 / main.py:324-327: local path or http(s) URL -> RGB PIL image."""
    if path_or_url.startswith("http"):
        import requests
        from io import BytesIO
        r = requests.get(path_or_url, timeout=timeout)
        r.raise_for_status()
        return Image.open(BytesIO(r.content)).convert("RGB")
    return Image.open(path_or_url).convert("RGB")
