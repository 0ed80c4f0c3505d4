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


def resample_plan(in_size: int, out_size: int):
    """Pillow's per-axis bicubic plan as computed by the library (clipvit_resample_plan):
    (bounds [out, 2] int32 = (first tap, tap count), kk [out, ksize] int32, 22 fraction bits).
    Host-only call (no GPU needed)."""
    import ctypes
    from . import _lib
    L = _lib.lib()
    ksize = ctypes.c_int(0)
    cap = out_size * (2 * (int(np.ceil(2.0 * max(in_size / out_size, 1.0))) + 1))
    bounds = np.zeros((out_size, 2), dtype=np.int32)
    kk = np.zeros(cap, dtype=np.int32)
    _lib.check(L.clipvit_resample_plan(
        in_size, out_size, ctypes.byref(ksize),
        bounds.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
        kk.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), cap))
    return bounds, kk[: out_size * ksize.value].reshape(out_size, ksize.value)


def preprocess_batch_gpu(images, n_px: int = 224, device=None, dtype: torch.dtype = torch.float32,
                         out: torch.Tensor | None = None) -> torch.Tensor:
    """_transform(n_px) of a list of RGB PIL images (or HWC uint8 arrays) on the GPU
    (clipvit_preprocess): the decoded bytes go to HBM once, resize + crop + normalise run as
    two HIP kernels on the current stream. Bit-identical to :func:`to_pixels` for fp32 output.
    Returns [B, 3, n_px, n_px] of ``dtype`` (float32 / bfloat16 / float16) on ``device``."""
    import ctypes
    from . import _lib
    codes = {torch.float32: _lib.F32, torch.bfloat16: _lib.BF16, torch.float16: _lib.F16}
    if dtype not in codes:
        raise ValueError(f"unsupported output dtype {dtype}")
    device = torch.device("cuda", 0) if device is None else torch.device(device)
    arrs = []
    for im in images:
        a = np.asarray(im.convert("RGB") if isinstance(im, Image.Image) else im, dtype=np.uint8)
        if a.ndim != 3 or a.shape[2] != 3:
            raise ValueError(f"expected an HWC RGB image, got shape {a.shape}")
        arrs.append(np.ascontiguousarray(a))
    B = len(arrs)
    if out is None:
        out = torch.empty((B, 3, n_px, n_px), dtype=dtype, device=device)
    if B == 0:
        return out
    if out.shape != (B, 3, n_px, n_px) or out.dtype != dtype or not out.is_contiguous():
        raise ValueError("out must be a contiguous [B, 3, n_px, n_px] tensor of dtype")
    table = (_lib.Image * B)()
    off = 0
    for i, a in enumerate(arrs):
        table[i].offset, table[i].height, table[i].width = off, a.shape[0], a.shape[1]
        off += a.nbytes
    host = torch.from_numpy(np.concatenate([a.reshape(-1) for a in arrs]))
    if torch.cuda.is_available():
        host = host.pin_memory()
    rgb = host.to(device, non_blocking=True)
    with torch.cuda.device(device):
        s = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
        _lib.check(_lib.lib().clipvit_preprocess(s, ctypes.c_void_p(rgb.data_ptr()), table, B, n_px,
                                                 codes[dtype], ctypes.c_void_p(out.data_ptr())))
    rgb.record_stream(torch.cuda.current_stream(device))
    return out
