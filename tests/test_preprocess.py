"""GPU preprocessing (clipvit_preprocess, csrc/preprocess.hip) against CLIP's _transform [3p]
(main.py:201, main.py:438, main.py:489) as restated by preprocess.to_pixels / the oracle.

CPU: the library's resampling plans (clipvit_resample_plan, host code) driven through a
numpy restatement of the two integer passes reproduce PIL.Image.resize(BICUBIC) + crop
byte for byte, for up-, down- and identity-scaled axes. GPU: the kernels' output equals
to_pixels (PIL + numpy) bit for bit in fp32, and its bf16/fp16 rounding in 16-bit.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch
from PIL import Image

from interior_amd import preprocess as PP

PREC = 22
# (width, height): downscale, upscale, odd, identity axis, tall, extreme aspect, exact
SIZES = [(640, 480), (1024, 768), (100, 80), (333, 777), (224, 500), (500, 224), (224, 224),
         (1920, 1080), (225, 224), (57, 301), (3000, 2000)]


def _img(w, h, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    # smooth structure + noise so taps of both signs matter
    yy, xx = np.mgrid[0:h, 0:w]
    a = (a // 4 + (127 * (1 + np.sin(xx / 7.0) * np.cos(yy / 11.0)))[..., None] * 0.75).astype(np.uint8)
    return Image.fromarray(a, "RGB")


def _clip8(v):
    return np.where(v >= (1 << PREC << 8), 255, np.where(v <= 0, 0, v >> PREC)).astype(np.uint8)


def _pass(src, bounds, kk, idx, axis):
    """one Pillow 8-bit pass over `axis` for the output indices idx (int64 accumulation)."""
    src = np.moveaxis(src, axis, 0).astype(np.int64)
    out = np.empty((len(idx),) + src.shape[1:], dtype=np.uint8)
    for o, i in enumerate(idx):
        lo, n = bounds[i]
        acc = np.full(src.shape[1:], 1 << (PREC - 1), dtype=np.int64)
        for j in range(n):
            acc += src[lo + j] * int(kk[i, j])
        out[o] = _clip8(acc)
    return np.moveaxis(out, 0, axis)


def _emulate(img: Image.Image, n_px: int) -> np.ndarray:
    w, h = img.size
    nw, nh = PP.resize_size(w, h, n_px)
    top, left = int(round((nh - n_px) / 2.0)), int(round((nw - n_px) / 2.0))
    a = np.asarray(img)
    bh, kh = PP.resample_plan(w, nw)
    bv, kv = PP.resample_plan(h, nh)
    rows = range(bv[top][0], bv[top + n_px - 1][0] + bv[top + n_px - 1][1])
    inter = _pass(a[rows.start:rows.stop], bh, kh, range(left, left + n_px), axis=1)
    bv = bv.copy()
    bv[:, 0] -= rows.start
    return _pass(inter, bv, kv, range(top, top + n_px), axis=0)


def _pil(img: Image.Image, n_px: int) -> np.ndarray:
    w, h = img.size
    nw, nh = PP.resize_size(w, h, n_px)
    top, left = int(round((nh - n_px) / 2.0)), int(round((nw - n_px) / 2.0))
    return np.asarray(img.resize((nw, nh), Image.BICUBIC).crop((left, top, left + n_px, top + n_px)))


@pytest.mark.parametrize("w,h", SIZES[:8])
def test_plan_reproduces_pil_bytes(w, h):
    img = _img(w, h, w * 7 + h)
    assert np.array_equal(_emulate(img, 224), _pil(img, 224))


def test_plan_reproduces_pil_bytes_336_and_fixture_images(golden_dir):
    img = _img(800, 600, 3)
    assert np.array_equal(_emulate(img, 336), _pil(img, 336))
    for p in sorted((golden_dir / "images").glob("*.jpg"))[:2]:
        im = Image.open(p).convert("RGB")
        assert np.array_equal(_emulate(im, 224), _pil(im, 224))


def test_plan_identity_and_weights_sum():
    b, k = PP.resample_plan(224, 224)
    assert k.shape == (224, 1) and (k == 1 << PREC).all() and (b[:, 1] == 1).all()
    for i, o in [(640, 298), (100, 224), (3000, 224)]:
        b, k = PP.resample_plan(i, o)
        assert (np.abs(k.sum(axis=1) - (1 << PREC)) <= k.shape[1]).all()
        assert (b[:, 0] >= 0).all() and (b[:, 0] + b[:, 1] <= i).all()


def test_plan_bad_args_raise():
    from interior_amd import _lib
    with pytest.raises(_lib.ClipVitError):
        PP.resample_plan(0, 224)


@pytest.mark.gpu
def test_gpu_preprocess_bit_identical(gpu, golden_dir):
    imgs = [_img(w, h, i) for i, (w, h) in enumerate(SIZES)]
    imgs += [Image.open(p).convert("RGB") for p in sorted((golden_dir / "images").glob("*.jpg"))]
    ref = torch.stack([torch.from_numpy(PP.to_pixels(im, 224)) for im in imgs])
    got = PP.preprocess_batch_gpu(imgs, 224, gpu, torch.float32)
    torch.cuda.synchronize()
    got = got.cpu()
    assert torch.equal(got, ref), f"max diff {(got - ref).abs().max().item()}"
    for dt in (torch.float16, torch.bfloat16):
        g16 = PP.preprocess_batch_gpu(imgs, 224, gpu, dt).cpu()
        assert torch.equal(g16, ref.to(dt))


@pytest.mark.gpu
def test_gpu_preprocess_336_and_single(gpu):
    imgs = [_img(800, 600, 1), _img(337, 336, 2)]
    ref = torch.stack([torch.from_numpy(PP.to_pixels(im, 336)) for im in imgs])
    got = PP.preprocess_batch_gpu(imgs, 336, gpu).cpu()
    assert torch.equal(got, ref)
    one = PP.preprocess_batch_gpu([imgs[0]], 336, gpu).cpu()
    assert torch.equal(one[0], ref[0])


@pytest.mark.gpu
def test_gpu_preprocess_feeds_classify_like_host_path(gpu):
    """the GPU-preprocessed batch classifies exactly like the host-preprocessed one."""
    from interior_amd import config as C
    from interior_amd.engine import VisionEngine
    from interior_amd.weights import synthetic_state_dict
    cfg = C.VIT_B32
    eng = VisionEngine(cfg, gpu, "fp16", max_batch=4)
    eng.load_state_dict(synthetic_state_dict(cfg, 0))
    T = torch.nn.functional.normalize(torch.randn(437, cfg.embed_dim, generator=torch.Generator().manual_seed(1)), dim=-1)
    eng.set_text_features(T.numpy(), [0, 40, 60, 359, 395, 425, 437])
    imgs = [_img(640, 480, 5), _img(300, 900, 6), _img(224, 224, 7)]
    host = PP.preprocess_batch(imgs, 224, pin=False).to(gpu)
    dev = PP.preprocess_batch_gpu(imgs, 224, gpu)
    a = eng.classify(host).logits.cpu()
    b = eng.classify(dev).logits.cpu()
    eng.close()
    assert torch.equal(a, b)
