"""CPU precision study of the vision tower's number formats (test infrastructure).

Runs the oracle's ViT forward (oracle/clip_ref.py, fp32) with chosen tensors rounded to 16 bits
and reports the bench's parity metric (per image max|dlogit| / max|logit_ref|) and the feature
error against the all-fp32 forward, on the bench's inputs: seeded synthetic weights + merged LoRA
r=8, 8 seeded images, 437 random unit text rows.

Rows: weights + GEMM activations in fp16 / bf16 with the residual stream x in fp32 (what the HIP
path computes) or rounded to the 16-bit type after every residual add (what the reference's own
fp16 CUDA model does, and what a LayerNorm fold without fp32 x would need).

    python tests/precision_study.py ViT-B/32 [ViT-B/16 ...]
Measured (ViT-B/32): fp16/fp32-x 4.9e-4, fp16/fp16-x 1.49e-3, bf16/fp32-x 5.1e-3, bf16/bf16-x 1.1e-2.
"""
from __future__ import annotations

import math
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import amd_pkg  # noqa: E402

amd_pkg.load()
from interior_amd import config as C  # noqa: E402
from interior_amd.lora import synthetic_adapters  # noqa: E402
from interior_amd.weights import synthetic_state_dict  # noqa: E402
from oracle import clip_ref  # noqa: E402

SEGMENTS = [0, 40, 60, 359, 395, 425, 437]


def _r(t, dt):
    return t.to(dt).float() if dt is not None else t


def encode(sd, geo, px, wdt=None, adt=None, xdt=None):
    """clip_ref.encode_image with weights rounded to `wdt`, GEMM inputs / outputs to `adt` and the
    residual stream to `xdt` (None = fp32)."""
    p = "visual."
    B = px.shape[0]
    W = lambda k: _r(sd[k].float(), wdt)  # noqa: E731
    x = F.conv2d(_r(px.float(), adt), W(p + "conv1.weight"), stride=geo.patch_size)
    x = x.reshape(B, geo.width, -1).permute(0, 2, 1)
    x = torch.cat([sd[p + "class_embedding"].float().expand(B, 1, geo.width), x], 1) + sd[p + "positional_embedding"].float()
    x = _r(clip_ref.layer_norm(x, sd[p + "ln_pre.weight"], sd[p + "ln_pre.bias"]), xdt)
    for i in range(geo.layers):
        r = f"{p}transformer.resblocks.{i}."
        h = _r(clip_ref.layer_norm(x, sd[r + "ln_1.weight"], sd[r + "ln_1.bias"]), adt)
        Bn, N, D = h.shape
        H, dh = geo.heads, D // geo.heads
        qkv = _r(h @ W(r + "attn.in_proj_weight").t() + sd[r + "attn.in_proj_bias"].float(), adt)
        q, k, v = [t.reshape(Bn, N, H, dh).transpose(1, 2) for t in qkv.split(D, -1)]
        o = ((q @ k.transpose(-1, -2)) / math.sqrt(dh)).softmax(-1) @ v
        o = _r(o.transpose(1, 2).reshape(Bn, N, D), adt)
        y = _r(o @ W(r + "attn.out_proj.weight").t() + sd[r + "attn.out_proj.bias"].float(), adt)
        x = _r(x + y, xdt)
        h = _r(clip_ref.layer_norm(x, sd[r + "ln_2.weight"], sd[r + "ln_2.bias"]), adt)
        u = _r(clip_ref.quick_gelu(h @ W(r + "mlp.c_fc.weight").t() + sd[r + "mlp.c_fc.bias"].float()), adt)
        y = _r(u @ W(r + "mlp.c_proj.weight").t() + sd[r + "mlp.c_proj.bias"].float(), adt)
        x = _r(x + y, xdt)
    x = clip_ref.layer_norm(x[:, 0, :], sd[p + "ln_post.weight"], sd[p + "ln_post.bias"])
    return x @ sd[p + "proj"].float()


def study(name: str, images: int = 8):
    cfg = C.get_config(name)
    geo = clip_ref.GEOMETRIES[cfg.name]
    sd = synthetic_state_dict(cfg, 0)
    for ad in synthetic_adapters(cfg, rank=8):
        sd[ad.target] = clip_ref.merge_lora(sd[ad.target], torch.from_numpy(ad.A), torch.from_numpy(ad.B), ad.scaling)
    g = torch.Generator().manual_seed(0)
    px = torch.randn(images, 3, cfg.image_size, cfg.image_size, generator=g).clamp_(-1.8, 2.2)
    T = F.normalize(torch.randn(437, cfg.embed_dim, generator=g), dim=-1)
    rows = []
    with torch.no_grad():
        f0 = encode(sd, geo, px)
        _, l0, _, _, _ = clip_ref.head(f0, T, SEGMENTS)
        for tag, kw in [("fp16 weights+act, fp32 x", dict(wdt=torch.float16, adt=torch.float16)),
                        ("fp16 weights+act, fp16 x", dict(wdt=torch.float16, adt=torch.float16, xdt=torch.float16)),
                        ("bf16 weights+act, fp32 x", dict(wdt=torch.bfloat16, adt=torch.bfloat16)),
                        ("bf16 weights+act, bf16 x", dict(wdt=torch.bfloat16, adt=torch.bfloat16, xdt=torch.bfloat16))]:
            f = encode(sd, geo, px, **kw)
            _, lg, _, _, _ = clip_ref.head(f, T, SEGMENTS)
            e = float(((lg - l0).abs().amax(1) / l0.abs().amax(1)).max())
            fe = float(((f - f0).norm(dim=1) / f0.norm(dim=1)).max())
            rows.append((tag, e, fe))
            print(f"{name:9s} {tag:26s} logit rel {e:.2e}  feature rel {fe:.2e}", flush=True)
    return rows


if __name__ == "__main__":
    torch.set_num_threads(8)
    for n in sys.argv[1:] or ["ViT-B/32"]:
        study(n)
