"""ORACLE — test infrastructure only. CPU fp32 restatement of the reference hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline. The product path
(``ai-interior-image-classifier_amd``) never imports it and has no CPU fallback.

What it restates (reference = M1A5TO/AI-interior-image-classifier, mounted read-only):

* ``encode_image``: OpenAI-CLIP ``VisionTransformer.forward`` [third-party ``clip`` package,
  unpinned in python-worker/requirements.txt:3,17, not vendored], called at main.py:204,
  main.py:444, main.py:503::

      x = conv1(pixels)                              # no bias, stride = kernel = patch
      x = cat([class_embedding, x]) + positional_embedding
      x = ln_pre(x)                                  # CLIP LayerNorm: fp32, eps 1e-5
      for each block: x = x + attn(ln_1(x)); x = x + mlp(ln_2(x))
          attn = nn.MultiheadAttention (packed in_proj, scale 1/sqrt(64), no mask)
          mlp  = c_fc -> QuickGELU (x * sigmoid(1.702 x)) -> c_proj
      f = ln_post(x[:, 0]) @ proj

* the head (main.py:205-217 detector, main.py:445-459 batch, main.py:504-509 single):
  ``f / ||f||`` -> ``softmax(100 * f @ T^T)`` per label segment -> ``topk(min(5, n))``.
* LoRA merge (main.py:19-31): ``linear(x) + (x @ A @ B) * (alpha / r)``
  == ``x @ (W + s * (A @ B)^T)^T + b``.
* the detector decision (main.py:207-222).

Parity status: the reference holds no golden vectors for this path, and
the real ``clip`` package/weights are absent offline. The restatement is pinned by
(1) ``transformers`` CLIPVisionModelWithProjection (independent implementation, same
architecture) on identical seeded weights, (2) torch's own ``nn.MultiheadAttention`` via the
module mirror in ``clip_module.py``, and (3) the reference's own harness code (main.py
``CachedInteriorAnalyzer``, ``replace_linears_with_lora``, ``load_lora_weights_to_model``)
run on top of the mirror, whose outputs are committed under ``tests/golden/``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F


@dataclass(frozen=True)
class Geometry:
    image_size: int
    patch_size: int
    width: int
    layers: int
    heads: int
    embed_dim: int

    @property
    def grid(self) -> int:
        return self.image_size // self.patch_size

    @property
    def tokens(self) -> int:
        return self.grid * self.grid + 1


GEOMETRIES = {
    # clip.load names -> VisionTransformer(input_resolution, patch_size, width, layers, heads, output_dim)
    "ViT-B/32": Geometry(224, 32, 768, 12, 12, 512),
    "ViT-B/16": Geometry(224, 16, 768, 12, 12, 512),
    "ViT-L/14": Geometry(224, 14, 1024, 24, 16, 768),
    "ViT-L/14@336px": Geometry(336, 14, 1024, 24, 16, 768),
}


def layer_norm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """CLIP ``LayerNorm``: upcast to fp32, torch layer_norm, eps 1e-5 [3p]."""
    return F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), 1e-5)


def quick_gelu(x: torch.Tensor) -> torch.Tensor:
    """CLIP ``QuickGELU`` [3p]: x * sigmoid(1.702 x)."""
    return x * torch.sigmoid(1.702 * x)


def attention(x: torch.Tensor, in_w, in_b, out_w, out_b, heads: int, mask=None) -> torch.Tensor:
    """nn.MultiheadAttention(x, x, x, need_weights=False, attn_mask=mask) restated for
    batch-first x [B,N,D] (mask: additive [N,N], CLIP's text tower passes -inf above the
    diagonal)."""
    B, N, D = x.shape
    dh = D // heads
    qkv = x @ in_w.t() + in_b
    q, k, v = qkv.split(D, dim=-1)
    q = q.reshape(B, N, heads, dh).transpose(1, 2)
    k = k.reshape(B, N, heads, dh).transpose(1, 2)
    v = v.reshape(B, N, heads, dh).transpose(1, 2)
    s = (q @ k.transpose(-1, -2)) / math.sqrt(dh)
    if mask is not None:
        s = s + mask
    o = s.softmax(dim=-1) @ v
    o = o.transpose(1, 2).reshape(B, N, D)
    return o @ out_w.t() + out_b


def encode_image(sd: dict, geo: Geometry, pixels: torch.Tensor) -> torch.Tensor:
    """``model.encode_image(pixels)`` in fp32 on CPU -> [B, embed_dim] (not normalised)."""
    p = "visual."
    x = pixels.float()
    B = x.shape[0]
    w = sd[p + "conv1.weight"].float()
    x = F.conv2d(x, w, stride=geo.patch_size)                  # [B, D, G, G]
    x = x.reshape(B, geo.width, -1).permute(0, 2, 1)            # [B, G*G, D]
    cls = sd[p + "class_embedding"].float().expand(B, 1, geo.width)
    x = torch.cat([cls, x], dim=1) + sd[p + "positional_embedding"].float()
    x = layer_norm(x, sd[p + "ln_pre.weight"], sd[p + "ln_pre.bias"])
    for i in range(geo.layers):
        r = f"{p}transformer.resblocks.{i}."
        h = layer_norm(x, sd[r + "ln_1.weight"], sd[r + "ln_1.bias"])
        x = x + attention(h, sd[r + "attn.in_proj_weight"].float(), sd[r + "attn.in_proj_bias"].float(),
                          sd[r + "attn.out_proj.weight"].float(), sd[r + "attn.out_proj.bias"].float(),
                          geo.heads)
        h = layer_norm(x, sd[r + "ln_2.weight"], sd[r + "ln_2.bias"])
        h = quick_gelu(h @ sd[r + "mlp.c_fc.weight"].float().t() + sd[r + "mlp.c_fc.bias"].float())
        x = x + (h @ sd[r + "mlp.c_proj.weight"].float().t() + sd[r + "mlp.c_proj.bias"].float())
    x = layer_norm(x[:, 0, :], sd[p + "ln_post.weight"], sd[p + "ln_post.bias"])
    return x @ sd[p + "proj"].float()


def encode_text(sd: dict, tokens, heads: int = 8) -> torch.Tensor:
    """``model.encode_text(tokens)`` [3p] (CLIP.encode_text; main.py:181, main.py:308) in fp32:

        x = token_embedding[tokens] + positional_embedding
        for each block (causal mask = -inf above the diagonal, CLIP.build_attention_mask):
            x = x + attn(ln_1(x), mask); x = x + mlp(ln_2(x))
        f = ln_final(x)[arange(B), tokens.argmax(-1)] @ text_projection
    -> [B, embed_dim], not normalised (main.py:182 / main.py:309 normalise)."""
    ids = torch.as_tensor(np.asarray(tokens)).long()
    x = sd["token_embedding.weight"].float()[ids] + sd["positional_embedding"].float()[: ids.shape[1]]
    n = ids.shape[1]
    mask = torch.full((n, n), float("-inf")).triu_(1)
    layers = sum(1 for k in sd if k.startswith("transformer.resblocks.") and k.endswith(".ln_1.weight"))
    for i in range(layers):
        r = f"transformer.resblocks.{i}."
        h = layer_norm(x, sd[r + "ln_1.weight"], sd[r + "ln_1.bias"])
        x = x + attention(h, sd[r + "attn.in_proj_weight"].float(), sd[r + "attn.in_proj_bias"].float(),
                          sd[r + "attn.out_proj.weight"].float(), sd[r + "attn.out_proj.bias"].float(),
                          heads, mask)
        h = layer_norm(x, sd[r + "ln_2.weight"], sd[r + "ln_2.bias"])
        h = quick_gelu(h @ sd[r + "mlp.c_fc.weight"].float().t() + sd[r + "mlp.c_fc.bias"].float())
        x = x + (h @ sd[r + "mlp.c_proj.weight"].float().t() + sd[r + "mlp.c_proj.bias"].float())
    x = layer_norm(x, sd["ln_final.weight"], sd["ln_final.bias"])
    return x[torch.arange(x.shape[0]), ids.argmax(dim=-1)] @ sd["text_projection"].float()


def merge_lora(W: torch.Tensor, A: torch.Tensor, B: torch.Tensor, scaling: float) -> torch.Tensor:
    """LoRALayer (main.py:19-31) folded into the Linear weight: W + s * (A @ B)^T."""
    return W.float() + scaling * (A.float() @ B.float()).t()


def head(f: torch.Tensor, T: torch.Tensor, seg_offsets: list[int]):
    """main.py:205-211 / 445-457 / 504-507 for every segment at once.

    Returns (f_hat [B,E], logits [B,C], probs [B,C], top_idx [B,nseg,5], top_prob [B,nseg,5])
    with top_idx relative to the segment start and -1 padding where the segment has < 5 labels.
    """
    f = f.float()
    f_hat = f / f.norm(dim=-1, keepdim=True)
    logits = 100.0 * f_hat @ T.float().t()
    B = f.shape[0]
    nseg = len(seg_offsets) - 1
    probs = torch.empty_like(logits)
    top_idx = torch.full((B, nseg, 5), -1, dtype=torch.int32)
    top_prob = torch.zeros((B, nseg, 5), dtype=torch.float32)
    for s in range(nseg):
        a, b = seg_offsets[s], seg_offsets[s + 1]
        p = logits[:, a:b].softmax(dim=-1)
        probs[:, a:b] = p
        k = min(5, b - a)
        v, i = p.topk(k, dim=-1)
        top_idx[:, s, :k] = i.int()
        top_prob[:, s, :k] = v
    return f_hat, logits, probs, top_idx, top_prob


def detector_decision(det_probs: torch.Tensor, categories: list[str], n_interior: int = 11,
                      threshold: float = 0.3):
    """InteriorImageDetector.is_interior_image (main.py:207-222) for one image's 40 probs."""
    top_conf, top_i = det_probs.topk(1)
    interior = det_probs[:n_interior].sum().item()
    non_interior = det_probs[n_interior:].sum().item()
    is_int = interior > non_interior and top_conf.item() > threshold
    return is_int, interior, categories[top_i.item()]


# ---------------------------------------------------------------------------------------
# preprocess: clip._transform(n_px) [3p] = Resize(n_px, BICUBIC) -> CenterCrop(n_px) ->
# convert("RGB") -> ToTensor -> Normalize(mean, std); used at main.py:201, 438, 489.
CLIP_MEAN = np.array([0.48145466, 0.4578275, 0.40821073], dtype=np.float32)
CLIP_STD = np.array([0.26862954, 0.26130258, 0.27577711], dtype=np.float32)


def preprocess(img, n_px: int = 224) -> torch.Tensor:
    """Restatement of the torchvision transforms CLIP composes (numpy + PIL only)."""
    from PIL import Image

    w, h = img.size
    short, long = (w, h) if w <= h else (h, w)
    new_short, new_long = n_px, int(n_px * long / short)
    nw, nh = (new_short, new_long) if w <= h else (new_long, new_short)
    img = img.resize((nw, nh), Image.BICUBIC)
    top = int(round((nh - n_px) / 2.0))
    left = int(round((nw - n_px) / 2.0))
    img = img.crop((left, top, left + n_px, top + n_px)).convert("RGB")
    a = np.asarray(img, dtype=np.float32) / 255.0          # HWC
    a = (a - CLIP_MEAN) / CLIP_STD
    return torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))
