"""Vision-tower weights keyed by OpenAI-CLIP state-dict names.

Two sources:
* ``synthetic_state_dict`` — seeded CLIP-style random init (there is no network for the real
  OpenAI checkpoints here; BASELINE.json's configs are benchmarked on synthetic weights of the
  exact architecture);
* ``load_openai_checkpoint`` — a LOCAL OpenAI ``ViT-*.pt`` (TorchScript archive as downloaded
  by clip.load [3p]) or a plain state dict, for real-weight runs where such a file exists.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import torch

from .config import ViTConfig


def visual_names(cfg: ViTConfig) -> list[tuple[str, tuple[int, ...]]]:
    """Every ``visual.*`` tensor the encoder consumes, in a fixed generation order."""
    D, P = cfg.width, cfg.patch_size
    out = [("visual.conv1.weight", (D, 3, P, P)), ("visual.class_embedding", (D,)),
           ("visual.positional_embedding", (cfg.tokens, D)), ("visual.ln_pre.weight", (D,)),
           ("visual.ln_pre.bias", (D,))]
    for i in range(cfg.layers):
        r = f"visual.transformer.resblocks.{i}."
        out += [(r + "ln_1.weight", (D,)), (r + "ln_1.bias", (D,)),
                (r + "attn.in_proj_weight", (3 * D, D)), (r + "attn.in_proj_bias", (3 * D,)),
                (r + "attn.out_proj.weight", (D, D)), (r + "attn.out_proj.bias", (D,)),
                (r + "ln_2.weight", (D,)), (r + "ln_2.bias", (D,)),
                (r + "mlp.c_fc.weight", (4 * D, D)), (r + "mlp.c_fc.bias", (4 * D,)),
                (r + "mlp.c_proj.weight", (D, 4 * D)), (r + "mlp.c_proj.bias", (D,))]
    out += [("visual.ln_post.weight", (D,)), ("visual.ln_post.bias", (D,)),
            ("visual.proj", (D, cfg.embed_dim))]
    return out


def synthetic_state_dict(cfg: ViTConfig, seed: int = 0) -> dict[str, torch.Tensor]:
    """Seeded CLIP-style weights (torch.Generator on CPU: identical on every host with the
    same torch build). Linear/conv ~ N(0, 0.02); class/pos/proj ~ N(0, width^-0.5) as
    OpenAI's VisionTransformer.__init__ [3p]; LayerNorm gamma = 1 + N(0, 0.1), beta and biases
    ~ N(0, 0.02) so parity tests exercise every affine term."""
    g = torch.Generator().manual_seed(seed)
    scale = cfg.width ** -0.5
    sd = {}
    for name, shape in visual_names(cfg):
        if name.endswith(("class_embedding", "positional_embedding")) or name == "visual.proj":
            t = torch.randn(shape, generator=g) * scale
        elif ".ln_" in name or name.startswith("visual.ln_"):
            t = torch.randn(shape, generator=g) * (0.1 if name.endswith("weight") else 0.02)
            if name.endswith("weight"):
                t += 1.0
        elif name.endswith("bias"):
            t = torch.randn(shape, generator=g) * 0.02
        else:
            t = torch.randn(shape, generator=g) * 0.02
        sd[name] = t.float().contiguous()
    return sd


def text_names(tc) -> list[tuple[str, tuple[int, ...]]]:
    """OpenAI state-dict names/shapes of the text tower (CLIP [3p]: token_embedding,
    positional_embedding, transformer.resblocks.i.*, ln_final, text_projection)."""
    D = tc.width
    out = [("token_embedding.weight", (tc.vocab, D)), ("positional_embedding", (tc.context, D))]
    for i in range(tc.layers):
        r = f"transformer.resblocks.{i}."
        out += [(r + "ln_1.weight", (D,)), (r + "ln_1.bias", (D,)),
                (r + "attn.in_proj_weight", (3 * D, D)), (r + "attn.in_proj_bias", (3 * D,)),
                (r + "attn.out_proj.weight", (D, D)), (r + "attn.out_proj.bias", (D,)),
                (r + "ln_2.weight", (D,)), (r + "ln_2.bias", (D,)),
                (r + "mlp.c_fc.weight", (4 * D, D)), (r + "mlp.c_fc.bias", (4 * D,)),
                (r + "mlp.c_proj.weight", (D, 4 * D)), (r + "mlp.c_proj.bias", (D,))]
    out += [("ln_final.weight", (D,)), ("ln_final.bias", (D,)),
            ("text_projection", (D, tc.embed_dim))]
    return out


def synthetic_text_state_dict(tc, seed: int = 1) -> dict[str, torch.Tensor]:
    """Seeded text-tower weights in the scales of CLIP.initialize_parameters [3p]
    (token 0.02, positional 0.01, projection width^-0.5), LayerNorm/bias terms perturbed
    like synthetic_state_dict so parity exercises every affine term."""
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for name, shape in text_names(tc):
        if name == "positional_embedding":
            t = torch.randn(shape, generator=g) * 0.01
        elif name == "text_projection":
            t = torch.randn(shape, generator=g) * tc.width ** -0.5
        elif "ln_" in name:
            t = torch.randn(shape, generator=g) * (0.1 if name.endswith("weight") else 0.02)
            if name.endswith("weight"):
                t += 1.0
        else:
            t = torch.randn(shape, generator=g) * 0.02
        sd[name] = t.float().contiguous()
    return sd


def state_dict_checksum(sd: dict[str, torch.Tensor]) -> float:
    """Order-independent float64 checksum used to prove fixtures were regenerated identically."""
    return float(sum(float(v.double().abs().sum()) for v in sd.values()))


def load_openai_checkpoint(path: str | Path, text: bool = False) -> dict[str, torch.Tensor]:
    """Local OpenAI CLIP checkpoint -> fp32 ``visual.*`` state dict (``text=True``: the text
    tower's tensors instead, for TextEngine / InteriorAnalyzer(text_state_dict=...)).

    Tries a plain state dict with ``torch.load(weights_only=True)`` first; an OpenAI
    TorchScript archive (what clip.load downloads) is opened with ``torch.jit.load``, which
    only a user-supplied file may be given to (nothing shipped in the reference is loaded).
    """
    path = Path(path)
    try:
        sd = torch.load(path, map_location="cpu", weights_only=True)
        if hasattr(sd, "state_dict"):
            sd = sd.state_dict()
    except Exception:
        sd = torch.jit.load(str(path), map_location="cpu").state_dict()
    keep = (lambda k: not k.startswith("visual.") and k not in ("logit_scale", "input_resolution",
                                                                 "context_length", "vocab_size")) \
        if text else (lambda k: k.startswith("visual."))
    return {k: v.float().contiguous() for k, v in sd.items() if keep(k)}


def as_host_f32(t) -> np.ndarray:
    if isinstance(t, torch.Tensor):
        return np.ascontiguousarray(t.detach().to("cpu", torch.float32).numpy())
    return np.ascontiguousarray(np.asarray(t, dtype=np.float32))
