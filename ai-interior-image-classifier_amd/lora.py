"""LoRA for the vision tower: the reference's checkpoint format and binding rule, merged at
load time instead of run as a side branch.

Reference behaviour restated (main.py:19-113):
* ``LoRALayer``: ``lora_A [in, r] ~ 0.02 N``, ``lora_B [r, out] = 0``, ``scaling = alpha / r``,
  ``forward = (x @ A @ B) * scaling`` (main.py:19-31).
* ``replace_linears_with_lora`` wraps EVERY ``nn.Linear`` reached through ``named_children``
  (main.py:62-74). On OpenAI CLIP that is ``attn.out_proj``, ``mlp.c_fc`` and ``mlp.c_proj`` of
  every residual block of both towers: 72 Linears for the 12+12-block B models. ``attn``'s packed
  ``in_proj_weight`` is a bare Parameter and is never wrapped.
* The ``attn.out_proj`` wrapper is dead code: nn.MultiheadAttention hands
  ``out_proj.weight/.bias`` straight to F.multi_head_attention_forward, and LoRALinear only
  proxies ``.weight``/``.bias`` (main.py:45-51), so its LoRA branch never runs.
* ``load_lora_weights_to_model`` binds each model parameter whose name contains ``'lora'``:
  exact key match, else the FIRST checkpoint key ``k`` (checkpoint order) with
  ``k.endswith(name) or name.endswith(k)`` (main.py:93-109); unmatched parameters keep their
  init, i.e. ``lora_B = 0`` => zero delta. It prints ``loaded`` and ``missing`` counts.

The shipped ``comprehensive_lora*.pth`` hold only text-tower ``mlp.{c_fc,c_proj}`` adapters
(keys ``clip_model.transformer.resblocks.{i}.mlp.*.lora.lora_{A,B}``), so with the reference's
rule every vision adapter stays zero (48 loaded / 96 missing). ``merge_items`` turns whatever
binds into ``clipvit_load_lora`` items: ``W' = W + scaling * (A @ B)^T``.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from pathlib import Path

import numpy as np
import torch

from .config import ViTConfig

WRAPPED_LEAVES = ("attn.out_proj", "mlp.c_fc", "mlp.c_proj")  # nn.Linear children per block
LIVE_VISION_LEAVES = ("mlp.c_fc", "mlp.c_proj")  # out_proj LoRA never executes (see header)
TARGET_WEIGHT = {"attn.out_proj": "attn.out_proj.weight", "mlp.c_fc": "mlp.c_fc.weight",
                 "mlp.c_proj": "mlp.c_proj.weight", "attn.in_proj": "attn.in_proj_weight"}


@dataclass
class LoraAdapter:
    target: str          # OpenAI name of the Linear weight, e.g. visual...mlp.c_fc.weight
    A: np.ndarray        # [in, r] fp32
    B: np.ndarray        # [r, out] fp32
    scaling: float

    @property
    def rank(self) -> int:
        return int(self.A.shape[1])


def load_lora_checkpoint(path: str | Path) -> "OrderedDict[str, torch.Tensor]":
    """``comprehensive_lora*.pth``: an OrderedDict of fp32 tensors (torch zip). Loaded with
    ``weights_only=True`` only — nothing in the file is executed."""
    path = Path(path)
    if not path.exists():
        raise FileNotFoundError(str(path))  # main.py:87-88
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    return OrderedDict((k, v) for k, v in ckpt.items())


def wrapped_lora_param_names(vision_layers: int = 12, text_layers: int = 12) -> list[str]:
    """Names ``replace_linears_with_lora`` creates on OpenAI CLIP, in named_parameters order
    (visual tower first, as CLIP registers ``visual`` before ``transformer``)."""
    names = []
    for prefix, n in (("visual.transformer", vision_layers), ("transformer", text_layers)):
        for i in range(n):
            for leaf in WRAPPED_LEAVES:
                base = f"{prefix}.resblocks.{i}.{leaf}.lora."
                names += [base + "lora_A", base + "lora_B"]
    return names


def bind(ckpt: "OrderedDict[str, torch.Tensor]", param_names: list[str]):
    """The reference matching rule (main.py:93-109). Returns ({name: tensor}, missing)."""
    keys = list(ckpt.keys())
    bound, missing = {}, []
    for name in param_names:
        if "lora" not in name:
            continue
        if name in ckpt:
            bound[name] = ckpt[name]
            continue
        hit = next((k for k in keys if k.endswith(name) or name.endswith(k)), None)
        if hit is not None:
            bound[name] = ckpt[hit]
        else:
            missing.append(name)
    return bound, missing


def vision_adapters_from_checkpoint(ckpt, cfg: ViTConfig, rank: int = 4, alpha: float = 8.0,
                                    text_layers: int = 12, live_only: bool = True):
    """Apply the reference binding to a checkpoint and return the vision adapters that change
    the image path (both A and B bound, B non-zero), plus (loaded, missing) like main.py:110.
    ``live_only`` drops ``attn.out_proj`` adapters, which the reference never executes."""
    names = wrapped_lora_param_names(cfg.layers, text_layers)
    bound, missing = bind(ckpt, names)
    scaling = alpha / rank  # main.py:28
    items = []
    leaves = LIVE_VISION_LEAVES if live_only else WRAPPED_LEAVES
    for i in range(cfg.layers):
        for leaf in leaves:
            base = f"visual.transformer.resblocks.{i}.{leaf}.lora."
            A, B = bound.get(base + "lora_A"), bound.get(base + "lora_B")
            if A is None or B is None or not torch.any(B != 0):
                continue  # unbound lora_B keeps its zero init: delta = 0
            items.append(LoraAdapter(f"visual.transformer.resblocks.{i}.{TARGET_WEIGHT[leaf]}",
                                     np.ascontiguousarray(A.float().numpy()),
                                     np.ascontiguousarray(B.float().numpy()), scaling))
    return items, len(bound), missing


def text_adapters_from_checkpoint(ckpt, text_layers: int = 12, rank: int = 4, alpha: float = 8.0,
                                  vision_layers: int = 12):
    """The same binding (main.py:93-109) for the TEXT tower, where the shipped checkpoints'
    adapters live (``clip_model.transformer.resblocks.{i}.mlp.{c_fc,c_proj}``): merge items
    for ``clipvit_text_load_lora`` (targets ``transformer.resblocks.{i}.mlp.*.weight``), plus
    (loaded, missing). ``attn.out_proj`` adapters are dropped (never executed, see header)."""
    names = wrapped_lora_param_names(vision_layers, text_layers)
    bound, missing = bind(ckpt, names)
    scaling = alpha / rank  # main.py:28
    items = []
    for i in range(text_layers):
        for leaf in LIVE_VISION_LEAVES:
            base = f"transformer.resblocks.{i}.{leaf}.lora."
            A, B = bound.get(base + "lora_A"), bound.get(base + "lora_B")
            if A is None or B is None or not torch.any(B != 0):
                continue
            items.append(LoraAdapter(f"transformer.resblocks.{i}.{TARGET_WEIGHT[leaf]}",
                                     np.ascontiguousarray(A.float().numpy()),
                                     np.ascontiguousarray(B.float().numpy()), scaling))
    return items, len(bound), missing


def synthetic_adapters(cfg: ViTConfig, rank: int = 8, alpha: float | None = None, seed: int = 1,
                       leaves=("attn.in_proj", "attn.out_proj", "mlp.c_fc", "mlp.c_proj")):
    """BASELINE.json's 'ViT-B/32 + LoRA r=8' (and r=16 for L/14): seeded adapters on every
    vision Linear including the fused QKV projection, alpha = 2 r by the reference's convention
    (main.py:20, main.py:522). A ~ N(0, 0.02), B ~ N(0, 0.01) so the merge is exercised."""
    alpha = 2.0 * rank if alpha is None else alpha
    g = torch.Generator().manual_seed(seed)
    D = cfg.width
    dims = {"attn.in_proj": (D, 3 * D), "attn.out_proj": (D, D), "mlp.c_fc": (D, 4 * D),
            "mlp.c_proj": (4 * D, D)}
    items = []
    for i in range(cfg.layers):
        for leaf in leaves:
            fin, fout = dims[leaf]
            A = torch.randn(fin, rank, generator=g) * 0.02
            B = torch.randn(rank, fout, generator=g) * 0.01
            items.append(LoraAdapter(f"visual.transformer.resblocks.{i}.{TARGET_WEIGHT[leaf]}",
                                     A.numpy().copy(), B.numpy().copy(), alpha / rank))
    return items
