"""Vision-tower geometries of the CLIP models the reference (and BASELINE.json) name.

``clip.load("ViT-B/16")`` is what the reference actually runs (main.py:152, main.py:241,
python-worker/main_API.py:137, train_lora.py:174); BASELINE.json's metric is quoted on
ViT-B/32, with ViT-L/14@336px as the LDS-tiling stress config.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class ViTConfig:
    name: str
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

    def gflop_per_image(self) -> float:
        """Algorithmic GFLOP per image: GEMMs 2MNK, attention 4 N^2 D
        per layer; LayerNorm/softmax/GELU not counted; merged LoRA adds 0."""
        N, D, G2 = self.tokens, self.width, self.grid ** 2
        patch = 2.0 * G2 * (3 * self.patch_size ** 2) * D
        per_layer = 2.0 * N * D * (3 * D + D + 4 * D + 4 * D) + 4.0 * N * N * D
        head = 2.0 * D * self.embed_dim
        return (patch + self.layers * per_layer + head) / 1e9


VIT_B32 = ViTConfig("ViT-B/32", 224, 32, 768, 12, 12, 512)
VIT_B16 = ViTConfig("ViT-B/16", 224, 16, 768, 12, 12, 512)
VIT_L14 = ViTConfig("ViT-L/14", 224, 14, 1024, 24, 16, 768)
VIT_L14_336 = ViTConfig("ViT-L/14@336px", 336, 14, 1024, 24, 16, 768)

MODELS = {c.name: c for c in (VIT_B32, VIT_B16, VIT_L14, VIT_L14_336)}


def get_config(name: str) -> ViTConfig:
    if name not in MODELS:
        raise ValueError(f"unknown model {name!r}; available: {sorted(MODELS)}")
    return MODELS[name]


@dataclass(frozen=True)
class TextConfig:
    """OpenAI-CLIP text tower (CLIP.__init__ [3p]: transformer_width/layers/heads,
    context_length, vocab_size, embed_dim), used by encode_text at main.py:181 / main.py:308.
    B/32 and B/16 share it; L/14 has width 768, 12 heads, embed 768."""
    width: int = 512
    layers: int = 12
    heads: int = 8
    context: int = 77
    vocab: int = 49408
    embed_dim: int = 512

    def gflop_per_text(self) -> float:
        N, D = self.context, self.width
        return (self.layers * (2.0 * N * D * 12 * D + 4.0 * N * N * D) + 2.0 * D * self.embed_dim) / 1e9


TEXT_B = TextConfig()
TEXT_L = TextConfig(width=768, heads=12, embed_dim=768)


def text_config_for(vision: ViTConfig, vocab: int = 49408) -> TextConfig:
    base = TEXT_L if vision.width == 1024 else TEXT_B
    return TextConfig(base.width, base.layers, base.heads, base.context, vocab, base.embed_dim)
