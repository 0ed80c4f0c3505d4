"""MI355X-native CLIP-ViT + LoRA image path for the AI interior image classifier.

Import name: ``interior_amd`` (the directory name has hyphens; ``amd_pkg.load()`` at the repo
root registers it). Layout:
    csrc/          hand-written gfx950 HIP kernels + the C ABI (include/clipvit.h)
    _lib.py        ctypes binding (GIL released inside every call)
    engine.py      VisionEngine: one handle = one GPU
    analyzer.py    the reference's predict / analyze surface (main.py, main_API.py)
    lora.py        comprehensive_lora*.pth format + binding rule, merged at load
    weights.py     OpenAI names, synthetic seeded weights, local checkpoint loader
    preprocess.py  clip _transform on the host
    labels.py      detector + analyzer label table
    dp.py          data-parallel sharding + RCCL all-gather of logits
    clip_api.py    clip.load-shaped facade
"""
from .config import MODELS, VIT_B16, VIT_B32, VIT_L14, VIT_L14_336, ViTConfig, get_config

__all__ = ["MODELS", "VIT_B16", "VIT_B32", "VIT_L14", "VIT_L14_336", "ViTConfig", "get_config"]
