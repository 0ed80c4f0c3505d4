"""A ``clip``-shaped facade so main.py-style code runs on the GPU path unchanged:

    model, preprocess = clip_api.load("ViT-B/16", device="cuda")      # main.py:152 / 241
    feats = model.encode_image(preprocess(img).unsqueeze(0).to(dev))    # main.py:201-204

``encode_image`` runs in libclipvit_hip.so. The text tower is not part of this path
(SURVEY.md §8(f) rank 3): ``encode_text`` serves precomputed features registered with
``register_text_features`` (or raises), which is what the reference does after its one-time
text-feature cache (main.py:179-182, 296-311).
"""
from __future__ import annotations

import numpy as np
import torch

from .config import get_config
from .engine import VisionEngine
from .preprocess import preprocess as _pp
from .weights import load_openai_checkpoint, synthetic_state_dict


class ClipVisionModel:
    def __init__(self, engine: VisionEngine):
        self.engine = engine
        self.visual = engine.cfg
        self._text: dict[str, np.ndarray] = {}

    def encode_image(self, image: torch.Tensor) -> torch.Tensor:
        return self.engine.encode_image(image)

    def register_text_features(self, texts: list[str], feats) -> None:
        feats = np.asarray(feats, dtype=np.float32)
        for t, f in zip(texts, feats):
            self._text[t] = f

    def encode_text(self, texts) -> torch.Tensor:
        strings = texts.strings if hasattr(texts, "strings") else list(texts)
        missing = [s for s in strings if s not in self._text]
        if missing:
            raise NotImplementedError(f"no text tower on the GPU path; unregistered prompts: {missing[:3]}")
        return torch.from_numpy(np.stack([self._text[s] for s in strings])).to(self.engine.device)

    def eval(self):
        return self


def load(name: str = "ViT-B/16", device: str | int = "cuda", weights: str | dict | None = None,
         compute_dtype: str = "bf16", max_batch: int = 64, seed: int = 0):
    """(model, preprocess) like clip.load; ``weights`` = local OpenAI .pt path, a state dict,
    or None for seeded synthetic weights (no network here)."""
    cfg = get_config(name)
    dev = torch.device(device if not isinstance(device, int) else f"cuda:{device}")
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    eng = VisionEngine(cfg, device=dev, compute_dtype=compute_dtype, max_batch=max_batch)
    if weights is None:
        sd = synthetic_state_dict(cfg, seed)
    elif isinstance(weights, dict):
        sd = weights
    else:
        sd = load_openai_checkpoint(weights)
    eng.load_state_dict(sd)
    return ClipVisionModel(eng), (lambda img: _pp(img, cfg.image_size))
