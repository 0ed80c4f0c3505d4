"""A ``clip``-shaped facade so main.py-style code runs on the GPU path unchanged:

    from interior_amd import clip_api as clip
    model, preprocess = clip.load("ViT-B/16", device="cuda")              # main.py:152 / 241
    text = model.encode_text(clip.tokenize(categories).to(device))       # main.py:179-182
    feats = model.encode_image(preprocess(img).unsqueeze(0).to(device))  # main.py:201-204
    model.load_lora_checkpoint("lora_models/comprehensive_lora.pth", 4, 8)  # main.py:247-251

``encode_image`` runs in libclipvit_hip.so's vision engine, ``encode_text`` in its text tower
(both hand-written gfx950 kernels, fp16 MFMA operands by default — the dtype clip.load gives a
CUDA model); ``tokenize`` is clip.tokenize (``tokenizer.SimpleTokenizer``) over the BPE merges
given by ``set_bpe_path`` / ``load(bpe_path=...)`` / the ``CLIPVIT_BPE_PATH`` environment
variable — the OpenAI merges file ``bpe_simple_vocab_16e6.txt.gz`` is not shipped here.
``load_lora_checkpoint`` applies the reference's binding rule (main.py:86-113: exact or
suffix match, absent adapters stay zero) to both towers and merges the bound adapters.
There is no CPU fallback: without a HIP device ``load`` raises.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .config import TextConfig, get_config, text_config_for
from .engine import VisionEngine
from .lora import load_lora_checkpoint, text_adapters_from_checkpoint, vision_adapters_from_checkpoint
from .preprocess import preprocess as _pp
from .text import TextEngine
from .tokenizer import SimpleTokenizer
from .weights import (load_openai_checkpoint, synthetic_state_dict, synthetic_text_state_dict,
                      text_names, visual_names)

_TOKENIZER: SimpleTokenizer | None = None


def set_tokenizer(tokenizer: SimpleTokenizer | None) -> None:
    """The tokenizer ``tokenize`` uses (None: rebuild from CLIPVIT_BPE_PATH on next use)."""
    global _TOKENIZER
    _TOKENIZER = tokenizer


def set_bpe_path(path) -> SimpleTokenizer:
    """Load a CLIP BPE merges file (``bpe_simple_vocab_16e6.txt[.gz]`` or a learned list)."""
    set_tokenizer(SimpleTokenizer(bpe_path=path))
    return _TOKENIZER


def _tokenizer() -> SimpleTokenizer:
    if _TOKENIZER is None:
        path = os.environ.get("CLIPVIT_BPE_PATH")
        if not path:
            raise RuntimeError("clip_api.tokenize needs the CLIP BPE merges: call set_bpe_path(...), "
                               "load(..., bpe_path=...) or set CLIPVIT_BPE_PATH")
        set_bpe_path(path)
    return _TOKENIZER


def tokenize(texts, context_length: int = 77, truncate: bool = False) -> torch.Tensor:
    """clip.tokenize [3p]: LongTensor [n, context_length] = sot, BPE ids, eot, zero padding;
    RuntimeError for a prompt longer than the context unless ``truncate``."""
    return torch.from_numpy(_tokenizer().tokenize(texts, context_length, truncate).astype(np.int64))


class ClipModel:
    """What ``clip.load`` returns, restricted to what main.py / main_API.py use."""

    def __init__(self, vision: VisionEngine, text: TextEngine | None):
        self.engine = vision
        self.text_engine = text
        self.visual = vision.cfg
        self.device = vision.device
        self.dtype = torch.float16 if vision.compute_dtype in ("fp16", "f16") else torch.bfloat16

    def eval(self):
        return self

    def encode_image(self, image: torch.Tensor) -> torch.Tensor:
        """[B, 3, R, R] -> [B, E] fp32 on the device (un-normalised, like CLIP)."""
        return self.engine.encode_image(image)

    def encode_text(self, text: torch.Tensor) -> torch.Tensor:
        """[K, 77] token ids -> [K, E] fp32 on the device (un-normalised, like CLIP)."""
        if self.text_engine is None:
            raise RuntimeError("this model was loaded without a text tower")
        ids = text.detach().to("cpu").numpy() if torch.is_tensor(text) else np.asarray(text)
        n = self.text_engine.max_batch
        parts = [self.text_engine.encode_text(ids[a:a + n]) for a in range(0, len(ids), n)]
        if not parts:
            return torch.empty((0, self.text_engine.cfg.embed_dim), device=self.device)
        return torch.cat(parts, dim=0)

    def load_lora_checkpoint(self, path, rank: int = 4, alpha: float = 8.0) -> dict:
        """replace_linears_with_lora + load_lora_weights_to_model (main.py:62-113, 247-251):
        bind the checkpoint's adapters by the reference's rule and merge them into both towers
        (the shipped checkpoints bind text-tower MLP adapters only; vision deltas stay zero)."""
        ckpt = load_lora_checkpoint(path)
        vis, loaded, missing = vision_adapters_from_checkpoint(ckpt, self.visual, rank, alpha)
        self.engine.load_lora(vis)
        txt = []
        if self.text_engine is not None:
            txt, _, _ = text_adapters_from_checkpoint(ckpt, self.text_engine.cfg.layers, rank, alpha,
                                                      self.visual.layers)
            self.text_engine.load_lora(txt)
        return {"loaded": loaded, "missing": len(missing), "vision_adapters": len(vis),
                "text_adapters": len(txt)}

    def close(self):
        self.engine.close()
        if self.text_engine is not None:
            self.text_engine.close()


def load(name: str = "ViT-B/16", device: str | int | torch.device = "cuda", jit: bool = False,
         weights: str | dict | None = None, compute_dtype: str = "fp16", max_batch: int = 64,
         seed: int = 0, text_seed: int = 1, bpe_path=None, text: bool = True):
    """(model, preprocess) like clip.load. ``weights``: a LOCAL OpenAI ``ViT-*.pt`` path (read
    without executing code from it), a state dict with OpenAI names, or ``"synthetic"`` for
    seeded stand-in weights (tests, bench). There is no download here, and the reference's
    ``clip.load`` never returns a random model (main.py:152, 241), so ``weights=None`` raises.
    ``jit`` is accepted and ignored. ``text=False`` skips the text tower."""
    del jit
    if weights is None:
        raise ValueError(f"clip_api.load({name!r}) needs weights: a local OpenAI ViT-*.pt path or a "
                         "state dict (nothing is downloaded here); weights='synthetic' gives seeded "
                         "stand-in weights")
    if not isinstance(weights, (str, os.PathLike, dict)):
        raise TypeError(f"weights must be a path, a state dict or 'synthetic', got {type(weights).__name__}")
    if bpe_path is not None:
        set_bpe_path(bpe_path)
    cfg = get_config(name)
    dev = torch.device(device if not isinstance(device, int) else f"cuda:{device}")
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    if isinstance(weights, str) and weights == "synthetic":
        vis_sd = synthetic_state_dict(cfg, seed)
        vocab = _TOKENIZER.vocab_size if _TOKENIZER is not None else TextConfig().vocab
        txt_sd = synthetic_text_state_dict(text_config_for(cfg, vocab), text_seed) if text else None
    elif isinstance(weights, (str, os.PathLike)):
        vis_sd = load_openai_checkpoint(weights)
        txt_sd = load_openai_checkpoint(weights, text=True) if text else None
    else:  # dict
        vis_sd = weights
        txt_sd = weights if text else None
    if any(n not in vis_sd for n, _ in visual_names(cfg)):
        raise KeyError(f"weights lack the {name} vision tower")
    eng = VisionEngine(cfg, device=dev, compute_dtype=compute_dtype, max_batch=max_batch)
    te = None
    try:
        eng.load_state_dict(vis_sd)
        if txt_sd is not None and "token_embedding.weight" in txt_sd:
            tc = text_config_for(cfg, int(np.asarray(txt_sd["token_embedding.weight"]).shape[0]))
            if all(n in txt_sd for n, _ in text_names(tc)):
                te = TextEngine(tc, dev, "bf16" if compute_dtype == "bf16" else "fp16", max_batch=256)
                te.load_state_dict(txt_sd)
    except Exception:
        eng.close()
        if te is not None:
            te.close()
        raise
    return ClipModel(eng, te), (lambda img: _pp(img, cfg.image_size))
