"""TextEngine: the CLIP text tower on one GPU (clipvit_text_* in libclipvit_hip.so).

Replaces ``model.encode_text(clip.tokenize(prompts))`` as the reference runs it once per prompt
set (main.py:179-182 detector, main.py:296-311 analyzer), with the shipped checkpoints' text
LoRA merged (``lora.text_adapters_from_checkpoint``). ``label_matrix`` returns the normalised
T [C, E] that ``VisionEngine.set_text_features`` consumes. No CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .config import TextConfig
from .lora import LoraAdapter
from .weights import as_host_f32, text_names

_DT = {"bf16": _lib.BF16, "fp16": _lib.F16, "f16": _lib.F16}


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


class TextEngine:
    def __init__(self, cfg: TextConfig, device: int | str | torch.device = 0,
                 compute_dtype: str = "fp16", max_batch: int = 256):
        if not torch.cuda.is_available():
            raise _lib.ClipVitError(_lib.E_STATE, "no HIP device visible: the MI355X path needs a GPU")
        dev = torch.device(device if not isinstance(device, int) else f"cuda:{device}")
        self.device = torch.device("cuda", dev.index if dev.index is not None else torch.cuda.current_device())
        self.cfg = cfg
        self.max_batch = int(max_batch)
        self._L = _lib.lib()
        c = _lib.TextConfig(cfg.width, cfg.layers, cfg.heads, cfg.context, cfg.vocab, cfg.embed_dim,
                            _DT[compute_dtype], self.max_batch)
        h = ctypes.c_void_p()
        _lib.check(self._L.clipvit_text_create(ctypes.byref(c), self.device.index, ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.clipvit_text_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_state_dict(self, sd: dict) -> None:
        """Text-tower tensors (OpenAI names; a full CLIP state dict works: visual.* is skipped)."""
        names = text_names(self.cfg)
        keep, arr = [], (_lib.Tensor * len(names))()
        for i, (name, shape) in enumerate(names):
            if name not in sd:
                raise KeyError(f"missing {name}")
            a = as_host_f32(sd[name])
            if tuple(a.shape) != tuple(shape):
                raise ValueError(f"{name}: shape {a.shape} != {shape}")
            bn = name.encode()
            keep += [a, bn]
            arr[i].name, arr[i].data, arr[i].ndim = bn, _fptr(a), a.ndim
            for d in range(a.ndim):
                arr[i].shape[d] = a.shape[d]
        _lib.check(self._L.clipvit_text_load_weights(self._h, arr, len(names)))

    def load_lora(self, adapters: list[LoraAdapter]) -> None:
        keep, arr = [], (_lib.Lora * max(len(adapters), 1))()
        for i, ad in enumerate(adapters):
            A, B = as_host_f32(ad.A), as_host_f32(ad.B)
            t = ad.target.encode()
            keep += [A, B, t]
            arr[i].target, arr[i].A, arr[i].B = t, _fptr(A), _fptr(B)
            arr[i].in_features, arr[i].out_features = A.shape[0], B.shape[1]
            arr[i].rank, arr[i].scaling = A.shape[1], float(ad.scaling)
        _lib.check(self._L.clipvit_text_load_lora(self._h, arr, len(adapters)))

    def encode_text(self, tokens, normalize: bool = False) -> torch.Tensor:
        """tokens [B, context] ids (clip.tokenize layout) -> [B, E] fp32 on the device;
        batches above max_batch are the caller's to split (ClipVitError, like the ABI)."""
        ids = np.ascontiguousarray(np.asarray(tokens), dtype=np.int32)
        if ids.ndim != 2 or ids.shape[1] != self.cfg.context:
            raise ValueError(f"tokens must be [B, {self.cfg.context}], got {ids.shape}")
        if ids.size and (ids.min() < 0 or ids.max() >= self.cfg.vocab):
            raise ValueError(f"token ids must lie in [0, {self.cfg.vocab})")
        B = ids.shape[0]
        out = torch.empty((B, self.cfg.embed_dim), dtype=torch.float32, device=self.device)
        if B == 0:
            return out
        dev_ids = torch.from_numpy(ids).to(self.device)
        with torch.cuda.device(self.device):
            s = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
            _lib.check(self._L.clipvit_encode_text(self._h, s, ctypes.c_void_p(dev_ids.data_ptr()), B,
                                                   int(bool(normalize)), ctypes.c_void_p(out.data_ptr())))
        torch.cuda.current_stream(self.device).synchronize()
        return out

    def label_matrix(self, tokenizer, texts: list[str]) -> np.ndarray:
        """main.py:306-310 for a list of prompts: normalised features [len(texts), E] (host)."""
        rows = []
        for a in range(0, len(texts), self.max_batch):
            ids = tokenizer.tokenize(texts[a:a + self.max_batch], self.cfg.context)
            rows.append(self.encode_text(ids, normalize=True).cpu().numpy())
        return np.concatenate(rows, axis=0) if rows else np.zeros((0, self.cfg.embed_dim), np.float32)
