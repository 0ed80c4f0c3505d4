"""The reference's Python surface, served by one GPU pass per image.

Mirrors main.py's ``InteriorImageDetector`` (main.py:149-226) and ``CachedInteriorAnalyzer``
(main.py:232-510) and fills the per-image contract python-worker/main_API.py expects
(``{'style', 'confidence'}`` + detector ``room_type``, main_API.py:186-196, 219-236):

* ``predict(image) -> {is_interior, interior_confidence, detected_category, room_type, style,
  confidence, attributes{styles, characteristics, materials, colors, room_types}, reason}``
* ``predict_batch(images, batch_size)``
* ``is_interior_image(img, confidence_threshold=0.3) -> (bool, float, str)``  (main.py:191)
* ``analyze_images_batch(paths, batch_size=16, filter_interiors=True,
  confidence_threshold=0.3) -> {path: result}``                               (main.py:371)
* ``analyze_image_from_url(url, filter_interiors=True) -> result``            (main.py:472)

The reference runs TWO ViT forwards per image (detector model at batch 1, analyzer model at
batch 16). Both use the same base vision weights and the vision LoRA is zero/merged, so here
one ``classify`` call produces the detector's 40 columns and the analyzer's columns together
(SURVEY.md §8(f) rank 1). Errors never escape ``is_interior_image``; batch results carry the
reference's sentinel dicts (main.py:224-226, 329-330, 418-426).
"""
from __future__ import annotations

import zlib
from pathlib import Path

import numpy as np
import torch

from . import labels as L
from .config import ViTConfig, get_config
from .engine import VisionEngine
from .lora import load_lora_checkpoint, vision_adapters_from_checkpoint
from .preprocess import load_image, preprocess_batch, preprocess_batch_gpu
from .weights import synthetic_state_dict


def synthetic_text_features(texts: list[str], dim: int) -> np.ndarray:
    """Deterministic stand-in text features (no text tower / BPE vocab offline): a crc32-seeded
    Gaussian per prompt, L2-normalised like main.py:182 / main.py:309."""
    out = np.empty((len(texts), dim), dtype=np.float32)
    for i, t in enumerate(texts):
        g = torch.Generator().manual_seed(zlib.crc32(t.encode("utf-8")))
        v = torch.randn(dim, generator=g)
        out[i] = (v / v.norm()).numpy()
    return out


SYNTHETIC = "synthetic"  # explicit opt-in to seeded stand-in weights / text rows (tests, bench)


class InteriorAnalyzer:
    """``state_dict``: the vision tower's weights (OpenAI names), or ``"synthetic"`` for seeded
    stand-in weights (``weights_seed``). Text rows: ``text_features`` (array or per-segment
    dict), or ``text_state_dict`` (+ BPE) for the GPU text tower, or ``text_features=
    "synthetic"`` for crc32-seeded stand-in rows. Like ``clip.load`` in the reference
    (main.py:152, 241), which never hands back a random model, anything else raises: a silent
    random model would produce meaningless labels with no error."""

    def __init__(self, model: str | ViTConfig = "ViT-B/16", state_dict: dict | str | None = None,
                 use_lora: bool = False, lora_weights_path: str | None = None, lora_rank: int = 4,
                 lora_alpha: float = 8, device: int | str = 0, compute_dtype: str = "fp16",
                 dataset_json: str | Path = "interior_dataset.json",
                 text_features: dict[str, np.ndarray] | np.ndarray | str | None = None,
                 categories: dict[str, list[str]] | None = None, max_batch: int = 64,
                 weights_seed: int = 0, gpu_preprocess: bool = True,
                 text_state_dict: dict | None = None, bpe_path: str | None = None, tokenizer=None,
                 extra_segments: dict[str, tuple[list[str], list[str]]] | None = None):
        self.gpu_preprocess = bool(gpu_preprocess)  # _transform on the GPU (bit-identical)
        self.cfg = model if isinstance(model, ViTConfig) else get_config(model)
        if state_dict is None:
            raise ValueError("InteriorAnalyzer needs vision weights: state_dict=<OpenAI-named state dict> "
                             "(weights.load_openai_checkpoint reads a local ViT-*.pt), or "
                             "state_dict='synthetic' for seeded stand-in weights")
        if isinstance(state_dict, str) and state_dict != SYNTHETIC:
            raise ValueError(f"state_dict must be a dict or {SYNTHETIC!r}, got {state_dict!r}")
        if text_features is None and text_state_dict is None:
            raise ValueError("InteriorAnalyzer needs label features: text_features=<[C, E] rows or "
                             "{segment: rows}>, text_state_dict=<text tower weights> (+ bpe_path / "
                             "tokenizer), or text_features='synthetic' for seeded stand-in rows")
        if isinstance(text_features, str) and text_features != SYNTHETIC:
            raise ValueError(f"text_features must be an array, a dict or {SYNTHETIC!r}, got {text_features!r}")
        self.engine = VisionEngine(self.cfg, device=device, compute_dtype=compute_dtype,
                                   max_batch=max_batch)
        self.engine.load_state_dict(synthetic_state_dict(self.cfg, weights_seed)
                                    if isinstance(state_dict, str) else state_dict)
        self.use_lora = bool(use_lora)
        self.lora_report = None
        ckpt = None
        if use_lora and lora_weights_path and Path(lora_weights_path).exists():
            ckpt = load_lora_checkpoint(lora_weights_path)
            items, loaded, missing = vision_adapters_from_checkpoint(ckpt, self.cfg, lora_rank, lora_alpha)
            self.engine.load_lora(items)
            self.lora_report = {"loaded": loaded, "missing": len(missing), "vision_adapters": len(items)}
        if categories is None:
            categories = L.extract_categories(L.load_training_data(dataset_json))
        self.all_categories = categories
        self.table = L.build_label_table(categories)
        for name, (labels, texts) in (extra_segments or {}).items():  # e.g. worker.WORKER_STYLES
            if len(labels) != len(texts) or not labels:
                raise ValueError(f"extra segment {name!r}: labels and prompts must be non-empty, same length")
            self.table.segments.append(name)
            self.table.labels.append(list(labels))
            self.table.texts.append(list(texts))
        if text_features is None:
            text_features = self._encode_labels(text_state_dict, ckpt, lora_rank, lora_alpha,
                                                bpe_path, tokenizer, compute_dtype, device)
        T = self._text_matrix(text_features)
        self.text_matrix = T  # [C, E] host copy of the label features the head uses
        self.engine.set_text_features(T, self.table.offsets)

    def _encode_labels(self, text_sd, ckpt, rank, alpha, bpe_path, tokenizer, compute_dtype, device):
        """The reference's two text caches on the GPU text tower: the detector prompts through
        the BASE text tower (InteriorImageDetector's own clip.load, main.py:152/179-182), the
        analyzer prompts through the LoRA text tower (main.py:241-251, 296-311)."""
        from .config import text_config_for
        from .lora import text_adapters_from_checkpoint
        from .text import TextEngine
        from .tokenizer import SimpleTokenizer
        tok = tokenizer if tokenizer is not None else SimpleTokenizer(bpe_path=bpe_path)
        tc = text_config_for(self.cfg, int(np.asarray(text_sd["token_embedding.weight"]).shape[0]))
        te = TextEngine(tc, device, "bf16" if compute_dtype == "bf16" else "fp16", max_batch=256)
        try:
            te.load_state_dict(text_sd)
            det = te.label_matrix(tok, self.table.texts[0])
            if ckpt is not None:
                items, loaded, _ = text_adapters_from_checkpoint(ckpt, tc.layers, rank, alpha, self.cfg.layers)
                te.load_lora(items)
                self.lora_report = dict(self.lora_report or {}, text_adapters=len(items))
            rest = te.label_matrix(tok, [t for ts in self.table.texts[1:] for t in ts])
        finally:
            te.close()
        return np.concatenate([det, rest], axis=0)

    def _text_matrix(self, text_features) -> np.ndarray:
        E = self.cfg.embed_dim
        if isinstance(text_features, str):  # SYNTHETIC (checked in __init__)
            return synthetic_text_features(self.table.all_texts, E)
        if isinstance(text_features, np.ndarray) or torch.is_tensor(text_features):
            T = np.asarray(text_features, dtype=np.float32)
            if T.shape != (len(self.table.all_texts), E):
                raise ValueError(f"text_features must be [{len(self.table.all_texts)}, {E}]")
            return T
        # dict: segment name -> [n, E]
        return np.concatenate([np.asarray(text_features[s], dtype=np.float32)
                               for s in self.table.segments], axis=0)

    # ------------------------------------------------------------------ core batch pass
    def _pixels(self, images) -> torch.Tensor:
        """preprocess (main.py:201/438/489) of RGB PIL images: on the GPU by default
        (clipvit_preprocess), else PIL on host threads; both give the same fp32 bits."""
        if self.gpu_preprocess:
            return preprocess_batch_gpu(images, self.cfg.image_size, self.engine.device)
        return preprocess_batch(images, self.cfg.image_size)

    def _run(self, pixels: torch.Tensor):
        out = self.engine.classify(pixels)
        return (out.probs.cpu().numpy(), out.top_idx.cpu().numpy(), out.top_prob.cpu().numpy())

    def _detector(self, probs_row: np.ndarray, threshold: float):
        """main.py:207-222 on the detector segment."""
        det = probs_row[: len(L.DETECTOR_CATEGORIES)]
        top_i = int(np.argmax(det))
        top_conf = float(det[top_i])
        interior = float(det[:L.N_INTERIOR].sum())
        non_interior = float(det[L.N_INTERIOR:].sum())
        is_int = interior > non_interior and top_conf > threshold
        return is_int, interior, L.DETECTOR_CATEGORIES[top_i]

    def _analysis(self, top_idx: np.ndarray, top_prob: np.ndarray) -> dict:
        """main.py:451-459: {category: [(label, prob) x min(5, n)]}."""
        res = {}
        for s, cat in enumerate(self.table.segments):
            if s == 0:
                continue
            labs = self.table.labels[s]
            k = min(5, len(labs))
            res[cat] = [(labs[int(top_idx[s, j])], float(top_prob[s, j])) for j in range(k)]
        return res

    def _result(self, probs_row, tidx, tprob, threshold, filter_interiors=True) -> dict:
        is_int, conf, cat = self._detector(probs_row, threshold)
        analysis = self._analysis(tidx, tprob)
        style = analysis.get("styles", [(None, 0.0)])[0]
        room = analysis.get("room_types", [(None, 0.0)])[0]
        if filter_interiors and not is_int:
            return {"is_interior": False, "interior_confidence": conf, "detected_category": cat,
                    "room_type": None, "style": None, "confidence": 0.0, "analysis": {},
                    "attributes": {}, "reason": f"Nie wnętrze: {cat} (confidence: {conf:.3f})"}
        return {"is_interior": True, "interior_confidence": conf if filter_interiors else 1.0,
                "detected_category": "interior", "room_type": room[0], "style": style[0],
                "confidence": style[1], "analysis": analysis, "attributes": analysis,
                "reason": "Success - interior image analyzed"}

    # ------------------------------------------------------------------ public API
    def logits(self, images, batch_size: int = 64) -> np.ndarray:
        """The head's 100 * cos logits [n, C] of RGB PIL images (main.py:208 / 456 before the
        softmax): detector columns first, then each analyzer segment (``self.table``)."""
        rows = []
        for a in range(0, len(images), batch_size):
            out = self.engine.classify(self._pixels(images[a:a + batch_size]))
            rows.append(out.logits.cpu().numpy())
        return np.concatenate(rows, axis=0) if rows else np.zeros((0, self.engine.C), np.float32)

    def predict_batch(self, images, batch_size: int = 64, confidence_threshold: float = 0.3,
                      filter_interiors: bool = True) -> list[dict]:
        out = []
        n_px = self.cfg.image_size
        for a in range(0, len(images), batch_size):
            chunk = images[a:a + batch_size]
            px = self._pixels(chunk)
            probs, tidx, tprob = self._run(px)
            for i in range(len(chunk)):
                out.append(self._result(probs[i], tidx[i], tprob[i], confidence_threshold, filter_interiors))
        return out

    def predict(self, image, confidence_threshold: float = 0.3, filter_interiors: bool = True) -> dict:
        return self.predict_batch([image], 1, confidence_threshold, filter_interiors)[0]

    def is_interior_image(self, image, confidence_threshold: float = 0.3):
        if image is None:
            return False, 0.0, "invalid image"                       # main.py:196-197
        try:
            px = self._pixels([image])
            probs, _, _ = self._run(px)
            return self._detector(probs[0], confidence_threshold)
        except Exception as e:                                       # main.py:224-226
            return False, 0.0, f"error: {e}"

    def analyze_images_batch(self, image_paths, batch_size: int = 16, filter_interiors: bool = True,
                             confidence_threshold: float = 0.3) -> dict:
        results, imgs, keep = {}, [], []
        for p in image_paths:
            try:
                imgs.append(load_image(p))
                keep.append(p)
            except Exception as e:
                if filter_interiors:                                 # main.py:328-330, 336-338
                    results[p] = {"is_interior": False, "interior_confidence": 0.0,
                                  "detected_category": f"error: {e}", "analysis": {},
                                  "reason": f"Nie wnętrze: error: {e} (confidence: 0.000)"}
                else:                                                # main.py:418-426
                    results[p] = {"is_interior": False, "interior_confidence": 0.0,
                                  "detected_category": "load error", "analysis": {},
                                  "reason": f"Błąd ładowania: {e}"}
        preds = self.predict_batch(imgs, batch_size, confidence_threshold, filter_interiors)
        for p, r in zip(keep, preds):
            results[p] = {k: r[k] for k in ("is_interior", "interior_confidence",
                                            "detected_category", "analysis", "reason")}
        return results

    def analyze_image_from_url(self, url: str, filter_interiors: bool = True) -> dict:
        try:
            img = load_image(url)
        except Exception:
            return {"is_interior": False, "reason": "Failed to load image"}   # main.py:474-475
        r = self.predict(img, 0.3, filter_interiors)
        if not r["is_interior"]:
            return {"is_interior": False, "interior_confidence": r["interior_confidence"],
                    "detected_category": r["detected_category"], "analysis": {},
                    "reason": f"Not an interior image: {r['detected_category']}"}
        return {k: r[k] for k in ("is_interior", "interior_confidence", "detected_category",
                                  "analysis", "reason")}
