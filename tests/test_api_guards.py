"""The product surface refuses to build a model it was not given.

The reference's ``clip.load`` always loads real weights (main.py:152, main.py:241); a silent
random model would return meaningless labels with no error. ``clip_api.load`` and
``InteriorAnalyzer`` therefore raise unless weights (and label features) are passed, or the
caller opts into seeded stand-ins explicitly with ``"synthetic"`` (tests and bench do). The
checks run before any device work, so they are CPU tests. Also: the tuning hook of the C ABI
rejects a null handle (CPU-checkable part of clipvit_set_tuning).
"""
import ctypes

import pytest

from interior_amd import _lib
from interior_amd import clip_api
from interior_amd.analyzer import InteriorAnalyzer


def test_clip_load_without_weights_raises():
    with pytest.raises(ValueError, match="needs weights"):
        clip_api.load("ViT-B/32", device="cuda")


def test_clip_load_rejects_unknown_weight_kind():
    with pytest.raises(TypeError):
        clip_api.load("ViT-B/32", device="cuda", weights=12345)


def test_analyzer_without_vision_weights_raises(golden_dir):
    with pytest.raises(ValueError, match="needs vision weights"):
        InteriorAnalyzer("ViT-B/32", text_features="synthetic",
                         dataset_json=golden_dir / "interior_dataset.json")


def test_analyzer_without_label_features_raises(golden_dir):
    with pytest.raises(ValueError, match="needs label features"):
        InteriorAnalyzer("ViT-B/32", state_dict="synthetic",
                         dataset_json=golden_dir / "interior_dataset.json")


def test_analyzer_rejects_other_strings(golden_dir):
    with pytest.raises(ValueError):
        InteriorAnalyzer("ViT-B/32", state_dict="random", text_features="synthetic")
    with pytest.raises(ValueError):
        InteriorAnalyzer("ViT-B/32", state_dict="synthetic", text_features="random")


def test_set_tuning_null_handle():
    L = _lib.lib()
    assert L.clipvit_set_tuning(ctypes.c_void_p(), b"split_min=0") == _lib.E_INVALID
