"""Registers the package directory ``ai-interior-image-classifier_amd/`` under the import
name ``interior_amd`` (a hyphenated directory is not importable by name)."""
from __future__ import annotations

import importlib.util
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG_DIR = ROOT / "ai-interior-image-classifier_amd"
NAME = "interior_amd"


def load():
    mod = sys.modules.get(NAME)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(NAME, PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod


def build(force: bool = False):
    """Compile libclipvit_hip.so in-tree (see ai-interior-image-classifier_amd/build.py)."""
    load()
    from interior_amd import build as b  # noqa: E402
    return b.build(force=force)
