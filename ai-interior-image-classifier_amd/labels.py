"""Label vocabulary and prompts of the classifier head.

* Detector prompts: the 40 English categories of InteriorImageDetector (main.py:155-176),
  the first 11 are "interior" (main.py:185-186).
* Analyzer labels: unique styles / characteristics / materials / colors / room types of
  ``interior_dataset.json`` (main.py:264-294), prompts ``"wnętrze z {a}"`` except room types,
  which are used bare (main.py:300-305).

The reference collects labels into Python ``set``s, so its column order depends on
PYTHONHASHSEED. Here the order is first appearance in the dataset, which is
deterministic; results are reported keyed by label string, which is what the reference's
output dicts expose, so the two orders are interchangeable.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from pathlib import Path

DETECTOR_CATEGORIES = [
    "interior of a room", "living room", "bedroom", "kitchen", "bathroom",
    "dining room", "office interior", "apartment interior", "house interior",
    "interior design", "home decor",
    "building exterior", "outside of building", "street view", "garden",
    "landscape", "cityscape", "outdoor",
    "floor plan", "blueprint", "architectural plan", "diagram",
    "map", "technical drawing",
    "company logo", "brand logo", "text", "signature",
    "advertisement", "brochure", "flyer",
    "person", "people", "animal", "pet", "car", "vehicle",
    "close-up of object", "product photo", "furniture close-up",
]
N_INTERIOR = 11
ANALYZER_CATEGORIES = ("styles", "characteristics", "materials", "colors", "room_types")


def load_training_data(json_path: str | Path) -> list[dict]:
    """main.py:264-271 (returns [] on any error, like the reference)."""
    try:
        with open(json_path, "r", encoding="utf-8") as f:
            return json.load(f).get("training_data", [])
    except Exception:
        return []


def extract_categories(training_data: list[dict]) -> dict[str, list[str]]:
    """main.py:273-294 with deterministic (first-appearance) order."""
    seen = {k: {} for k in ANALYZER_CATEGORIES}
    for item in training_data:
        seen["styles"].setdefault(item.get("style", ""), None)
        seen["room_types"].setdefault(item.get("room_type", ""), None)
        for c in item.get("characteristics", []):
            seen["characteristics"].setdefault(c, None)
        for m in item.get("materials", []):
            seen["materials"].setdefault(m, None)
        for col in item.get("colors", []):
            seen["colors"].setdefault(col, None)
    return {k: [a for a in seen[k] if a] for k in ANALYZER_CATEGORIES}


def prompts(category: str, attrs: list[str]) -> list[str]:
    """main.py:300-305."""
    return [f"{a}" for a in attrs] if category == "room_types" else [f"wnętrze z {a}" for a in attrs]


@dataclass
class LabelTable:
    """Concatenated head columns: segment 0 = detector, then one segment per non-empty
    analyzer category, in main.py's dict order."""
    segments: list[str] = field(default_factory=list)
    labels: list[list[str]] = field(default_factory=list)
    texts: list[list[str]] = field(default_factory=list)

    @property
    def offsets(self) -> list[int]:
        off = [0]
        for l in self.labels:
            off.append(off[-1] + len(l))
        return off

    @property
    def all_texts(self) -> list[str]:
        return [t for ts in self.texts for t in ts]

    def segment(self, name: str) -> int:
        return self.segments.index(name)


def build_label_table(categories: dict[str, list[str]]) -> LabelTable:
    t = LabelTable()
    t.segments.append("detector")
    t.labels.append(list(DETECTOR_CATEGORIES))
    t.texts.append(list(DETECTOR_CATEGORIES))
    for cat in ANALYZER_CATEGORIES:
        attrs = categories.get(cat, [])
        if not attrs:
            continue  # main.py:299
        t.segments.append(cat)
        t.labels.append(list(attrs))
        t.texts.append(prompts(cat, attrs))
    return t
