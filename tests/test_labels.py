"""Label vocabulary and prompt table vs the reference harness (main.py:155-186, 264-311)."""
import json

from interior_amd import labels as L


def test_categories_equal_reference_sets(golden_dir):
    js = json.loads((golden_dir / "harness_vitb32_lora.json").read_text())
    mine = L.extract_categories(L.load_training_data(golden_dir / "interior_dataset.json"))
    ref = js["categories"]  # reference order under PYTHONHASHSEED=0 (set order)
    assert {k: len(v) for k, v in mine.items()} == {"styles": 20, "characteristics": 299,
                                                   "materials": 36, "colors": 30, "room_types": 12}
    for k in mine:
        assert sorted(mine[k]) == sorted(ref[k]), k


def test_detector_categories_match_reference(golden_dir):
    js = json.loads((golden_dir / "harness_vitb32_lora.json").read_text())
    assert L.DETECTOR_CATEGORIES == js["detector_categories"]
    assert L.N_INTERIOR == 11


def test_label_table_offsets_and_prompts(golden_dir):
    cats = L.extract_categories(L.load_training_data(golden_dir / "interior_dataset.json"))
    t = L.build_label_table(cats)
    assert t.segments == ["detector", "styles", "characteristics", "materials", "colors", "room_types"]
    assert t.offsets == [0, 40, 60, 359, 395, 425, 437]
    assert t.texts[1][0] == f"wnętrze z {cats['styles'][0]}"
    assert t.texts[5][0] == cats["room_types"][0]  # room types are bare (main.py:300-301)


def test_missing_dataset_gives_empty(tmp_path):
    assert L.load_training_data(tmp_path / "nope.json") == []
    t = L.build_label_table(L.extract_categories([]))
    assert t.segments == ["detector"]
