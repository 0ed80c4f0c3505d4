"""python-worker contract (worker.py; main_API.py:129-345), SURVEY.md §8(f) rank 4.

CPU: aggregation helpers and the in-memory database interface. GPU: the whole apartment
pipeline through InteriorAnalyzer (one classify pass per batch) — per-image database updates,
non-interior sentinel rows, and the per-image style equal to the worker-style segment's top-1
of the same predict_batch call.
"""
from __future__ import annotations

import numpy as np
import pytest
from PIL import Image

from interior_amd import worker as W


def test_dominant_style_and_room_distribution():
    ra = [{"room_type": "salon", "style": "boho", "style_confidence": 0.5},
          {"room_type": "kuchnia", "style": "retro", "style_confidence": 0.9},
          {"room_type": "salon", "style": "boho", "style_confidence": 0.6}]
    d = W.dominant_style(ra)
    assert d["style"] == "boho" and abs(d["confidence"] - 1.1 / 3) < 1e-12
    assert list(d["votes"]) == ["boho", "retro"]
    assert W.room_distribution(ra) == {"salon": 2, "kuchnia": 1}
    assert W.dominant_style([])["style"] is None and W.room_distribution([]) == {}


def test_worker_segment_prompts():
    seg = W.worker_style_segment()[W.WORKER_SEGMENT]
    assert seg[0] == W.WORKER_STYLES and seg[1][0] == "wnętrze w stylu nowoczesny" and len(seg[1]) == 10


def test_in_memory_database_interface():
    db = W.InMemoryDatabase({"a1": {"title": "t", "images": [{"_id": 1, "url": "u1"}, {"_id": 2, "url": "u2"}]},
                             "a2": {"title": "s", "images": [{"_id": 3, "url": "u3"}]}})
    assert sorted(p["_id"] for p in db.get_pending_apartments()) == ["a1", "a2"]
    db.update_image_analysis(1, "salon", "boho", 0.4)
    assert len(db.get_apartment_with_images("a1")["images"]) == 1
    assert db.get_apartment_with_images("nope") is None


@pytest.mark.gpu
def test_gpu_apartment_pipeline(gpu, golden_dir):
    from interior_amd.analyzer import InteriorAnalyzer
    an = InteriorAnalyzer("ViT-B/32", state_dict="synthetic", text_features="synthetic", device=gpu,
                          compute_dtype="fp16", max_batch=8, dataset_json=golden_dir / "interior_dataset.json",
                          extra_segments=W.worker_style_segment())
    files = sorted((golden_dir / "images").glob("*.jpg"))[::12]  # 13 of the 151 fixture photos
    rng = np.random.default_rng(0)
    noise = Image.fromarray(rng.integers(0, 256, (300, 400, 3), dtype=np.uint8), "RGB")
    imgs = {str(p): Image.open(p).convert("RGB") for p in files}
    imgs["noise"] = noise
    db = W.InMemoryDatabase({
        "apt1": {"title": "A", "images": [{"_id": i, "url": u} for i, u in enumerate(imgs)]},
        "apt2": {"title": "B", "images": [{"_id": 100, "url": "missing"}]}})

    def loader(u):
        if u not in imgs:
            raise FileNotFoundError(u)
        return imgs[u]

    w = W.DatabaseStyleRoomAnalyzer(db, an, image_loader=loader)
    # threshold 0 with synthetic weights: the detector decides on interior vs non-interior sums
    res = w.analyze_apartment_from_db("apt1", batch_size=4, confidence_threshold=0.0)
    preds = an.predict_batch(list(imgs.values()), 4, 0.0)
    n_int = sum(p["is_interior"] for p in preds)
    if n_int == 0:
        assert res is None
    else:
        assert res["interior_images"] == n_int and res["total_images"] == len(imgs)
        assert sum(res["room_distribution"].values()) == n_int
        assert db.analysis_results["apt1"]["analyzed_images"] == n_int
    for i, p in enumerate(preds):
        row = db.images[i]
        assert row["analysis_status"] == "completed"
        if p["is_interior"]:
            assert (row["style"], row["room_type"]) == (p["analysis"][W.WORKER_SEGMENT][0][0], p["room_type"])
        else:
            assert (row["room_type"], row["style"], row["analysis_confidence"]) == ("not_interior", "unknown", 0.0)
    styles = w._analyze_styles_batch(list(imgs.values()), 4)
    assert [s["style"] for s in styles] == [p["analysis"][W.WORKER_SEGMENT][0][0] for p in
                                            an.predict_batch(list(imgs.values()), 4, filter_interiors=False)]
    assert w.analyze_apartment_from_db("apt2") is None and db.images[100]["analysis_status"] == "pending"
    out = W.process_apartments_pipeline(db, an)
    assert set(out) == {"apt2"}  # apt1 fully processed; apt2's only image cannot be loaded
    an.engine.close()
