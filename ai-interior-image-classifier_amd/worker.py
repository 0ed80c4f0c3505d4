"""The python-worker consumer (python-worker/main_API.py), made real on top of predict_batch
(SURVEY.md §8(f) rank 4).

main_API.py's ``DatabaseStyleRoomAnalyzer`` expects a detector that returns a 4-tuple with
``room_type`` (main_API.py:186-188), a ``_analyze_styles_batch`` returning
``[{'style', 'confidence'}]`` (main_API.py:213-236), and ``_calculate_dominant_style`` /
``_calculate_room_distribution`` (main_API.py:243-244) — but in the reference those three
bodies are ``pass`` ("identyczna jak poprzednio", main_API.py:268-281) and the detector class is
not defined in that file, so the worker cannot run as shipped. Here:

* one GPU ``classify`` pass per batch yields detector + room type (analyzer ``room_types``
  segment) + the worker's own style head (10 styles, prompts ``"wnętrze w stylu {s}"``,
  main_API.py:152-161, an extra label segment of the same pass);
* ``_calculate_dominant_style``: confidence-weighted vote — the style whose summed
  ``style_confidence`` over the apartment's interior images is largest; its confidence is
  that sum divided by the number of interior images (semantics defined here, the
  reference's body is elided);
* ``_calculate_room_distribution``: ``{room_type: count}`` over interior images, most frequent
  first (same caveat);
* the database is any object with main_API.py's ``LocalDatabaseClient`` methods
  (``get_pending_apartments``, ``get_apartment_with_images``, ``update_image_analysis``,
  ``save_apartment_analysis``); ``InMemoryDatabase`` is a dependency-free one (MongoDB is out of
  scope).
"""
from __future__ import annotations

from collections import Counter, defaultdict

from .preprocess import load_image

WORKER_STYLES = ["nowoczesny", "klasyczny", "skandynawski", "industrialny", "rustykalny",
                 "glamour", "minimalistyczny", "retro", "boho", "farmhouse"]  # main_API.py:152-155
WORKER_SEGMENT = "worker_styles"


def worker_style_segment() -> dict[str, tuple[list[str], list[str]]]:
    """``extra_segments`` entry for InteriorAnalyzer: labels + prompts (main_API.py:161)."""
    return {WORKER_SEGMENT: (list(WORKER_STYLES), [f"wnętrze w stylu {s}" for s in WORKER_STYLES])}


def dominant_style(room_analyses: list[dict]) -> dict:
    if not room_analyses:
        return {"style": None, "confidence": 0.0, "votes": {}}
    votes: dict[str, float] = defaultdict(float)
    for r in room_analyses:
        votes[r["style"]] += float(r["style_confidence"])
    best = max(votes.items(), key=lambda kv: (kv[1], kv[0]))
    return {"style": best[0], "confidence": best[1] / len(room_analyses),
            "votes": dict(sorted(votes.items(), key=lambda kv: -kv[1]))}


def room_distribution(room_analyses: list[dict]) -> dict:
    c = Counter(r["room_type"] for r in room_analyses)
    return dict(sorted(c.items(), key=lambda kv: (-kv[1], str(kv[0]))))


class InMemoryDatabase:
    """LocalDatabaseClient's interface (main_API.py:18-120) over dicts."""

    def __init__(self, apartments: dict):
        # apartments: {apartment_id: {"title": str, "images": [{"_id", "url"}]}}
        self.apartments = {k: dict(v) for k, v in apartments.items()}
        self.images = {img["_id"]: dict(img, apartment_id=k, analysis_status="pending")
                       for k, v in apartments.items() for img in v["images"]}
        self.analysis_results = {}

    def get_pending_apartments(self):
        pend = defaultdict(int)
        for img in self.images.values():
            if img["analysis_status"] == "pending":
                pend[img["apartment_id"]] += 1
        return [{"_id": k, "title": self.apartments[k].get("title", ""), "pending_count": n}
                for k, n in pend.items()]

    def get_apartment_with_images(self, apartment_id):
        apt = self.apartments.get(apartment_id)
        if apt is None:
            return None
        imgs = [i for i in self.images.values()
                if i["apartment_id"] == apartment_id and i["analysis_status"] == "pending"]
        return {"id": apartment_id, "title": apt.get("title", ""), "images": imgs}

    def update_image_analysis(self, image_id, room_type, style, confidence):
        self.images[image_id].update(room_type=room_type, style=style, analysis_status="completed",
                                     analysis_confidence=confidence)

    def save_apartment_analysis(self, apartment_id, analysis_result):
        self.analysis_results[apartment_id] = {
            "overall_style": analysis_result["overall_style"],
            "room_distribution": analysis_result["room_distribution"],
            "analyzed_images": analysis_result["interior_images"],
            "total_images": analysis_result["total_images"]}


class DatabaseStyleRoomAnalyzer:
    """main_API.py:129-290 on an InteriorAnalyzer built with ``extra_segments=
    worker_style_segment()`` (one GPU pass per batch for detector, room type and style)."""

    def __init__(self, db_client, analyzer, image_loader=load_image):
        if WORKER_SEGMENT not in analyzer.table.segments:
            raise ValueError("analyzer needs extra_segments=worker_style_segment()")
        self.db = db_client
        self.analyzer = analyzer
        self.styles = list(WORKER_STYLES)
        self.load_image = image_loader

    def _analyze_styles_batch(self, images, batch_size: int = 8) -> list[dict]:
        res = self.analyzer.predict_batch(images, batch_size, filter_interiors=False)
        return [{"style": r["analysis"][WORKER_SEGMENT][0][0],
                 "confidence": r["analysis"][WORKER_SEGMENT][0][1]} for r in res]

    def _calculate_dominant_style(self, room_analyses):
        return dominant_style(room_analyses)

    def _calculate_room_distribution(self, room_analyses):
        return room_distribution(room_analyses)

    def analyze_apartment_from_db(self, apartment_id, batch_size: int = 8,
                                  confidence_threshold: float = 0.3):
        data = self.db.get_apartment_with_images(apartment_id)
        if not data or not data.get("images"):
            return None
        loaded = []
        for img in data["images"]:
            try:
                loaded.append((img, self.load_image(img["url"])))
            except Exception:
                continue  # main_API.py:204-205: skipped, left pending
        preds = self.analyzer.predict_batch([im for _, im in loaded], batch_size,
                                            confidence_threshold, filter_interiors=True) if loaded else []
        room_analyses = []
        for (img, _), r in zip(loaded, preds):
            if not r["is_interior"]:
                self.db.update_image_analysis(img["_id"], "not_interior", "unknown", 0.0)
                continue
            style, conf = r["analysis"][WORKER_SEGMENT][0]
            self.db.update_image_analysis(img["_id"], r["room_type"], style, conf)
            room_analyses.append({"room_type": r["room_type"], "style": style,
                                  "style_confidence": conf,
                                  "detection_confidence": r["interior_confidence"]})
        if not room_analyses:
            return None
        result = {"apartment_id": apartment_id, "total_images": len(data["images"]),
                  "interior_images": len(room_analyses),
                  "overall_style": self._calculate_dominant_style(room_analyses),
                  "room_distribution": self._calculate_room_distribution(room_analyses)}
        self.db.save_apartment_analysis(apartment_id, result)
        return result


def process_apartments_pipeline(db_client, analyzer, max_apartments=None, batch_size: int = 8,
                                confidence_threshold: float = 0.3) -> dict:
    """main_API.py:295-345 without the Mongo connection / JSON export: returns
    {apartment_id: result or None}."""
    pending = db_client.get_pending_apartments()
    if max_apartments:
        pending = pending[:max_apartments]
    w = DatabaseStyleRoomAnalyzer(db_client, analyzer)
    out = {}
    for apt in pending:
        try:
            out[apt["_id"]] = w.analyze_apartment_from_db(apt["_id"], batch_size, confidence_threshold)
        except Exception:  # main_API.py:339-340
            out[apt["_id"]] = None
    return out
