"""The GPU path against the reference harness's own outputs (tests/golden/harness_*.json).

The fixtures are the dicts that main.py's CachedInteriorAnalyzer.analyze_images_batch and
InteriorImageDetector.is_interior_image returned (reference code, oracle mirror as ``clip``,
seeded weights, shipped comprehensive_lora.pth, PYTHONHASHSEED=0). Here the same images go
through this package's InteriorAnalyzer (host preprocess -> libclipvit_hip.so classify, fp16
MFMA) with the same seeded weights, label order and text matrices, and must give the same
result dicts: identical flags/labels (where the reference's top-k margin exceeds the
tolerance), probabilities within 2e-3.
"""
import json

import numpy as np
import pytest

from interior_amd.analyzer import InteriorAnalyzer

pytestmark = pytest.mark.gpu
PROB_TOL = 2e-3


def _load(golden_dir, tag):
    js = json.loads((golden_dir / f"harness_{tag}.json").read_text())
    npz = np.load(golden_dir / f"harness_{tag}.npz")
    T = {"detector": npz["T_det"], **{c: npz[f"T_{c}"] for c in js["segments"]}}
    return js, T


def _compare(ref, got, where):
    assert got["is_interior"] == ref["is_interior"], where
    assert abs(got["interior_confidence"] - ref["interior_confidence"]) < PROB_TOL, where
    assert got["detected_category"] == ref["detected_category"], where
    assert got["reason"].split(" (")[0] == ref["reason"].split(" (")[0], where
    assert set(got["analysis"]) == set(ref["analysis"]), where
    for cat, rlist in ref["analysis"].items():
        glist = got["analysis"][cat]
        assert len(glist) == len(rlist)
        for j, ((gl, gp), (rl, rp)) in enumerate(zip(glist, rlist)):
            assert abs(gp - rp) < PROB_TOL, (where, cat, j, gp, rp)
            nxt = rlist[j + 1][1] if j + 1 < len(rlist) else -1.0
            prv = rlist[j - 1][1] if j > 0 else 2.0
            if rp - nxt > 2 * PROB_TOL and prv - rp > 2 * PROB_TOL:
                assert gl == rl, (where, cat, j, gl, rl)


@pytest.mark.parametrize("tag", ["vitb32", "vitb16"])
def test_analyzer_reproduces_reference_harness(gpu, golden_dir, tag):
    js, T = _load(golden_dir, tag)
    an = InteriorAnalyzer(model=js["model"], compute_dtype="fp16", device=0,
                          categories=js["categories"], text_features=T,
                          weights_seed=js["weights_seed"], max_batch=16)
    paths = [str(golden_dir / "images" / n) for n in js["images"]]
    for flt, key in ((True, "filter_true"), (False, "filter_false")):
        res = an.analyze_images_batch(paths, batch_size=16, filter_interiors=flt,
                                      confidence_threshold=0.3)
        for p, name in zip(paths, js["images"]):
            _compare(js[key][name], res[p], (tag, key, name))
    from PIL import Image
    for name in js["images"]:
        img = Image.open(golden_dir / "images" / name).convert("RGB")
        ok, conf, cat = an.is_interior_image(img, 0.3)
        r = js["detector"][name]
        assert ok == r[0] and cat == r[2] and abs(conf - r[1]) < PROB_TOL
        pred = an.predict(img)
        assert set(pred) >= {"is_interior", "interior_confidence", "detected_category", "room_type",
                             "style", "confidence", "attributes", "reason"}
    an.engine.close()
