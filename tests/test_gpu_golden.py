"""The GPU path against the reference harness's own outputs (tests/golden/harness_*).

The fixtures are what main.py's CachedInteriorAnalyzer (use_lora=True with each shipped
checkpoint) and InteriorImageDetector returned — reference code, the oracle's OpenAI-CLIP
mirror as ``clip``, seeded weights, PYTHONHASHSEED=0 — on interior_sample.jpg and all 150
dataset images (75 larger than 256 px: the downscale path; interior87.jpg, listed twice with
conflicting labels in interior_dataset.json), plus the harness's 100*cos logits. Here the same
JPEGs go through this package's InteriorAnalyzer (GPU preprocess -> libclipvit_hip.so classify,
fp16 MFMA operands) built with ``use_lora=True`` on the same shipped-format checkpoint:

* logits, with the harness's own text matrices: per image max|dlogit| / max|logit_ref|. These
  synthetic text features are nearly orthogonal to the image features (max|logit| 4.6-9 for
  ViT-B/32, 10-16 for B/16, against ~20-35 for real CLIP), which inflates this relative
  measure: the assertion is HARNESS_TOL, and the distribution is printed (DESIGN.md §3 has the
  error-source analysis: fp16 rounding of the Linear weights alone gives 8.6e-4 here);
* logits at CLIP's real logit scale (text rows = 0.3 x an image's reference feature + noise,
  max|logit| ~ 30) on all 151 images: <= 1e-3, the north-star bar;
* labels: the per-segment argmax and every top-5 label identical wherever the reference's
  margin to the neighbouring label exceeds twice the measured error; the near-tie exemptions
  are counted and printed (and bounded);
* the result dicts of analyze_images_batch (filter on / off) and is_interior_image;
* the text caches rebuilt on the GPU text tower (clip.tokenize over the committed BPE merges,
  the checkpoint's text-MLP LoRA merged for the analyzer prompts) against the harness's.
"""
import json

import numpy as np
import pytest
from PIL import Image

from interior_amd import labels as L
from interior_amd.analyzer import InteriorAnalyzer
from interior_amd.config import TextConfig
from interior_amd.tokenizer import SimpleTokenizer
from interior_amd.weights import synthetic_text_state_dict

pytestmark = pytest.mark.gpu
LOGIT_TOL = 1e-3
HARNESS_TOL = 1.5e-3
PROB_TOL = 2e-3
TEXT_TOL = 2e-3
CASES = [(m, c) for m in ("vitb32", "vitb16") for c in ("lora", "lora_new")]


def _load(golden_dir, model, ckpt):
    js = json.loads((golden_dir / f"harness_{model}_{ckpt}.json").read_text())
    logits = np.load(golden_dir / f"harness_{model}_{ckpt}.npz")["logits"]
    tz = np.load(golden_dir / f"text_{ckpt}.npz")
    T = {"detector": tz["T_det"], **{c: tz[f"T_{c}"] for c in js["segments"]}}
    return js, logits, T


def _columns(js, table):
    """Fixture column of every (segment, label) of the analyzer's table (keyed by label string)."""
    ref_cols, off = {}, 0
    for s, labs in [("detector", js["detector_categories"])] + [(c, js["categories"][c]) for c in js["segments"]]:
        for j, l in enumerate(labs):
            ref_cols[(s, l)] = off + j
        off += len(labs)
    return np.array([ref_cols[(s, l)] for s, labs in zip(table.segments, table.labels) for l in labs])


@pytest.fixture(scope="module")
def images(golden_dir):
    js = json.loads((golden_dir / "harness_vitb32_lora.json").read_text())
    return js["images"], [Image.open(golden_dir / "images" / n).convert("RGB") for n in js["images"]]


def _seg_probs(logits_row, js, cat):
    """The reference's softmax over one analyzer segment (from the fixture logits)."""
    off = len(js["detector_categories"])
    for c in js["segments"]:
        n = len(js["categories"][c])
        if c == cat:
            z = logits_row[off:off + n].astype(np.float64)
            e = np.exp(z - z.max())
            return e / e.sum()
        off += n
    raise KeyError(cat)


def _compare(ref, got, where, err, ref_logits, js):
    """Result dict vs the reference's: flags and probabilities, and every top-5 label wherever
    the reference's probability margin to the labels ranked next to it (from its full segment
    softmax, so the 5th entry is compared against the 6th too) exceeds `err`. Returns the
    number of near-tie label swaps."""
    assert got["is_interior"] == ref["is_interior"], where
    assert abs(got["interior_confidence"] - ref["interior_confidence"]) < PROB_TOL, where
    tie = int(got["detected_category"] != ref["detected_category"])  # near-tie only (logit test)
    assert got["reason"].split(":")[0] == ref["reason"].split(":")[0], where
    assert set(got["analysis"]) == set(ref["analysis"]), where
    for cat, rlist in ref["analysis"].items():
        glist = got["analysis"][cat]
        assert len(glist) == len(rlist)
        srt = np.sort(_seg_probs(ref_logits, js, cat))[::-1]
        for j, ((gl, gp), (rl, rp)) in enumerate(zip(glist, rlist)):
            assert abs(gp - rp) < PROB_TOL, (where, cat, j, gp, rp)
            nxt = srt[j + 1] if j + 1 < len(srt) else -1.0
            prv = srt[j - 1] if j > 0 else 2.0
            if min(srt[j] - nxt, prv - srt[j]) > err:
                assert gl == rl, (where, cat, j, gl, rl)
            elif gl != rl:
                tie += 1
    return tie


@pytest.mark.parametrize("model,ckpt", CASES)
def test_logits_and_results_match_reference_harness(gpu, golden_dir, images, model, ckpt):
    js, ref, T = _load(golden_dir, model, ckpt)
    names, imgs = images
    assert js["images"] == names and js["detector_categories"] == L.DETECTOR_CATEGORIES
    an = InteriorAnalyzer(model=js["model"], device=0, categories=js["categories"], text_features=T,
                          weights_seed=js["weights_seed"], max_batch=64, use_lora=True,
                          lora_weights_path=str(golden_dir / "lora" / js["checkpoint"]))
    assert an.engine.compute_dtype == "fp16" and an.lora_report["loaded"] == 48
    try:
        got = an.logits(imgs)
        cols = _columns(js, an.table)
        r = ref[:, cols]
        rel = np.abs(got - r).max(axis=1) / np.abs(r).max(axis=1)
        worst = float(rel.max())
        print(f"\n[{model}/{ckpt}] rel logit err over {len(rel)} images: worst {worst:.2e} "
              f"({names[int(rel.argmax())]}), p95 {np.percentile(rel, 95):.2e}, median {np.median(rel):.2e}, "
              f"> 1e-3: {int((rel > 1e-3).sum())}")
        assert worst <= HARNESS_TOL, (model, ckpt, worst, names[int(rel.argmax())])
        # per-segment argmax: identical unless the reference's top-1/top-2 margin is within
        # twice this image's absolute logit error
        off, exempt, checked = an.table.offsets, 0, 0
        for i in range(len(names)):
            e = float(np.abs(got[i] - r[i]).max())
            for s in range(len(off) - 1):
                rs, gs = r[i, off[s]:off[s + 1]], got[i, off[s]:off[s + 1]]
                top2 = np.sort(rs)[-2:]
                checked += 1
                if top2[1] - top2[0] > 2 * e:
                    assert rs.argmax() == gs.argmax(), (names[i], an.table.segments[s])
                else:
                    exempt += 1
        print(f"[{model}/{ckpt}] argmax checks {checked - exempt}/{checked}, near-tie exemptions {exempt}")
        assert exempt <= 0.02 * checked
        # the result dicts (probabilities of 100*cos softmaxes: err in p <= ~ |dlogit|)
        paths = [str(golden_dir / "images" / n) for n in names]
        ties = 0
        for flt, key in ((True, "filter_true"), (False, "filter_false")):
            res = an.analyze_images_batch(paths, batch_size=64, filter_interiors=flt, confidence_threshold=0.3)
            for i, (p, n) in enumerate(zip(paths, names)):
                ties += _compare(js[key][n], res[p], (model, ckpt, key, n), 2 * PROB_TOL, ref[i], js)
        for n, img in zip(names[:24], imgs[:24]):
            ok, conf, cat = an.is_interior_image(img, 0.3)
            rd = js["detector"][n]
            assert ok == rd[0] and abs(conf - rd[1]) < PROB_TOL, n
            ties += cat != rd[2]
        print(f"[{model}/{ckpt}] result-dict near-tie label swaps: {ties}")
        assert ties <= 0.01 * len(names) * 12
    finally:
        an.engine.close()


@pytest.mark.parametrize("ckpt", ["lora", "lora_new"])
def test_text_caches_from_gpu_text_tower(gpu, golden_dir, images, ckpt):
    """T rebuilt on the GPU text tower: detector prompts through the base tower
    (main.py:179-182), analyzer prompts through the checkpoint's LoRA tower (main.py:296-311);
    then the whole path (GPU text + GPU image) against the harness logits."""
    js, ref, T = _load(golden_dir, "vitb32", ckpt)
    facts = json.loads((golden_dir / "lora_binding.json").read_text())["text_weights"]
    tok = SimpleTokenizer(bpe_path=golden_dir / "bpe_merges.txt")
    assert tok.vocab_size == facts["vocab"]
    text_sd = synthetic_text_state_dict(TextConfig(vocab=tok.vocab_size), facts["seed"])
    an = InteriorAnalyzer(model=js["model"], device=0, categories=js["categories"],
                          weights_seed=js["weights_seed"], max_batch=64, use_lora=True,
                          lora_weights_path=str(golden_dir / "lora" / js["checkpoint"]),
                          text_state_dict=text_sd, tokenizer=tok)
    try:
        assert an.lora_report["text_adapters"] == 24
        Tref = np.concatenate([T[s] for s in an.table.segments], axis=0)
        rel = np.abs(an.text_matrix - Tref).max(axis=1) / np.abs(Tref).max(axis=1)
        assert rel.max() <= TEXT_TOL, float(rel.max())
        names, imgs = images
        got = an.logits(imgs[:32])
        r = ref[:32][:, _columns(js, an.table)]
        err = float((np.abs(got - r).max(axis=1) / np.abs(r).max(axis=1)).max())
        print(f"\n[{ckpt}] text rows max rel err {rel.max():.2e}; GPU text + image logits {err:.2e}")
        assert err <= 3 * LOGIT_TOL  # the fp16 text tower adds ~1.5e-3 (T rows within TEXT_TOL)
    finally:
        an.engine.close()


@pytest.mark.parametrize("model", ["vitb32", "vitb16"])
def test_logits_at_clip_scale_meet_bar_on_all_images(gpu, golden_dir, images, model):
    """The north-star bar (1e-3 relative on logits, argmax identical) on all 151 fixture images
    at CLIP's real logit scale: label rows T_c = normalize(0.3 f_ref[c mod 151] + 0.95 r_c)
    (f_ref = the reference harness's L2-normalised features, r_c random unit vectors), so each
    image's best labels sit at 100 cos ~ 30 like real CLIP; reference logits = 100 f_ref T^T."""
    import torch
    js, _, _ = _load(golden_dir, model, "lora")
    f_ref = np.load(golden_dir / f"harness_{model}_lora.npz")["features"].astype(np.float64)
    names, imgs = images
    g = torch.Generator().manual_seed(42)
    C_ = 437
    r = torch.nn.functional.normalize(torch.randn(C_, f_ref.shape[1], generator=g, dtype=torch.float64), dim=-1).numpy()
    T = 0.3 * f_ref[np.arange(C_) % len(names)] + 0.95 * r
    T = (T / np.linalg.norm(T, axis=1, keepdims=True)).astype(np.float32)
    an = InteriorAnalyzer(model=js["model"], device=0, categories=js["categories"], text_features=T,
                          weights_seed=js["weights_seed"], max_batch=64, use_lora=True,
                          lora_weights_path=str(golden_dir / "lora" / js["checkpoint"]))
    try:
        got = an.logits(imgs)
        ref = (100.0 * f_ref @ T.astype(np.float64).T)
        rel = np.abs(got - ref).max(axis=1) / np.abs(ref).max(axis=1)
        print(f"\n[{model}] CLIP-scale logits (max|logit| median {np.median(np.abs(ref).max(axis=1)):.1f}): "
              f"worst rel err {rel.max():.2e}, median {np.median(rel):.2e}")
        assert rel.max() <= LOGIT_TOL, (float(rel.max()), names[int(rel.argmax())])
        off = an.table.offsets
        for i in range(len(names)):
            e = float(np.abs(got[i] - ref[i]).max())
            for s in range(len(off) - 1):
                rs, gs = ref[i, off[s]:off[s + 1]], got[i, off[s]:off[s + 1]]
                top2 = np.sort(rs)[-2:]
                if top2[1] - top2[0] > 2 * e:
                    assert rs.argmax() == gs.argmax(), (names[i], s)
    finally:
        an.engine.close()
