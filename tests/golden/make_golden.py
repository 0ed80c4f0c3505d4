"""Generate the committed golden fixtures from the REFERENCE'S OWN harness code.

Runs only in the build container (it imports /root/reference/main.py, which never travels to
the GPU box). The real ``clip`` package and weights are absent offline, so ``sys.modules['clip']``
is the oracle's OpenAI-CLIP module mirror (oracle/clip_module.py) carrying seeded synthetic
weights (vision tower AND text tower, OpenAI names) and a ``clip.tokenize`` over a BPE merges
list learned from the reference's own prompt vocabulary; everything AFTER ``clip.load`` /
``clip.tokenize`` is the reference's code, unmodified:

  * LoRA binding facts: main.py ``replace_linears_with_lora`` + ``load_lora_weights_to_model``
    (main.py:62-113) on the mirror with the shipped ``lora_models/comprehensive_lora*.pth``
    -> lora_binding.json (counts, missing names, vision delta, dead out_proj delta).
  * Harness outputs, for BOTH models (ViT-B/32, ViT-B/16) x BOTH shipped checkpoints: main.py
    ``CachedInteriorAnalyzer(use_lora=True, <checkpoint>)`` + ``InteriorImageDetector`` on
    interior_sample.jpg and ALL 150 dataset images (75 of them larger than 256 px, up to
    2592x1944: the downscale path; interior87.jpg is the image listed twice with conflicting
    labels in interior_dataset.json), PYTHONHASHSEED=0 (label order)
    -> harness_<model>_<ckpt>.json (result dicts of analyze_images_batch with and without the
    interior filter, is_interior_image per image, label order) + harness_<model>_<ckpt>.npz
    (the harness's 100*cos logits [151, 40 + C], its L2-normalised image features and pixel
    checksums) + text_<ckpt>.npz (the detector's and the analyzer's cached text matrices), and
    the single-image surface: analyze_image_from_url on the first 16 images, filter on / off.
  * The same harness calls at CLIP's logit scale: after the analyzer is
    built, ``an.text_features_cache`` and ``an.detector.text_features`` are overwritten with
    rows normalise(0.3 f + 0.95 r) (f = the reference's fp32 image features, r seeded random
    unit vectors: max|logit| ~ 30); everything downstream is main.py's code
    -> harness_<model>_<ckpt>_clipscale.{json,npz} + clipscale_text_<model>.npz.
  * Copies the input JPEGs, interior_dataset.json and the two LoRA checkpoints (data files the
    reference reads at run time) into tests/golden/ so the GPU-box tests need nothing from
    /root/reference; writes the learned merges to bpe_merges.txt.

    python tests/golden/make_golden.py            # re-executes itself with PYTHONHASHSEED=0
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
REF = Path("/root/reference")
IMAGES = ["interior_sample.jpg"] + [f"dataset_images/interior{i}.jpg" for i in range(1, 151)]
MODELS = ["ViT-B/32", "ViT-B/16"]
CKPTS = ["comprehensive_lora.pth", "comprehensive_lora_new.pth"]
WEIGHT_SEED = 0
TEXT_SEED = 1
N_MERGES = 600


def tag_of(model, ckpt):
    return model.replace("/", "").replace("-", "").lower() + "_" + ckpt.replace("comprehensive_", "").replace(".pth", "")


def _setup():
    sys.path.insert(0, str(ROOT))
    import amd_pkg
    amd_pkg.load()
    import torch
    from interior_amd import labels as L
    from interior_amd import tokenizer as TK
    from interior_amd.config import TextConfig, get_config
    from interior_amd.weights import state_dict_checksum, synthetic_state_dict, synthetic_text_state_dict
    from oracle.clip_module import make_clip_shim, read_merges_file
    # merges learned from the reference's own prompts (detector + analyzer label prompts)
    cats = L.extract_categories(L.load_training_data(REF / "interior_dataset.json"))
    corpus = L.build_label_table(cats).all_texts
    merges = TK.learn_merges(corpus, N_MERGES)
    (HERE / "bpe_merges.txt").write_text("#version: learned from the reference's label prompts (tests/golden/make_golden.py)\n"
                                        + "\n".join(" ".join(m) for m in merges) + "\n", encoding="utf-8")
    merges = read_merges_file(HERE / "bpe_merges.txt")
    tc = TextConfig(vocab=514 + len(merges))
    text_sd = synthetic_text_state_dict(tc, TEXT_SEED)
    sds = {m: {**synthetic_state_dict(get_config(m), WEIGHT_SEED), **text_sd} for m in MODELS}
    shim = make_clip_shim(sds, merges)
    # the oracle's tokenize (HF tokenizers) and the product tokenizer agree on every prompt
    mine = TK.SimpleTokenizer(bpe_path=HERE / "bpe_merges.txt")
    assert (shim.tokenize(corpus).numpy() == mine.tokenize(corpus)).all()
    sys.modules["clip"] = shim
    sys.path.insert(0, str(REF))
    import main as ref_main  # the reference harness
    checks = {"weights": {m: {"seed": WEIGHT_SEED, "checksum": state_dict_checksum(synthetic_state_dict(get_config(m), WEIGHT_SEED))}
                          for m in MODELS},
              "text_weights": {"seed": TEXT_SEED, "vocab": tc.vocab, "checksum": state_dict_checksum(text_sd)}}
    return torch, ref_main, shim, checks


def lora_facts(torch, ref_main, shim, ckpt_name):
    model, _ = shim.load("ViT-B/16", "cpu")
    px = torch.randn(2, 3, 224, 224, generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        before = model.encode_image(px)
    replaced = ref_main.replace_linears_with_lora(model, rank=4, alpha=8)
    loaded, missing = ref_main.load_lora_weights_to_model(model, str(REF / "lora_models" / ckpt_name))
    with torch.no_grad():
        after = model.encode_image(px)
        # the vision out_proj wrappers are bypassed by nn.MultiheadAttention: prove it
        for i in range(12):
            model.visual.transformer.resblocks[i].attn.out_proj.lora.lora_B.fill_(1.0)
        dead = model.encode_image(px)
    ckpt = torch.load(REF / "lora_models" / ckpt_name, map_location="cpu", weights_only=True)
    return {
        "checkpoint": ckpt_name,
        "replaced_linears": len(replaced),
        "loaded": loaded,
        "missing": len(missing),
        "missing_names": missing,
        "vision_delta_max_abs": float((after - before).abs().max()),
        "dead_out_proj_delta_max_abs": float((dead - after).abs().max()),
        "ckpt_keys": list(ckpt.keys()),
        "ckpt_shapes": {k: list(v.shape) for k, v in ckpt.items()},
        "ckpt_dtype": str(next(iter(ckpt.values())).dtype),
    }


SINGLE = IMAGES[:16]     # the single-image surface (analyze_image_from_url, bs 1)
CLIP_SCALE_SEED = 42


def _run_harness(torch, ref_main, an, paths):
    """The reference's own calls on one analyzer: analyze_images_batch (filter on / off),
    is_interior_image per image, analyze_image_from_url on SINGLE (filter on / off; the URL
    loader is stubbed by a local-file open, the one network call in the path)."""
    from PIL import Image
    with torch.no_grad():
        res_f = an.analyze_images_batch(paths, batch_size=16, filter_interiors=True,
                                        confidence_threshold=0.3)
        res_nf = an.analyze_images_batch(paths, batch_size=16, filter_interiors=False)
        det = [list(an.detector.is_interior_image(Image.open(p).convert("RGB"), 0.3)) for p in paths]
        loader = ref_main.URLImageLoader.load_image_from_url
        ref_main.URLImageLoader.load_image_from_url = staticmethod(lambda url, timeout=30: Image.open(url).convert("RGB"))
        try:
            single = {flt: {Path(p).name: an.analyze_image_from_url(str(REF / p), filter_interiors=flt) for p in SINGLE}
                      for flt in (True, False)}
        finally:
            ref_main.URLImageLoader.load_image_from_url = loader
    key = lambda p: Path(p).name
    return {"detector": {key(p): d for p, d in zip(IMAGES, det)},
            "filter_true": {key(k): v for k, v in res_f.items()},
            "filter_false": {key(k): v for k, v in res_nf.items()},
            "single_filter_true": single[True], "single_filter_false": single[False]}


def clip_scale_text(torch, f, sizes):
    """CLIP-scale label rows: row c = normalise(0.3 f[c mod n] +
    0.95 r_c) with f = the reference's fp32 L2-normalised features of the fixture images and r_c
    seeded random unit vectors, so every image's best labels sit at 100 cos ~ 30 like real CLIP.
    Returns one matrix per segment (sizes = rows per segment, detector first)."""
    g = torch.Generator().manual_seed(CLIP_SCALE_SEED)
    C = sum(sizes)
    r = torch.nn.functional.normalize(torch.randn(C, f.shape[1], generator=g, dtype=torch.float64), dim=-1)
    T = 0.3 * f.double()[torch.arange(C) % f.shape[0]] + 0.95 * r
    T = (T / T.norm(dim=-1, keepdim=True)).float()
    return list(torch.split(T, sizes))


def harness(torch, ref_main, shim, model_name, ckpt, clip_scale=True):
    from PIL import Image
    base_load = shim.base_load  # every clip.load(...) of the harness gets `model_name` weights
    ref_main.clip.load = lambda name, device="cpu", **kw: base_load(model_name, device)
    cwd = os.getcwd()
    os.chdir(REF)  # main.py:264 reads interior_dataset.json relative to the CWD
    try:
        an = ref_main.CachedInteriorAnalyzer(use_lora=True, lora_weights_path=f"lora_models/{ckpt}",
                                             lora_rank=4, lora_alpha=8, device="cpu")
        paths = [str(REF / p) for p in IMAGES]
        with torch.no_grad():
            pix = torch.stack([an.preprocess(Image.open(p).convert("RGB")) for p in paths])
            f = torch.cat([an.model.encode_image(pix[a:a + 16]) for a in range(0, len(paths), 16)])
            f = f / f.norm(dim=-1, keepdim=True)
        runs = {}
        for scale in ((False, True) if clip_scale else (False,)):
            if scale:  # the harness's caches replaced by CLIP-scale rows; all else is main.py's code
                segs = list(an.text_features_cache.keys())
                mats = clip_scale_text(torch, f, [len(an.detector.categories)] +
                                       [an.text_features_cache[c].shape[0] for c in segs])
                an.detector.text_features = mats[0]
                for c, m in zip(segs, mats[1:]):
                    an.text_features_cache[c] = m
            res = _run_harness(torch, ref_main, an, paths)
            T = {c: t.float().numpy() for c, t in an.text_features_cache.items()}
            T_det = an.detector.text_features.float().numpy()
            logits = 100.0 * f @ torch.cat([torch.from_numpy(T_det)] + [torch.from_numpy(T[c]) for c in T]).t()
            runs[scale] = (res, T, T_det, logits)
    finally:
        os.chdir(cwd)
    outs = {}
    for scale, (res, T, T_det, logits) in runs.items():
        out = {
            "model": model_name,
            "checkpoint": ckpt,
            "weights_seed": WEIGHT_SEED,
            "text_seed": TEXT_SEED,
            "clip_scale_seed": CLIP_SCALE_SEED if scale else None,
            "pythonhashseed": os.environ.get("PYTHONHASHSEED"),
            "images": [Path(p).name for p in IMAGES],
            "categories": an.all_categories,
            "segments": list(T.keys()),
            "detector_categories": an.detector.categories,
            **res,
        }
        flat = pix.reshape(len(IMAGES), -1)
        idx = torch.arange(0, flat.shape[1], 151)  # 997 fixed sample positions per image
        arrays = {"logits": logits.numpy(), "features": f.numpy(),
                  "pixels_sum": flat.double().sum(1).numpy(), "pixels_abs_sum": flat.double().abs().sum(1).numpy(),
                  "pixels_sample": flat[:, idx].numpy(), "pixels_sample_idx": idx.numpy()}
        text = {"T_det": T_det, **{f"T_{c}": t for c, t in T.items()}}
        outs[scale] = (out, arrays, text)
    return outs


def main():
    if os.environ.get("PYTHONHASHSEED") != "0":
        env = dict(os.environ, PYTHONHASHSEED="0")
        sys.exit(subprocess.call([sys.executable, __file__] + sys.argv[1:], env=env))
    import numpy as np
    torch, ref_main, shim, checks = _setup()
    (HERE / "images").mkdir(exist_ok=True)
    (HERE / "lora").mkdir(exist_ok=True)
    for p in IMAGES:
        shutil.copyfile(REF / p, HERE / "images" / Path(p).name)
    for c in CKPTS:
        shutil.copyfile(REF / "lora_models" / c, HERE / "lora" / c)
    shutil.copyfile(REF / "interior_dataset.json", HERE / "interior_dataset.json")
    facts = {**checks, "checkpoints": [lora_facts(torch, ref_main, shim, c) for c in CKPTS]}
    (HERE / "lora_binding.json").write_text(json.dumps(facts, indent=1, ensure_ascii=False))
    for c in CKPTS:
        ck = c.replace("comprehensive_", "").replace(".pth", "")
        for m in MODELS:
            outs = harness(torch, ref_main, shim, m, c)
            tag = tag_of(m, c)
            for scale, (out, arrays, text) in outs.items():
                sfx = "_clipscale" if scale else ""
                (HERE / f"harness_{tag}{sfx}.json").write_text(json.dumps(out, ensure_ascii=False))
                if scale:  # features and pixels are those of the flat run; the CLIP-scale rows per model
                    np.savez_compressed(HERE / f"harness_{tag}{sfx}.npz", logits=arrays["logits"])
                    mtag = tag_of(m, c).split("_")[0]
                    np.savez_compressed(HERE / f"clipscale_text_{mtag}.npz", **text)
                else:
                    np.savez_compressed(HERE / f"harness_{tag}.npz", **arrays)
                    np.savez_compressed(HERE / f"text_{ck}.npz", **text)
            print("wrote", tag, flush=True)


if __name__ == "__main__":
    main()
