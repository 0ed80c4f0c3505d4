"""Generate the committed golden fixtures from the REFERENCE'S OWN harness code.

Runs only in the build container (it imports /root/reference/main.py, which never travels to
the GPU box). The real ``clip`` package and weights are absent offline, so ``sys.modules['clip']``
is the oracle's OpenAI-CLIP module mirror (oracle/clip_module.py) carrying seeded synthetic
weights; everything AFTER ``clip.load`` is the reference's code, unmodified:

  * LoRA binding facts: main.py ``replace_linears_with_lora`` + ``load_lora_weights_to_model``
    (main.py:62-113) on the mirror with the shipped ``lora_models/comprehensive_lora*.pth``
    -> lora_binding.json (counts, missing names, vision delta, dead out_proj delta).
  * Harness outputs: main.py ``CachedInteriorAnalyzer`` (use_lora=True, the shipped checkpoint,
    CPU) + ``InteriorImageDetector`` on interior_sample.jpg and four dataset images, with
    PYTHONHASHSEED=0 (the label order depends on it) -> harness_<model>.json
    (result dicts, label order) + harness_<model>.npz (text matrices, oracle logits).
  * Copies the input JPEGs and interior_dataset.json (data files the reference reads at run
    time) into tests/golden/ so the GPU-box tests need nothing from /root/reference.

    python tests/golden/make_golden.py            # re-executes itself with PYTHONHASHSEED=0
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys
import types
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
REF = Path("/root/reference")
IMAGES = ["interior_sample.jpg", "dataset_images/interior5.jpg", "dataset_images/interior6.jpg",
          "dataset_images/interior7.jpg", "dataset_images/interior8.jpg"]
MODELS = ["ViT-B/32", "ViT-B/16"]
WEIGHT_SEED = 0


def _setup():
    sys.path.insert(0, str(ROOT))
    import amd_pkg
    amd_pkg.load()
    import torch
    from interior_amd.config import get_config
    from interior_amd.weights import synthetic_state_dict, state_dict_checksum
    from oracle.clip_module import make_clip_shim
    sds = {m: synthetic_state_dict(get_config(m), WEIGHT_SEED) for m in MODELS}
    shim = make_clip_shim(sds)
    sys.modules["clip"] = shim
    sys.path.insert(0, str(REF))
    import main as ref_main  # the reference harness
    return torch, ref_main, shim, sds, state_dict_checksum


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
        txt_before = None
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


def harness(torch, ref_main, shim, model_name):
    import numpy as np
    from PIL import Image
    base_load = shim.base_load  # every clip.load(...) of the harness gets `model_name` weights
    ref_main.clip.load = lambda name, device="cpu", **kw: base_load(model_name, device)
    cwd = os.getcwd()
    os.chdir(REF)  # main.py:264 reads interior_dataset.json relative to the CWD
    try:
        an = ref_main.CachedInteriorAnalyzer(use_lora=True,
                                             lora_weights_path="lora_models/comprehensive_lora.pth",
                                             lora_rank=4, lora_alpha=8, device="cpu")
        paths = [str(REF / p) for p in IMAGES]
        with torch.no_grad():
            res_f = an.analyze_images_batch(paths, batch_size=16, filter_interiors=True,
                                            confidence_threshold=0.3)
            res_nf = an.analyze_images_batch(paths, batch_size=16, filter_interiors=False)
            det = [list(an.detector.is_interior_image(Image.open(p).convert("RGB"), 0.3)) for p in paths]
            pix = torch.stack([an.preprocess(Image.open(p).convert("RGB")) for p in paths])
            f = an.model.encode_image(pix)
            f = f / f.norm(dim=-1, keepdim=True)
            T = {c: t.float().numpy() for c, t in an.text_features_cache.items()}
            T_det = an.detector.text_features.float().numpy()
            logits = {c: (100.0 * f @ torch.from_numpy(t).t()).numpy() for c, t in T.items()}
            logits["detector"] = (100.0 * f @ torch.from_numpy(T_det).t()).numpy()
    finally:
        os.chdir(cwd)
    key = lambda p: Path(p).name
    out = {
        "model": model_name,
        "weights_seed": WEIGHT_SEED,
        "pythonhashseed": os.environ.get("PYTHONHASHSEED"),
        "images": [Path(p).name for p in IMAGES],
        "categories": an.all_categories,
        "segments": list(T.keys()),
        "detector_categories": an.detector.categories,
        "detector": {Path(p).name: d for p, d in zip(IMAGES, det)},
        "filter_true": {key(k): v for k, v in res_f.items()},
        "filter_false": {key(k): v for k, v in res_nf.items()},
    }
    flat = pix.reshape(len(IMAGES), -1)
    idx = torch.arange(0, flat.shape[1], 151)  # 997 fixed sample positions per image
    arrays = {"T_det": T_det, **{f"T_{c}": t for c, t in T.items()},
              **{f"logits_{c}": v for c, v in logits.items()},
              "pixels_sum": flat.double().sum(1).numpy(), "pixels_abs_sum": flat.double().abs().sum(1).numpy(),
              "pixels_sample": flat[:, idx].numpy(), "pixels_sample_idx": idx.numpy()}
    return out, arrays


def main():
    if os.environ.get("PYTHONHASHSEED") != "0":
        env = dict(os.environ, PYTHONHASHSEED="0")
        sys.exit(subprocess.call([sys.executable, __file__], env=env))
    import numpy as np
    torch, ref_main, shim, sds, checksum = _setup()
    (HERE / "images").mkdir(exist_ok=True)
    for p in IMAGES:
        shutil.copyfile(REF / p, HERE / "images" / Path(p).name)
    shutil.copyfile(REF / "interior_dataset.json", HERE / "interior_dataset.json")
    facts = {"weights": {m: {"seed": WEIGHT_SEED, "checksum": checksum(sds[m])} for m in MODELS},
             "checkpoints": [lora_facts(torch, ref_main, shim, c)
                             for c in ("comprehensive_lora.pth", "comprehensive_lora_new.pth")]}
    (HERE / "lora_binding.json").write_text(json.dumps(facts, indent=1, ensure_ascii=False))
    for m in MODELS:
        out, arrays = harness(torch, ref_main, shim, m)
        tag = m.replace("/", "").replace("-", "").lower()
        (HERE / f"harness_{tag}.json").write_text(json.dumps(out, indent=1, ensure_ascii=False))
        np.savez_compressed(HERE / f"harness_{tag}.npz", **arrays)
        print("wrote", tag)


if __name__ == "__main__":
    main()
