"""The clip-shaped facade driven exactly as main.py drives ``clip`` (no NotImplementedError
anywhere): InteriorImageDetector.__init__ / is_interior_image (main.py:150-222) and
CachedInteriorAnalyzer's LoRA binding, text cache and batched encode (main.py:241-251,
296-311, 436-459) — against the reference harness's fixtures (tests/golden/harness_vitb32_lora.*:
the same seeded weights, the committed BPE merges, the shipped comprehensive_lora.pth)."""
import json

import numpy as np
import pytest
import torch
from PIL import Image

from interior_amd import clip_api as clip
from interior_amd import config as C
from interior_amd.weights import synthetic_state_dict, synthetic_text_state_dict

TEXT_TOL = 2e-3
PROB_TOL = 2e-3


@pytest.mark.gpu
def test_main_py_call_sequence_on_the_facade(gpu, golden_dir):
    js = json.loads((golden_dir / "harness_vitb32_lora.json").read_text())
    ref_logits = np.load(golden_dir / "harness_vitb32_lora.npz")["logits"]
    tz = np.load(golden_dir / "text_lora.npz")
    facts = json.loads((golden_dir / "lora_binding.json").read_text())["text_weights"]
    tok = clip.set_bpe_path(golden_dir / "bpe_merges.txt")
    sd = {**synthetic_state_dict(C.VIT_B32, js["weights_seed"]),
          **synthetic_text_state_dict(C.TextConfig(vocab=tok.vocab_size), facts["seed"])}
    device = "cuda"

    # ---- InteriorImageDetector.__init__ (main.py:150-182) -------------------------------
    model, preprocess = clip.load("ViT-B/32", device=device, weights=sd)
    categories = js["detector_categories"]
    with torch.no_grad():
        text_tokens = clip.tokenize(categories).to(device)
        text_features = model.encode_text(text_tokens)
        text_features = text_features / text_features.norm(dim=-1, keepdim=True)
    assert text_tokens.dtype == torch.int64 and tuple(text_tokens.shape) == (40, 77)
    T = text_features.cpu().numpy()
    assert (np.abs(T - tz["T_det"]).max(axis=1) / np.abs(tz["T_det"]).max(axis=1)).max() < TEXT_TOL

    # ---- is_interior_image (main.py:191-222) at batch 1 --------------------------------
    names = js["images"][:12] + js["images"][100:112]
    for name in names:
        image = Image.open(golden_dir / "images" / name).convert("RGB")
        image_input = preprocess(image).unsqueeze(0).to(device)
        with torch.no_grad():
            image_features = model.encode_image(image_input)
            image_features = image_features / image_features.norm(dim=-1, keepdim=True)
            similarities = (100.0 * image_features @ text_features.T).softmax(dim=-1)
            top_conf, top_idx = similarities[0].topk(1)
            interior_confidence = similarities[0, list(range(0, 11))].sum().item()
            non_interior_confidence = similarities[0, list(range(11, 40))].sum().item()
        is_interior = interior_confidence > non_interior_confidence and top_conf.item() > 0.3
        rd = js["detector"][name]
        assert is_interior == rd[0] and abs(interior_confidence - rd[1]) < PROB_TOL, name
        srt = np.sort(similarities[0].cpu().numpy())
        if srt[-1] - srt[-2] > 2 * PROB_TOL:
            assert categories[top_idx.item()] == rd[2], name
    model.close()

    # ---- CachedInteriorAnalyzer: LoRA binding + text cache (main.py:241-251, 296-311) --------
    model, preprocess = clip.load("ViT-B/32", device=device, weights=sd)
    rep = model.load_lora_checkpoint(golden_dir / "lora" / "comprehensive_lora.pth", 4, 8)
    assert rep == {"loaded": 48, "missing": 96, "vision_adapters": 0, "text_adapters": 24}
    cache = {}
    with torch.no_grad():
        for category, attributes in js["categories"].items():
            if not attributes:
                continue
            texts = [f"{a}" for a in attributes] if category == "room_types" else \
                [f"wnętrze z {a}" for a in attributes]
            tokenized = clip.tokenize(texts).to(device)
            tf = model.encode_text(tokenized)
            cache[category] = tf / tf.norm(dim=-1, keepdim=True)
            ref = tz[f"T_{category}"]
            got = cache[category].cpu().numpy()
            assert (np.abs(got - ref).max(axis=1) / np.abs(ref).max(axis=1)).max() < TEXT_TOL, category

    # ---- batched encode + per-category logits (main.py:436-459), 32 images, batch 16 ----
    imgs = [Image.open(golden_dir / "images" / n).convert("RGB") for n in js["images"][:32]]
    with torch.no_grad():
        feats = []
        for i in range(0, len(imgs), 16):
            batch = torch.stack([preprocess(im) for im in imgs[i:i + 16]]).to(device)
            f = model.encode_image(batch)
            feats.append(f / f.norm(dim=-1, keepdim=True))
        f = torch.cat(feats)
        off = 40
        for category in js["segments"]:
            lg = (100.0 * f @ cache[category].T).cpu().numpy()
            ref = ref_logits[:32, off:off + lg.shape[1]]
            off += lg.shape[1]
            err = np.abs(lg - ref).max(axis=1) / np.abs(ref_logits[:32]).max(axis=1)
            assert err.max() < 3e-3, (category, float(err.max()))  # fp16 text tower adds ~1.5e-3
    model.close()
    clip.set_tokenizer(None)


def test_tokenize_contract(golden_dir):
    """clip.tokenize: [n, 77] int64, sot ... eot, zero padding; too-long prompts raise unless
    truncate (then the last id is eot)."""
    tok = clip.set_bpe_path(golden_dir / "bpe_merges.txt")
    t = clip.tokenize(["living room", "kitchen"])
    assert t.dtype == torch.int64 and tuple(t.shape) == (2, 77)
    assert int(t[0, 0]) == tok.sot and tok.eot in t[0].tolist() and int(t[0, -1]) == 0
    with pytest.raises(RuntimeError):
        clip.tokenize("room " * 100)
    tt = clip.tokenize("room " * 100, truncate=True)
    assert int(tt[0, -1]) == tok.eot
    clip.set_tokenizer(None)
