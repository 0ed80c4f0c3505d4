"""Text tower: clip.tokenize + model.encode_text (main.py:179-182,
main.py:296-311), with the shipped checkpoints' text-MLP LoRA merged.

CPU: the oracle's encode_text is pinned against transformers' CLIPTextModelWithProjection
(independent implementation) on identical seeded weights. GPU: libclipvit_hip.so's text
encoder (clipvit_text_*) against the oracle, with and without merged LoRA, on prompts
tokenized from the reference's own label vocabulary.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from interior_amd import config as C
from interior_amd import labels as L
from interior_amd import tokenizer as TK
from interior_amd.weights import synthetic_text_state_dict
from oracle import clip_ref


@pytest.fixture(scope="module")
def prompts(golden_dir):
    cats = L.extract_categories(L.load_training_data(golden_dir / "interior_dataset.json"))
    return L.build_label_table(cats).all_texts


@pytest.fixture(scope="module")
def tok(prompts):
    return TK.SimpleTokenizer(TK.learn_merges(prompts, 600))


def _tc(tok, layers=12):
    return C.TextConfig(512, layers, 8, 77, tok.vocab_size, 512)


def _hf_model(sd, tc, eot):
    from transformers import CLIPTextConfig, CLIPTextModelWithProjection
    cfg = CLIPTextConfig(vocab_size=tc.vocab, hidden_size=tc.width, intermediate_size=4 * tc.width,
                         num_hidden_layers=tc.layers, num_attention_heads=tc.heads,
                         max_position_embeddings=tc.context, projection_dim=tc.embed_dim,
                         hidden_act="quick_gelu", layer_norm_eps=1e-5, eos_token_id=eot,
                         bos_token_id=eot - 1, pad_token_id=0)
    m = CLIPTextModelWithProjection(cfg).eval()
    D = tc.width
    hf = {"text_model.embeddings.token_embedding.weight": sd["token_embedding.weight"],
          "text_model.embeddings.position_embedding.weight": sd["positional_embedding"],
          "text_model.final_layer_norm.weight": sd["ln_final.weight"],
          "text_model.final_layer_norm.bias": sd["ln_final.bias"],
          "text_projection.weight": sd["text_projection"].t().contiguous()}
    for i in range(tc.layers):
        r, o = f"transformer.resblocks.{i}.", f"text_model.encoder.layers.{i}."
        W, b = sd[r + "attn.in_proj_weight"], sd[r + "attn.in_proj_bias"]
        for j, nm in enumerate("qkv"):
            hf[o + f"self_attn.{nm}_proj.weight"] = W[j * D:(j + 1) * D]
            hf[o + f"self_attn.{nm}_proj.bias"] = b[j * D:(j + 1) * D]
        hf[o + "self_attn.out_proj.weight"] = sd[r + "attn.out_proj.weight"]
        hf[o + "self_attn.out_proj.bias"] = sd[r + "attn.out_proj.bias"]
        for a, c in (("layer_norm1", "ln_1"), ("layer_norm2", "ln_2")):
            hf[o + a + ".weight"], hf[o + a + ".bias"] = sd[r + c + ".weight"], sd[r + c + ".bias"]
        hf[o + "mlp.fc1.weight"], hf[o + "mlp.fc1.bias"] = sd[r + "mlp.c_fc.weight"], sd[r + "mlp.c_fc.bias"]
        hf[o + "mlp.fc2.weight"], hf[o + "mlp.fc2.bias"] = sd[r + "mlp.c_proj.weight"], sd[r + "mlp.c_proj.bias"]
    missing, unexpected = m.load_state_dict(hf, strict=False)
    assert not unexpected and all("position_ids" in k for k in missing), (missing, unexpected)
    return m


def test_oracle_encode_text_matches_transformers(tok, prompts):
    tc = _tc(tok)
    sd = synthetic_text_state_dict(tc, 1)
    ids = tok.tokenize(prompts[:6] + ["salon", "wnętrze z drewnem i szkłem"])
    mine = clip_ref.encode_text(sd, ids, tc.heads)
    with torch.no_grad():
        ref = _hf_model(sd, tc, tok.eot)(input_ids=torch.from_numpy(ids).long()).text_embeds
    rel = ((mine - ref).abs().max() / ref.abs().max()).item()
    assert rel < 1e-5, rel


def test_text_adapters_from_shipped_checkpoint_format():
    """the shipped checkpoints bind text-MLP adapters only (main.py:93-109); the text-side
    binding yields 24 merge items (12 blocks x c_fc/c_proj), r = 4, scaling = alpha / r."""
    from collections import OrderedDict
    from interior_amd import lora
    g = torch.Generator().manual_seed(0)
    ck = OrderedDict()
    for i in range(12):
        for leaf, (i_f, o_f) in (("c_fc", (512, 2048)), ("c_proj", (2048, 512))):
            k = f"clip_model.transformer.resblocks.{i}.mlp.{leaf}.lora."
            ck[k + "lora_A"] = torch.randn(i_f, 4, generator=g)
            ck[k + "lora_B"] = torch.randn(4, o_f, generator=g)
    items, loaded, missing = lora.text_adapters_from_checkpoint(ck, 12, rank=4, alpha=8)
    assert loaded == 48 and len(items) == 24
    assert all(it.target.startswith("transformer.resblocks.") and it.scaling == 2.0 for it in items)
    it = items[0]
    assert it.target == "transformer.resblocks.0.mlp.c_fc.weight" and it.A.shape == (512, 4)


# ------------------------------------------------------------------------------------ GPU
def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float((np.abs(a - b).max(axis=1) / np.abs(b).max(axis=1)).max())


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp16", "bf16"])
def test_gpu_encode_text_matches_oracle(gpu, tok, prompts, dtype):
    from interior_amd.text import TextEngine
    tc = _tc(tok)
    sd = synthetic_text_state_dict(tc, 1)
    ids = tok.tokenize(prompts[:37] + ["x", "salon"])
    eng = TextEngine(tc, gpu, dtype, max_batch=64)
    eng.load_state_dict(sd)
    got = eng.encode_text(ids, normalize=False).cpu().numpy()
    nrm = eng.encode_text(ids, normalize=True).cpu().numpy()
    eng.close()
    ref = clip_ref.encode_text(sd, ids, tc.heads).numpy()
    tol = 2e-3 if dtype == "fp16" else 1.5e-2
    assert _rel(got, ref) < tol
    refn = ref / np.linalg.norm(ref, axis=1, keepdims=True)
    assert np.abs(nrm - refn).max() < tol


@pytest.mark.gpu
def test_gpu_encode_text_with_merged_lora(gpu, tok, prompts):
    from interior_amd.lora import LoraAdapter
    from interior_amd.text import TextEngine
    tc = _tc(tok)
    sd = synthetic_text_state_dict(tc, 2)
    rng = np.random.default_rng(0)
    ads = []
    for i in range(tc.layers):
        for leaf, (i_f, o_f) in (("c_fc", (512, 2048)), ("c_proj", (2048, 512))):
            ads.append(LoraAdapter(f"transformer.resblocks.{i}.mlp.{leaf}.weight",
                                   (rng.standard_normal((i_f, 4)) * 0.02).astype(np.float32),
                                   (rng.standard_normal((4, o_f)) * 0.02).astype(np.float32), 2.0))
    ids = tok.tokenize(prompts[40:100])
    eng = TextEngine(tc, gpu, "fp16", max_batch=64)
    eng.load_state_dict(sd)
    base = eng.encode_text(ids).cpu().numpy()
    eng.load_lora(ads)
    got = eng.encode_text(ids).cpu().numpy()
    eng.close()
    msd = dict(sd)
    for a in ads:
        msd[a.target] = clip_ref.merge_lora(sd[a.target], torch.from_numpy(a.A), torch.from_numpy(a.B), a.scaling)
    ref = clip_ref.encode_text(msd, ids, tc.heads).numpy()
    assert _rel(got, ref) < 2e-3
    assert _rel(base, ref) > 1e-2  # the merge changed the features


@pytest.mark.gpu
def test_gpu_text_batch_tails_and_errors(gpu, tok):
    from interior_amd import _lib
    from interior_amd.text import TextEngine
    tc = _tc(tok, layers=2)
    sd = synthetic_text_state_dict(tc, 3)
    eng = TextEngine(tc, gpu, "fp16", max_batch=8)
    eng.load_state_dict(sd)
    ids = tok.tokenize(["a", "wnętrze z cegłą", "salon", "kuchnia", "łazienka"])
    full = eng.encode_text(ids).cpu().numpy()
    for n in (1, 3):
        part = eng.encode_text(ids[:n]).cpu().numpy()
        assert np.array_equal(part, full[:n])  # rows are independent: bit-identical
    bad = ids.copy()
    bad[0, 3] = tc.vocab + 5
    with pytest.raises(ValueError):
        eng.encode_text(bad)
    with pytest.raises(_lib.ClipVitError):
        eng.encode_text(np.zeros((9, 77), np.int32))  # above max_batch
    eng.close()


@pytest.mark.gpu
def test_gpu_analyzer_label_matrix_from_text_tower(gpu, tok, golden_dir, tmp_path):
    """InteriorAnalyzer(text_state_dict=..., use_lora=True, lora_weights_path=ckpt): detector
    rows through the base text tower, analyzer rows through the LoRA text tower (main.py:179-182
    vs main.py:296-311), checkpoint in the shipped format (clip_model.transformer... keys)."""
    from collections import OrderedDict
    from interior_amd.analyzer import InteriorAnalyzer
    from interior_amd.lora import load_lora_checkpoint, text_adapters_from_checkpoint
    tc = _tc(tok)
    sd = synthetic_text_state_dict(tc, 4)
    g = torch.Generator().manual_seed(5)
    ck = OrderedDict()
    for i in range(12):
        for leaf, (i_f, o_f) in (("c_fc", (512, 2048)), ("c_proj", (2048, 512))):
            k = f"clip_model.transformer.resblocks.{i}.mlp.{leaf}.lora."
            ck[k + "lora_A"] = torch.randn(i_f, 4, generator=g) * 0.02
            ck[k + "lora_B"] = torch.randn(4, o_f, generator=g) * 0.02
    path = tmp_path / "comprehensive_lora.pth"
    torch.save(ck, path)
    an = InteriorAnalyzer("ViT-B/32", state_dict="synthetic", use_lora=True, lora_weights_path=str(path), lora_rank=4,
                          lora_alpha=8, device=gpu, compute_dtype="fp16",
                          dataset_json=golden_dir / "interior_dataset.json", max_batch=4,
                          text_state_dict=sd, tokenizer=tok)
    assert an.lora_report["text_adapters"] == 24
    texts = an.table.texts
    det_ids = tok.tokenize(texts[0])
    rest_ids = tok.tokenize([t for ts in texts[1:] for t in ts])
    ref_det = torch.nn.functional.normalize(clip_ref.encode_text(sd, det_ids), dim=-1)
    msd = dict(sd)
    items, _, _ = text_adapters_from_checkpoint(load_lora_checkpoint(path), 12, 4, 8)
    for a in items:
        msd[a.target] = clip_ref.merge_lora(sd[a.target], torch.from_numpy(a.A), torch.from_numpy(a.B), a.scaling)
    ref_rest = torch.nn.functional.normalize(clip_ref.encode_text(msd, rest_ids), dim=-1)
    ref = torch.cat([ref_det, ref_rest]).numpy()
    got = an.text_matrix
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() < 2e-3
