"""LoRA checkpoint format + the reference's binding rule (main.py:62-113), CPU only.

Pinned by tests/golden/lora_binding.json, which make_golden.py produced by running the
reference's OWN replace_linears_with_lora + load_lora_weights_to_model on both shipped
checkpoints: 72 Linears wrapped, 48 parameters bound, 96 missing, vision delta exactly 0,
the vision attn.out_proj adapter dead (delta 0 even with lora_B = 1)."""
import json
from collections import OrderedDict
from pathlib import Path

import numpy as np
import pytest
import torch

from interior_amd import config as C
from interior_amd import lora as L

REF_CKPT = Path("/root/reference/lora_models")


@pytest.fixture(scope="module")
def facts(golden_dir):
    return json.loads((golden_dir / "lora_binding.json").read_text())


def _fake_ckpt(f, seed=0):
    g = torch.Generator().manual_seed(seed)
    return OrderedDict((k, torch.randn(*f["ckpt_shapes"][k], generator=g)) for k in f["ckpt_keys"])


def test_binding_rule_reproduces_reference_counts(facts):
    for f in facts["checkpoints"]:
        names = L.wrapped_lora_param_names(12, 12)
        assert len(names) // 2 == f["replaced_linears"] == 72
        bound, missing = L.bind(_fake_ckpt(f), names)
        assert len(bound) == f["loaded"] == 48
        assert missing == f["missing_names"]
        assert len(missing) == f["missing"] == 96


def test_vision_adapters_from_reference_layout_are_empty(facts):
    """The shipped checkpoints only hold text-tower MLP adapters: no vision adapter binds,
    so the merged image path equals the base model (reference delta = 0.0)."""
    for f in facts["checkpoints"]:
        items, loaded, missing = L.vision_adapters_from_checkpoint(_fake_ckpt(f), C.VIT_B16, 4, 8)
        assert items == [] and loaded == 48 and len(missing) == 96
        assert f["vision_delta_max_abs"] == 0.0 and f["dead_out_proj_delta_max_abs"] == 0.0


def test_vision_keys_bind_and_merge_when_present():
    """A checkpoint WITH vision adapters (same naming scheme) binds by suffix and produces
    merge items; attn.out_proj is dropped in reference semantics (dead wrapper)."""
    ck = OrderedDict()
    for i in range(12):
        for leaf, (fin, fout) in {"attn.out_proj": (768, 768), "mlp.c_fc": (768, 3072),
                                  "mlp.c_proj": (3072, 768)}.items():
            base = f"clip_model.visual.transformer.resblocks.{i}.{leaf}.lora."
            ck[base + "lora_A"] = torch.ones(fin, 4)
            ck[base + "lora_B"] = torch.ones(4, fout)
    items, loaded, _ = L.vision_adapters_from_checkpoint(ck, C.VIT_B32, 4, 8)
    # 144, not 72: under main.py:101-104 ``k.endswith(name)`` a key
    # "clip_model.visual.transformer.resblocks.i.X" ALSO ends with the text tower's parameter
    # name "transformer.resblocks.i.X", so each vision key binds twice (reference quirk, kept).
    assert loaded == 144 and len(items) == 24
    assert {it.target.split(".", 4)[-1] for it in items} == {"mlp.c_fc.weight", "mlp.c_proj.weight"}
    assert all(it.scaling == 2.0 and it.rank == 4 for it in items)
    items_all, _, _ = L.vision_adapters_from_checkpoint(ck, C.VIT_B32, 4, 8, live_only=False)
    assert len(items_all) == 36


@pytest.mark.skipif(not REF_CKPT.exists(), reason="reference checkpoints not present")
def test_shipped_checkpoint_loads_weights_only():
    for name in ("comprehensive_lora.pth", "comprehensive_lora_new.pth"):
        ck = L.load_lora_checkpoint(REF_CKPT / name)
        assert len(ck) == 48 and all(v.dtype == torch.float32 for v in ck.values())
        items, loaded, missing = L.vision_adapters_from_checkpoint(ck, C.VIT_B16, 4, 8)
        assert items == [] and loaded == 48 and len(missing) == 96


def test_missing_checkpoint_raises():
    with pytest.raises(FileNotFoundError):
        L.load_lora_checkpoint("/nonexistent/lora.pth")  # main.py:87-88


def test_synthetic_adapters_cover_fused_qkv():
    items = L.synthetic_adapters(C.VIT_B32, rank=8)
    assert len(items) == 48
    qkv = [it for it in items if it.target.endswith("attn.in_proj_weight")]
    assert len(qkv) == 12 and qkv[0].A.shape == (768, 8) and qkv[0].B.shape == (8, 2304)
    assert all(it.scaling == 2.0 for it in items)  # alpha = 2 r (main.py:20, main.py:522)
    assert np.abs(qkv[0].B).max() > 0
