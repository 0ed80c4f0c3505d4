"""Checkpoint readers (weights.py): a local OpenAI TorchScript archive (what clip.load downloads,
main.py:152 / 241) or a plain state dict, read without executing anything from the file.

The archive here is one this test writes itself (the oracle's OpenAI-named module mirror,
traced, fp16 like the downloaded checkpoints); torch.jit.load is used only on that self-made
file, as the independent reader the code-free one is compared against."""
import pickle
import zipfile

import pytest
import torch

from interior_amd import config as C
from interior_amd import weights as W
from oracle.clip_module import CLIPMirror, load_params
from oracle.clip_ref import GEOMETRIES


class _Wrap(torch.nn.Module):
    def __init__(self, m):
        super().__init__()
        for k in ("visual", "transformer", "token_embedding", "positional_embedding", "ln_final",
                  "text_projection", "logit_scale"):
            setattr(self, k, getattr(m, k))

    def forward(self, x):
        return self.visual(x)


@pytest.fixture(scope="module")
def archive(tmp_path_factory):
    sd = W.synthetic_state_dict(C.VIT_B32, 0)
    m = CLIPMirror(GEOMETRIES["ViT-B/32"], vocab=600)
    load_params(m, sd)
    ts = torch.jit.trace(_Wrap(m.eval()), torch.randn(1, 3, 224, 224), check_trace=False).half()
    p = tmp_path_factory.mktemp("ckpt") / "ViT-B-32.pt"
    torch.jit.save(ts, str(p))
    return p, sd


def test_archive_reader_equals_jit_state_dict(archive):
    p, _ = archive
    assert W.is_torchscript_archive(p)
    ref = torch.jit.load(str(p)).state_dict()
    got = W.read_torchscript_archive(p)
    assert set(got) == set(ref)
    for k in ref:
        assert got[k].dtype == ref[k].dtype == torch.float16 and torch.equal(got[k], ref[k]), k


def test_load_openai_checkpoint_visual_and_text(archive):
    p, sd = archive
    vis = W.load_openai_checkpoint(p)
    assert set(vis) == {n for n, _ in W.visual_names(C.VIT_B32)}
    for k, v in vis.items():
        assert v.dtype == torch.float32 and torch.equal(v, sd[k].half().float()), k
    txt = W.load_openai_checkpoint(p, text=True)
    assert "token_embedding.weight" in txt and "ln_final.weight" in txt and "logit_scale" not in txt
    assert not any(k.startswith("visual.") for k in txt)


def test_plain_state_dict(tmp_path):
    sd = W.synthetic_state_dict(C.VIT_B32, 3)
    p = tmp_path / "sd.pth"
    torch.save(sd, p)
    assert not W.is_torchscript_archive(p)
    got = W.load_openai_checkpoint(p)
    assert all(torch.equal(got[k], sd[k]) for k in sd)


def test_archive_with_foreign_global_is_refused(tmp_path):
    """A data.pkl that names any global besides tensor rebuilding / __torch__ classes is refused."""
    class Evil:
        def __reduce__(self):
            return (print, ("pwned",))
    p = tmp_path / "evil.pt"
    with zipfile.ZipFile(p, "w") as zf:
        zf.writestr("evil/data.pkl", pickle.dumps({"visual.x": Evil()}, protocol=2))
        zf.writestr("evil/constants.pkl", pickle.dumps((), protocol=2))
    with pytest.raises(pickle.UnpicklingError, match="refusing global"):
        W.load_openai_checkpoint(p)


def test_missing_file_raises(tmp_path):
    with pytest.raises(FileNotFoundError):
        W.load_openai_checkpoint(tmp_path / "nope.pt")
