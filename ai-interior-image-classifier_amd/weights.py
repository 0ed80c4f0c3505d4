"""Vision-tower weights keyed by OpenAI-CLIP state-dict names.

Two sources:
* ``synthetic_state_dict`` — seeded CLIP-style random init (there is no network for the real
  OpenAI checkpoints here; BASELINE.json's configs are benchmarked on synthetic weights of the
  exact architecture);
* ``load_openai_checkpoint`` — a LOCAL OpenAI ``ViT-*.pt`` (TorchScript archive as downloaded
  by clip.load [3p]) or a plain state dict, for real-weight runs where such a file exists.
"""
from __future__ import annotations

import collections
import io
import pickle
import zipfile
from pathlib import Path

import numpy as np
import torch

from .config import ViTConfig


def visual_names(cfg: ViTConfig) -> list[tuple[str, tuple[int, ...]]]:
    """Every ``visual.*`` tensor the encoder consumes, in a fixed generation order."""
    D, P = cfg.width, cfg.patch_size
    out = [("visual.conv1.weight", (D, 3, P, P)), ("visual.class_embedding", (D,)),
           ("visual.positional_embedding", (cfg.tokens, D)), ("visual.ln_pre.weight", (D,)),
           ("visual.ln_pre.bias", (D,))]
    for i in range(cfg.layers):
        r = f"visual.transformer.resblocks.{i}."
        out += [(r + "ln_1.weight", (D,)), (r + "ln_1.bias", (D,)),
                (r + "attn.in_proj_weight", (3 * D, D)), (r + "attn.in_proj_bias", (3 * D,)),
                (r + "attn.out_proj.weight", (D, D)), (r + "attn.out_proj.bias", (D,)),
                (r + "ln_2.weight", (D,)), (r + "ln_2.bias", (D,)),
                (r + "mlp.c_fc.weight", (4 * D, D)), (r + "mlp.c_fc.bias", (4 * D,)),
                (r + "mlp.c_proj.weight", (D, 4 * D)), (r + "mlp.c_proj.bias", (D,))]
    out += [("visual.ln_post.weight", (D,)), ("visual.ln_post.bias", (D,)),
            ("visual.proj", (D, cfg.embed_dim))]
    return out


def synthetic_state_dict(cfg: ViTConfig, seed: int = 0) -> dict[str, torch.Tensor]:
    """Seeded CLIP-style weights (torch.Generator on CPU: identical on every host with the
    same torch build). Linear/conv ~ N(0, 0.02); class/pos/proj ~ N(0, width^-0.5) as
    OpenAI's VisionTransformer.__init__ [3p]; LayerNorm gamma = 1 + N(0, 0.1), beta and biases
    ~ N(0, 0.02) so parity tests exercise every affine term."""
    g = torch.Generator().manual_seed(seed)
    scale = cfg.width ** -0.5
    sd = {}
    for name, shape in visual_names(cfg):
        if name.endswith(("class_embedding", "positional_embedding")) or name == "visual.proj":
            t = torch.randn(shape, generator=g) * scale
        elif ".ln_" in name or name.startswith("visual.ln_"):
            t = torch.randn(shape, generator=g) * (0.1 if name.endswith("weight") else 0.02)
            if name.endswith("weight"):
                t += 1.0
        elif name.endswith("bias"):
            t = torch.randn(shape, generator=g) * 0.02
        else:
            t = torch.randn(shape, generator=g) * 0.02
        sd[name] = t.float().contiguous()
    return sd


def text_names(tc) -> list[tuple[str, tuple[int, ...]]]:
    """OpenAI state-dict names/shapes of the text tower (CLIP [3p]: token_embedding,
    positional_embedding, transformer.resblocks.i.*, ln_final, text_projection)."""
    D = tc.width
    out = [("token_embedding.weight", (tc.vocab, D)), ("positional_embedding", (tc.context, D))]
    for i in range(tc.layers):
        r = f"transformer.resblocks.{i}."
        out += [(r + "ln_1.weight", (D,)), (r + "ln_1.bias", (D,)),
                (r + "attn.in_proj_weight", (3 * D, D)), (r + "attn.in_proj_bias", (3 * D,)),
                (r + "attn.out_proj.weight", (D, D)), (r + "attn.out_proj.bias", (D,)),
                (r + "ln_2.weight", (D,)), (r + "ln_2.bias", (D,)),
                (r + "mlp.c_fc.weight", (4 * D, D)), (r + "mlp.c_fc.bias", (4 * D,)),
                (r + "mlp.c_proj.weight", (D, 4 * D)), (r + "mlp.c_proj.bias", (D,))]
    out += [("ln_final.weight", (D,)), ("ln_final.bias", (D,)),
            ("text_projection", (D, tc.embed_dim))]
    return out


def synthetic_text_state_dict(tc, seed: int = 1) -> dict[str, torch.Tensor]:
    """Seeded text-tower weights in the scales of CLIP.initialize_parameters [3p]
    (token 0.02, positional 0.01, projection width^-0.5), LayerNorm/bias terms perturbed
    like synthetic_state_dict so parity exercises every affine term."""
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for name, shape in text_names(tc):
        if name == "positional_embedding":
            t = torch.randn(shape, generator=g) * 0.01
        elif name == "text_projection":
            t = torch.randn(shape, generator=g) * tc.width ** -0.5
        elif "ln_" in name:
            t = torch.randn(shape, generator=g) * (0.1 if name.endswith("weight") else 0.02)
            if name.endswith("weight"):
                t += 1.0
        else:
            t = torch.randn(shape, generator=g) * 0.02
        sd[name] = t.float().contiguous()
    return sd


def state_dict_checksum(sd: dict[str, torch.Tensor]) -> float:
    """Order-independent float64 checksum used to prove fixtures were regenerated identically."""
    return float(sum(float(v.double().abs().sum()) for v in sd.values()))


class _ScriptObject:
    """Attribute bag standing in for a TorchScript class while an archive is read: the class's
    code (the archive's ``code/`` entries) is never loaded or run."""

    def __setstate__(self, state):
        self.state = state


_STORAGE_DTYPES = {"FloatStorage": torch.float32, "HalfStorage": torch.float16,
                   "BFloat16Storage": torch.bfloat16, "DoubleStorage": torch.float64,
                   "LongStorage": torch.int64, "IntStorage": torch.int32, "ShortStorage": torch.int16,
                   "CharStorage": torch.int8, "ByteStorage": torch.uint8, "BoolStorage": torch.bool}


class _StorageType:
    def __init__(self, dtype):
        self.dtype = dtype


def _rebuild_tensor(storage, offset, size, stride, *args):
    return storage.as_strided(tuple(size), tuple(stride), offset)


class _ArchiveUnpickler(pickle.Unpickler):
    """Restricted unpickler for a torch zip archive's ``data.pkl``: rebuilds tensors from the
    archive's raw storage records and turns every ``__torch__.*`` class into an inert
    ``_ScriptObject``; any other global is refused (nothing from the file is executed)."""

    def __init__(self, data: bytes, zf: zipfile.ZipFile, prefix: str):
        super().__init__(io.BytesIO(data))
        self.zf, self.prefix = zf, prefix

    def find_class(self, module, name):
        if module == "torch._utils" and name in ("_rebuild_tensor_v2", "_rebuild_tensor"):
            return _rebuild_tensor
        if module == "torch._utils" and name == "_rebuild_parameter":
            return lambda data, requires_grad, hooks: data
        if module == "collections" and name == "OrderedDict":
            return collections.OrderedDict
        if module == "torch" and name in _STORAGE_DTYPES:
            return _StorageType(_STORAGE_DTYPES[name])
        if module == "torch" and isinstance(getattr(torch, name, None), torch.dtype):
            return getattr(torch, name)
        if module.startswith("__torch__"):
            return type(name, (_ScriptObject,), {})
        raise pickle.UnpicklingError(f"refusing global {module}.{name} in a weights archive")

    def persistent_load(self, pid):
        kind, stype, key, _location, numel = pid[:5]
        if kind != "storage":
            raise pickle.UnpicklingError(f"unknown persistent record {kind!r}")
        dtype = stype.dtype if isinstance(stype, _StorageType) else stype
        raw = self.zf.read(f"{self.prefix}/data/{key}")
        return torch.frombuffer(bytearray(raw), dtype=dtype)[:numel] if numel else torch.empty(0, dtype=dtype)


def _flatten(obj, prefix: str, out: dict):
    if isinstance(obj, torch.Tensor):
        out[prefix[:-1]] = obj
    elif isinstance(obj, _ScriptObject):
        _flatten(getattr(obj, "state", None), prefix, out)
    elif isinstance(obj, dict):
        for k, v in obj.items():
            if isinstance(k, str):
                _flatten(v, prefix + k + ".", out)


def is_torchscript_archive(path: str | Path) -> bool:
    if not zipfile.is_zipfile(path):
        return False
    with zipfile.ZipFile(path) as zf:
        return any(n.endswith("/constants.pkl") or "/code/" in n for n in zf.namelist())


def read_torchscript_archive(path: str | Path) -> dict[str, torch.Tensor]:
    """Tensors of a TorchScript archive (what clip.load downloads: ``ViT-*.pt``) by dotted
    attribute path, e.g. ``visual.conv1.weight``, without executing anything from the file:
    ``<root>/data.pkl`` is read by a restricted unpickler, the ``code/`` entries are ignored."""
    with zipfile.ZipFile(path) as zf:
        pkls = [n for n in zf.namelist() if n.endswith("/data.pkl") and n.count("/") == 1]
        if not pkls:
            raise ValueError(f"{path}: not a torch zip archive (no <root>/data.pkl)")
        prefix = pkls[0].split("/")[0]
        root = _ArchiveUnpickler(zf.read(pkls[0]), zf, prefix).load()
        out: dict[str, torch.Tensor] = {}
        _flatten(root, "", out)
        return {k: v.clone() for k, v in out.items()}


def load_openai_checkpoint(path: str | Path, text: bool = False) -> dict[str, torch.Tensor]:
    """Local OpenAI CLIP checkpoint -> fp32 ``visual.*`` state dict (``text=True``: the text
    tower's tensors instead, for TextEngine / InteriorAnalyzer(text_state_dict=...)).

    A plain state dict is read with ``torch.load(weights_only=True)``; an OpenAI TorchScript
    archive (what clip.load downloads; recognised by its ``constants.pkl`` / ``code/``
    entries), which the weights-only loader refuses, is read by ``read_torchscript_archive`` —
    neither path runs code from the file. Errors (missing file, corrupt archive, a pickle the
    weights-only loader rejects) propagate unchanged.
    """
    path = Path(path)
    if is_torchscript_archive(path):
        sd = read_torchscript_archive(path)
    else:
        sd = torch.load(path, map_location="cpu", weights_only=True)
        if not isinstance(sd, dict):
            raise ValueError(f"{path}: expected a state dict, got {type(sd).__name__}")
    keep = (lambda k: not k.startswith("visual.") and k not in ("logit_scale", "input_resolution",
                                                                 "context_length", "vocab_size")) \
        if text else (lambda k: k.startswith("visual."))
    return {k: v.float().contiguous() for k, v in sd.items() if keep(k) and isinstance(v, torch.Tensor)}


def as_host_f32(t) -> np.ndarray:
    if isinstance(t, torch.Tensor):
        return np.ascontiguousarray(t.detach().to("cpu", torch.float32).numpy())
    return np.ascontiguousarray(np.asarray(t, dtype=np.float32))
