"""ORACLE — test infrastructure only. nn.Module mirror of the OpenAI-CLIP module tree.

Used (a) to pin ``clip_ref.encode_image`` against torch's own ``nn.MultiheadAttention``
path and (b) as the ``clip`` module injected into the *reference's own* harness
(main.py ``CachedInteriorAnalyzer``, ``InteriorImageDetector``, ``replace_linears_with_lora``,
``load_lora_weights_to_model``) when ``tests/golden/make_golden.py`` generates fixtures in the
build container. Never imported by the product package.

The attribute names reproduce OpenAI ``clip/model.py`` [3p, unpinned] exactly, because the
reference binds LoRA by parameter *name* (main.py:62-74 walks ``named_children``;
main.py:93-109 suffix-matches ``named_parameters`` against the checkpoint keys):

    visual.{conv1, class_embedding, positional_embedding, ln_pre, transformer.resblocks.i.
            {attn (nn.MultiheadAttention: in_proj_weight/bias, out_proj), ln_1,
             mlp.{c_fc, gelu, c_proj}, ln_2}, ln_post, proj}
    transformer.resblocks.i.*  (text tower, width 512, 8 heads), token_embedding,
    positional_embedding, ln_final, text_projection, logit_scale

The text tower is OpenAI's ``encode_text`` [3p] with real token ids: ``token_embedding`` of the
ids + ``positional_embedding`` -> the (LoRA-wrapped) causal transformer -> ``ln_final`` -> the
row at each prompt's end-of-text id (``text.argmax(-1)``) @ ``text_projection``. The OpenAI BPE
vocabulary file is absent offline, so ``tokenize`` is CLIP's ``tokenize`` (sot + ids + eot, zero
padding to 77) over a merges list learned from the reference's own prompt vocabulary
(tests/golden/bpe_merges.txt), with HF ``tokenizers`` (transformers' CLIPTokenizer) doing the
byte-level BPE — an implementation independent of the product's ``tokenizer.py``. Text weights
are seeded synthetic tensors with the OpenAI names.
"""
from __future__ import annotations

import types
from collections import OrderedDict

import torch
import torch.nn as nn

from .clip_ref import GEOMETRIES, Geometry, preprocess


class LayerNorm(nn.LayerNorm):
    def forward(self, x):
        orig = x.dtype
        return super().forward(x.type(torch.float32)).type(orig)


class QuickGELU(nn.Module):
    def forward(self, x):
        return x * torch.sigmoid(1.702 * x)


class ResidualAttentionBlock(nn.Module):
    def __init__(self, d_model: int, n_head: int, attn_mask=None):
        super().__init__()
        self.attn = nn.MultiheadAttention(d_model, n_head)
        self.ln_1 = LayerNorm(d_model)
        self.mlp = nn.Sequential(OrderedDict([
            ("c_fc", nn.Linear(d_model, d_model * 4)),
            ("gelu", QuickGELU()),
            ("c_proj", nn.Linear(d_model * 4, d_model)),
        ]))
        self.ln_2 = LayerNorm(d_model)
        self.attn_mask = attn_mask

    def attention(self, x):
        m = self.attn_mask.to(dtype=x.dtype, device=x.device) if self.attn_mask is not None else None
        return self.attn(x, x, x, need_weights=False, attn_mask=m)[0]

    def forward(self, x):
        x = x + self.attention(self.ln_1(x))
        return x + self.mlp(self.ln_2(x))


class Transformer(nn.Module):
    def __init__(self, width: int, layers: int, heads: int, attn_mask=None):
        super().__init__()
        self.width, self.layers = width, layers
        self.resblocks = nn.Sequential(*[ResidualAttentionBlock(width, heads, attn_mask) for _ in range(layers)])

    def forward(self, x):
        return self.resblocks(x)


class VisionTransformer(nn.Module):
    def __init__(self, geo: Geometry):
        super().__init__()
        w = geo.width
        self.input_resolution = geo.image_size
        self.conv1 = nn.Conv2d(3, w, kernel_size=geo.patch_size, stride=geo.patch_size, bias=False)
        self.class_embedding = nn.Parameter(torch.zeros(w))
        self.positional_embedding = nn.Parameter(torch.zeros(geo.tokens, w))
        self.ln_pre = LayerNorm(w)
        self.transformer = Transformer(w, geo.layers, geo.heads)
        self.ln_post = LayerNorm(w)
        self.proj = nn.Parameter(torch.zeros(w, geo.embed_dim))

    def forward(self, x):
        x = self.conv1(x)
        x = x.reshape(x.shape[0], x.shape[1], -1).permute(0, 2, 1)
        cls = self.class_embedding.to(x.dtype) + torch.zeros(x.shape[0], 1, x.shape[-1], dtype=x.dtype)
        x = torch.cat([cls, x], dim=1) + self.positional_embedding.to(x.dtype)
        x = self.ln_pre(x)
        x = x.permute(1, 0, 2)   # NLD -> LND (nn.MultiheadAttention is sequence-first)
        x = self.transformer(x)
        x = x.permute(1, 0, 2)
        x = self.ln_post(x[:, 0, :])
        return x @ self.proj


class CLIPMirror(nn.Module):
    def __init__(self, geo: Geometry, vocab: int, text_width=512, text_layers=12, text_heads=8,
                 context=77):
        super().__init__()
        self.context_length = context
        self.visual = VisionTransformer(geo)
        mask = torch.full((context, context), float("-inf")).triu_(1)
        self.transformer = Transformer(text_width, text_layers, text_heads, attn_mask=mask)
        self.token_embedding = nn.Embedding(vocab, text_width)
        self.positional_embedding = nn.Parameter(torch.zeros(context, text_width))
        self.ln_final = LayerNorm(text_width)
        self.text_projection = nn.Parameter(torch.zeros(text_width, geo.embed_dim))
        self.logit_scale = nn.Parameter(torch.tensor(4.6052))

    @property
    def dtype(self):
        return self.visual.conv1.weight.dtype

    def encode_image(self, image):
        return self.visual(image.type(self.dtype))

    def encode_text(self, text):
        x = self.token_embedding(text).type(self.dtype)
        x = x + self.positional_embedding.type(self.dtype)
        x = self.transformer(x.permute(1, 0, 2)).permute(1, 0, 2)
        x = self.ln_final(x).type(self.dtype)
        return x[torch.arange(x.shape[0]), text.argmax(dim=-1)] @ self.text_projection


def load_params(model: CLIPMirror, sd: dict):
    """Copy OpenAI-named tensors (``visual.*`` and text-tower names) into the mirror."""
    own = dict(model.named_parameters())
    with torch.no_grad():
        for k, v in sd.items():
            if k in own:
                own[k].copy_(torch.as_tensor(v, dtype=torch.float32).reshape(own[k].shape))


def clip_vocab(merges):
    """CLIP's vocabulary construction [3p simple_tokenizer]: 256 byte symbols, the same with
    ``</w>``, one entry per merge, then <|startoftext|>, <|endoftext|>."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs, n = bs[:], 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    syms = [chr(c) for c in cs]
    vocab = syms + [s + "</w>" for s in syms] + ["".join(m) for m in merges]
    vocab += ["<|startoftext|>", "<|endoftext|>"]
    return {v: i for i, v in enumerate(vocab)}


def read_merges_file(path):
    lines = open(path, encoding="utf-8").read().split("\n")[1:]
    return [tuple(l.split()) for l in lines if l.strip()]


def make_tokenize(merges):
    """``clip.tokenize`` over ``merges`` with HF tokenizers' byte-level BPE (CLIPTokenizer)."""
    from transformers import CLIPTokenizer
    hf = CLIPTokenizer(vocab=clip_vocab(merges), merges=[tuple(m) for m in merges])

    def tokenize(texts, context_length=77, truncate=False):
        texts = [texts] if isinstance(texts, str) else list(texts)
        out = torch.zeros(len(texts), context_length, dtype=torch.long)
        for i, t in enumerate(texts):
            ids = hf(t)["input_ids"]
            if len(ids) > context_length:
                if not truncate:
                    raise RuntimeError(f"Input {t} is too long for context length {context_length}")
                ids = ids[:context_length]
                ids[-1] = hf.eos_token_id
            out[i, :len(ids)] = torch.tensor(ids)
        return out

    return tokenize


def make_clip_shim(sd_by_name: dict, merges):
    """A module object usable as ``sys.modules['clip']`` for the reference's harness.

    ``load(name, device)`` returns (CLIPMirror carrying the seeded weights registered for
    ``name`` — ``visual.*`` and the text tower —, preprocess) exactly as main.py:152 /
    main.py:241 expect; ``tokenize`` is clip.tokenize over ``merges``.
    """
    shim = types.ModuleType("clip")
    vocab = len(merges) + 514

    def load(name, device="cpu", **kw):
        geo = GEOMETRIES[name]
        m = CLIPMirror(geo, vocab)
        load_params(m, sd_by_name[name])
        m.eval()
        return m, (lambda img: preprocess(img, geo.image_size))

    shim.load = load
    shim.base_load = load
    shim.tokenize = make_tokenize(merges)
    return shim
