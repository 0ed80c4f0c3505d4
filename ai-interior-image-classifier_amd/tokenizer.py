"""CLIP's byte-level BPE tokenizer, restated: ``clip.tokenize(texts, context_length=77)`` [3p]
as called at main.py:180 (detector prompts) and main.py:307 (analyzer prompts), feeding
``model.encode_text``.

Semantics followed (OpenAI ``clip/simple_tokenizer.py`` + ``clip.tokenize``, unpinned [3p]):

* vocabulary = the 256 byte symbols (``bytes_to_unicode``), the same with ``</w>``, one symbol
  per merge (merges = lines ``1 .. 49152-256-2`` of ``bpe_simple_vocab_16e6.txt.gz``), then
  ``<|startoftext|>`` and ``<|endoftext|>``: 49408 ids for the real file;
* text cleaning: ftfy ``fix_text`` (ftfy is not installed here: NFC normalisation, which is
  what ``fix_text`` does to text without mojibake), ``html.unescape`` twice, strip, collapse
  whitespace, lower-case;
* pre-tokenisation by CLIP's regex, each piece mapped through the byte encoder, then greedy
  lowest-rank BPE with ``</w>`` on the last symbol;
* ``tokenize``: ``[sot] + ids + [eot]`` zero-padded to ``context_length``; too long raises
  ``RuntimeError`` unless ``truncate`` (then the last kept id is ``eot``).

The merges file is data the caller supplies (``bpe_path``); it is not shipped with the
reference and cannot be fetched offline. Tests pin this restatement against an independent
implementation (HF ``tokenizers`` BPE via ``transformers.CLIPTokenizer``) on a merges list
learned from the reference's own label vocabulary.
"""
from __future__ import annotations

import gzip
import html
import unicodedata
from functools import lru_cache
from pathlib import Path

import numpy as np
import regex as re

SOT, EOT = "<|startoftext|>", "<|endoftext|>"
PATTERN = re.compile(
    r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+""",
    re.IGNORECASE)


@lru_cache()
def bytes_to_unicode() -> dict[int, str]:
    """Reversible byte -> printable unicode map (printable latin-1 ranges map to themselves,
    the other 68 bytes to code points 256+)."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, map(chr, cs)))


def get_pairs(word: tuple[str, ...]) -> set[tuple[str, str]]:
    return {(a, b) for a, b in zip(word[:-1], word[1:])}


def clean(text: str) -> str:
    text = unicodedata.normalize("NFC", text)      # ftfy.fix_text on mojibake-free text
    text = html.unescape(html.unescape(text)).strip()
    return re.sub(r"\s+", " ", text).strip().lower()


def read_merges(bpe_path: str | Path, n_merges: int | None = 49152 - 256 - 2) -> list[tuple[str, str]]:
    """Merges of a CLIP ``bpe_simple_vocab_16e6.txt(.gz)``: skip the header line, keep the
    first ``n_merges`` (None = all)."""
    p = Path(bpe_path)
    raw = gzip.open(p).read() if p.suffix == ".gz" else p.read_bytes()
    lines = raw.decode("utf-8").split("\n")
    lines = lines[1:] if n_merges is None else lines[1:n_merges + 1]
    return [tuple(l.split()) for l in lines if l.strip()]


class SimpleTokenizer:
    def __init__(self, merges: list[tuple[str, str]] | None = None, bpe_path: str | Path | None = None):
        if merges is None:
            if bpe_path is None:
                raise ValueError("CLIP tokenizer needs the BPE merges (bpe_path or merges)")
            merges = read_merges(bpe_path)
        self.byte_encoder = bytes_to_unicode()
        self.byte_decoder = {v: k for k, v in self.byte_encoder.items()}
        vocab = list(self.byte_encoder.values())
        vocab = vocab + [v + "</w>" for v in vocab]
        vocab += ["".join(m) for m in merges]
        vocab += [SOT, EOT]
        self.encoder = {v: i for i, v in enumerate(vocab)}
        self.decoder = {i: v for v, i in self.encoder.items()}
        self.bpe_ranks = {tuple(m): i for i, m in enumerate(merges)}
        self.cache = {SOT: SOT, EOT: EOT}
        self.sot, self.eot = self.encoder[SOT], self.encoder[EOT]

    @property
    def vocab_size(self) -> int:
        return len(self.encoder)

    def bpe(self, token: str) -> str:
        if token in self.cache:
            return self.cache[token]
        word = tuple(token[:-1]) + (token[-1] + "</w>",)
        pairs = get_pairs(word)
        if not pairs:
            return token + "</w>"
        while True:
            bigram = min(pairs, key=lambda p: self.bpe_ranks.get(p, float("inf")))
            if bigram not in self.bpe_ranks:
                break
            first, second = bigram
            new_word, i = [], 0
            while i < len(word):
                try:
                    j = word.index(first, i)
                except ValueError:
                    new_word.extend(word[i:])
                    break
                new_word.extend(word[i:j])
                i = j
                if word[i] == first and i < len(word) - 1 and word[i + 1] == second:
                    new_word.append(first + second)
                    i += 2
                else:
                    new_word.append(word[i])
                    i += 1
            word = tuple(new_word)
            if len(word) == 1:
                break
            pairs = get_pairs(word)
        out = " ".join(word)
        self.cache[token] = out
        return out

    def encode(self, text: str) -> list[int]:
        ids = []
        for tok in re.findall(PATTERN, clean(text)):
            tok = "".join(self.byte_encoder[b] for b in tok.encode("utf-8"))
            ids.extend(self.encoder[t] for t in self.bpe(tok).split(" "))
        return ids

    def decode(self, ids) -> str:
        text = "".join(self.decoder[int(i)] for i in ids)
        return bytearray(self.byte_decoder[c] for c in text).decode("utf-8", errors="replace") \
            .replace("</w>", " ")

    def tokenize(self, texts, context_length: int = 77, truncate: bool = False) -> np.ndarray:
        """``clip.tokenize``: int32 [n, context_length] (the reference returns int64/int32
        depending on the torch version; the ids are the same)."""
        if isinstance(texts, str):
            texts = [texts]
        out = np.zeros((len(texts), context_length), dtype=np.int32)
        for i, t in enumerate(texts):
            ids = [self.sot] + self.encode(t) + [self.eot]
            if len(ids) > context_length:
                if not truncate:
                    raise RuntimeError(f"Input {t} is too long for context length {context_length}")
                ids = ids[:context_length]
                ids[-1] = self.eot
            out[i, :len(ids)] = ids
        return out


def learn_merges(texts, n_merges: int) -> list[tuple[str, str]]:
    """A tiny BPE trainer (most frequent adjacent pair, ties by first occurrence) over the
    byte-encoded words of ``texts``: produces a CLIP-format merges list for tests and for
    running the text tower without the OpenAI vocabulary file."""
    enc = bytes_to_unicode()
    words: dict[tuple[str, ...], int] = {}
    for t in texts:
        for tok in re.findall(PATTERN, clean(t)):
            s = "".join(enc[b] for b in tok.encode("utf-8"))
            w = tuple(s[:-1]) + (s[-1] + "</w>",)
            words[w] = words.get(w, 0) + 1
    merges = []
    for _ in range(n_merges):
        counts: dict[tuple[str, str], int] = {}
        for w, c in words.items():
            for p in zip(w[:-1], w[1:]):
                counts[p] = counts.get(p, 0) + c
        if not counts:
            break
        best = max(counts.items(), key=lambda kv: kv[1])[0]
        merges.append(best)
        a, b = best
        nw = {}
        for w, c in words.items():
            out, i = [], 0
            while i < len(w):
                if i < len(w) - 1 and w[i] == a and w[i + 1] == b:
                    out.append(a + b)
                    i += 2
                else:
                    out.append(w[i])
                    i += 1
            nw[tuple(out)] = nw.get(tuple(out), 0) + c
        words = nw
    return merges
