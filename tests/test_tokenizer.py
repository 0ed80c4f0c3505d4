"""CLIP BPE tokenizer restatement (tokenizer.py) against an independent implementation:
HF ``tokenizers`` byte-level BPE behind ``transformers.CLIPTokenizer``, built from the same
vocabulary/merges. The OpenAI merges file is absent offline, so the merges are learned from
the reference's own prompt vocabulary (interior_dataset.json labels, main.py:296-311 prompt
templates, main.py:156-176 detector prompts) — parity on that vocabulary is pinned, the real
49408-id vocabulary is "parity unpinned" here (a drop-in run with bpe_path=... on a box that has it).
"""
from __future__ import annotations

import gzip

import numpy as np
import pytest

from interior_amd import labels as L
from interior_amd import tokenizer as TK

EXTRA = ["a photo of a modern living room", "Wnętrze z   DREWNIANĄ podłogą!!", "it's 4 o'clock",
         "kitchen & dining", "  trailing spaces  ", "naïve café 3D-render", "x", ""]


@pytest.fixture(scope="module")
def corpus(golden_dir):
    cats = L.extract_categories(L.load_training_data(golden_dir / "interior_dataset.json"))
    return L.build_label_table(cats).all_texts


@pytest.fixture(scope="module")
def merges(corpus):
    return TK.learn_merges(corpus, 600)


@pytest.fixture(scope="module")
def both(merges):
    from transformers import CLIPTokenizer
    mine = TK.SimpleTokenizer(merges)
    hf = CLIPTokenizer(vocab=dict(mine.encoder), merges=[tuple(m) for m in merges])
    return mine, hf


def test_vocab_layout(merges):
    tk = TK.SimpleTokenizer(merges)
    assert tk.vocab_size == 512 + len(merges) + 2
    assert tk.sot == tk.vocab_size - 2 and tk.eot == tk.vocab_size - 1
    enc = TK.bytes_to_unicode()
    assert len(set(enc.values())) == 256 and enc[ord("a")] == "a" and enc[ord(" ")] == "Ġ"


def test_ids_match_hf_tokenizers(both, corpus):
    mine, hf = both
    for t in list(corpus) + EXTRA:
        want = hf(t)["input_ids"]
        got = [mine.sot] + mine.encode(t) + [mine.eot]
        assert got == want, (t, got, want)


def test_html_unescape_like_clip(both):
    """CLIP's basic_clean unescapes HTML entities twice (HF's CLIPTokenizer does not)."""
    mine, _ = both
    assert mine.encode("kitchen &amp;amp; dining") == mine.encode("kitchen & dining")


def test_tokenize_padding_and_truncation(both):
    mine, _ = both
    a = mine.tokenize(["wnętrze z drewnem", "salon"], context_length=77)
    assert a.shape == (2, 77) and a.dtype == np.int32
    for row in a:
        n = int(np.argmax(row == mine.eot)) + 1
        assert row[0] == mine.sot and row[n - 1] == mine.eot and (row[n:] == 0).all()
        assert int(np.argmax(row)) == n - 1  # encode_text pools at argmax (the eot id is the max)
    long = " ".join(["słowo"] * 80)
    with pytest.raises(RuntimeError):
        mine.tokenize(long)
    t = mine.tokenize(long, truncate=True)
    assert t[0, -1] == mine.eot and (t[0] != 0).all()


def test_decode_round_trip(both, corpus):
    mine, _ = both
    for t in corpus[:50]:
        # CLIP's decode ends every pre-token with a space ("close-up" -> "close - up")
        assert mine.decode(mine.encode(t)).replace(" ", "") == TK.clean(t).replace(" ", "")


def test_read_merges_file(tmp_path, merges):
    p = tmp_path / "bpe.txt.gz"
    with gzip.open(p, "wt", encoding="utf-8") as f:
        f.write("#version: 0.2\n" + "\n".join(" ".join(m) for m in merges) + "\n")
    assert TK.read_merges(p, None) == merges
    assert TK.read_merges(p, 10) == merges[:10]
