"""GPU merge-rank encoder (gbpe_bpe_encode) vs the reference's
tokenizer-manager.js goldens and the oracle's restatement of it."""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "gpu-bpe_amd"))

import bpe_oracle as O  # noqa: E402
from gpubpe import BPEEngine, MergeEncoder, synth  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = BPEEngine().init()
    yield e
    e.close()


def test_merge_encode_vs_reference_goldens(engine):
    d = json.load(open(os.path.join(HERE, "golden", "ref_modules.json")))
    for inp, out in zip(d["inputs"]["merge_encode_cases"], d["outputs"]["merge_encode_cases"]):
        merges = inp["model"]["merges"]
        text = inp["text"]
        enc = MergeEncoder(engine, merges)
        got = enc.encode(text)["tokens"]
        assert got == out["tokens"], inp["name"]
        enc.destroy()


@pytest.mark.parametrize("kind,seed", [("english", 51), ("multilingual", 52), ("code", 53)])
def test_merge_encode_vs_oracle(engine, kind, seed):
    corpus = getattr(synth, kind)(60_000, seed=seed)
    merges = [m[:3] for m in O.train(corpus, 600)["merges"]]
    text = getattr(synth, kind)(12_000, seed=seed + 100)
    enc = MergeEncoder(engine, merges)
    assert enc.encode_bytes(text).tolist() == O.encode_merge_order(text, merges)


def test_merge_encode_edges(engine):
    a = ord("a")
    cases = [
        ([[a, a, 256]], b"a" * 9),                                  # overlapping run, left-to-right
        ([[a, a, 256], [256, a, 257], [256, 256, 258]], b"a" * 10_001 + b" aa"),   # run across 4096-byte chunks
        ([[256, a, 300], [a, a, 256]], b"aaaa"),                    # operand created later: never fires
        ([[a, ord("b"), 256], [a, ord("b"), 257], [256, ord("c"), 258]], b"abcabab c"),   # duplicate pair
        ([], b"hello"),
        ([[a, ord("b"), 256]], b""),
        ([[ord("x"), ord(" "), 256], [256, ord("y"), 257]], b"x yx y x"),   # merges across spaces
    ]
    for merges, text in cases:
        enc = MergeEncoder(engine, merges)
        assert enc.encode_bytes(text).tolist() == O.encode_merge_order(text, merges), (merges, text[:20])


def _np_merge_order(data: bytes, merges) -> np.ndarray:
    """numpy form of the oracle's encode_merge_order (one pass per merge, every
    occurrence left to right; runs of a == b pair up from their left end)."""
    tok = np.frombuffer(data, np.uint8).astype(np.int64)
    for a, b, nid in (m[:3] for m in merges):
        if tok.size < 2:
            break
        idx = np.flatnonzero((tok[:-1] == a) & (tok[1:] == b))
        if idx.size == 0:
            continue
        if a == b:
            k = np.arange(idx.size)
            start = np.ones(idx.size, bool)
            start[1:] = idx[1:] != idx[:-1] + 1
            rs = np.maximum.accumulate(np.where(start, k, 0))
            idx = idx[(k - rs) % 2 == 0]
        tok[idx] = nid
        rm = np.zeros(tok.size, bool)
        rm[idx + 1] = True
        tok = tok[~rm]
    return tok


def test_merge_encode_long_segment(engine):
    # a text with no cut at all (every byte pair of its alphabet is joined by some
    # merge): one segment of > 1 MB, encoded by the heap path on one lane; the
    # numpy restatement is first checked against the oracle on a 40 KB piece
    rng = np.random.default_rng(61)
    alpha = np.frombuffer(b"abcd", np.uint8)
    letters = alpha.tolist()
    order = rng.permutation(16)   # every byte pair of the alphabet merges (in a random rank order) ...
    merges = [[letters[k // 4], letters[k % 4], 256 + r] for r, k in enumerate(order.tolist())]
    for r in range(40):           # ... and so do pairs of those tokens
        i, j = rng.integers(0, 16, 2).tolist()
        merges.append([256 + i, 256 + j, 272 + r])
    small = bytes(alpha[rng.integers(0, 4, 40_000)])
    assert _np_merge_order(small, merges).tolist() == O.encode_merge_order(small, merges)
    big = bytes(alpha[rng.integers(0, 4, 1_300_000)])
    enc = MergeEncoder(engine, merges)
    got = enc.encode_bytes(big)
    assert np.array_equal(np.asarray(got, dtype=np.int64), _np_merge_order(big, merges))
    # a long run of one byte (a == b pairs) plus short segments around it
    text = b"xy " + b"a" * 300_000 + b" yx"
    m2 = [[97, 97, 256], [256, 97, 257], [256, 256, 258], [258, 258, 259]]
    enc2 = MergeEncoder(engine, m2)
    assert enc2.encode_bytes(text).tolist() == _np_merge_order(text, m2).tolist()
    enc.destroy()
    enc2.destroy()
