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
