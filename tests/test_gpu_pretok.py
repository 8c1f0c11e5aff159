"""GPT-4 rule word starts on the GPU (gbpe_pretokenize_gpt4) vs the reference's
pre_tokenizer.mjs goldens and the oracle restatement, plus training with the
device-computed mask (GBPE_TRAIN_GPT4_BOUNDARIES) vs the oracle."""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "gpu-bpe_amd"))

import bpe_oracle as O  # noqa: E402
from gpubpe import BPEEngine, BPETrainer, GpuPreTokenizer, _lib, synth  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = BPEEngine().init()
    yield e
    e.close()


def gpu_ws(engine, data: bytes) -> np.ndarray:
    return GpuPreTokenizer(engine).pre_tokenize_bytes(data)["wordStarts"]


def assert_same(got, exp, data, what=""):
    bad = np.flatnonzero(got != exp)
    assert bad.size == 0, f"{what}: {bad.size} mismatches, first {[(int(i), int(got[i]), int(exp[i]), data[max(0, i - 8):i + 8]) for i in bad[:5]]}"


def test_gpu_pretok_vs_reference_goldens(engine):
    d = json.load(open(os.path.join(HERE, "golden", "ref_pretok.json")))
    for inp, out in zip(d["inputs"], d["outputs"]):
        exp = np.frombuffer(bytes.fromhex(out["word_starts"]), np.uint8)
        np.testing.assert_array_equal(gpu_ws(engine, bytes.fromhex(inp["hex"])), exp, err_msg=inp["name"])


@pytest.mark.parametrize("kind,n,seed", [("code", 400_000, 41), ("multilingual", 300_000, 42),
                                         ("english", 300_000, 43)])
def test_gpu_pretok_vs_oracle_synthetic(engine, kind, n, seed):
    data = getattr(synth, kind)(n, seed=seed)
    exp = O.gpt4_word_starts(data)
    for rep in range(3):   # repeated calls: allocator reuse must not change the result
        assert_same(gpu_ws(engine, data), exp, data, f"{kind} rep {rep}")


def test_gpu_pretok_edges(engine):
    cases = [
        b"",
        b"x",
        b"7",
        "ğ".encode()[:1],                                # truncated 2-byte sequence
        "a你".encode()[:-1],                             # truncated 3-byte sequence at the end
        b"1" * 10_000 + b" x " + b"9" * 8191,            # digit runs across 4096-byte blocks
        (b"ab'll 12 " * 600) + "’s ’re ’ve’".encode(),
        b"\r\n\r\n  \t  \n",
        ("٣" * 5000).encode() + b"12345",                # multi-byte digits across blocks
    ]
    for c in cases:
        np.testing.assert_array_equal(gpu_ws(engine, c), O.gpt4_word_starts(c), err_msg=repr(c[:40]))


@pytest.mark.parametrize("exact", [False, True])
def test_train_with_gpt4_boundaries(engine, exact):
    data = synth.code(200_000, seed=44)
    tr = BPETrainer(engine, exact_compaction=exact)
    tr._flags |= _lib.GBPE_TRAIN_GPT4_BOUNDARIES        # device-computed GPT-4 word starts
    got = tr.train(data, target_vocab_size=700)
    exp = O.train(data, 700, word_starts=O.gpt4_word_starts(data), compaction="exact" if exact else "reference")
    assert [m[:3] for m in exp["merges"]] == [list(m) for m in got["merges"]]
    # the same run through the PreTokenizer-shaped API (external mask, trainer.js:62-99)
    got2 = BPETrainer(engine, exact_compaction=exact).train(data, target_vocab_size=700,
                                                            pre_tokenizer=GpuPreTokenizer(engine))
    assert got2["merges"] == got["merges"]
