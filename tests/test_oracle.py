"""Pin the CPU oracle (oracle/bpe_oracle.py) before trusting it.

* against outputs of the reference's own vocab.js / trie.js /
  tokenizer-manager.js executed under Node 12 (tests/golden/ref_modules.json);
* against hand-derived known answers for the WGSL kernels
  (tests/golden/known_answers.json);
* against brute-force pure-Python restatements on random inputs.
"""
import json
import os

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

import bpe_oracle as O

from conftest import GOLDEN


@pytest.fixture(scope="module")
def ref():
    with open(os.path.join(GOLDEN, "ref_modules.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def ka():
    with open(os.path.join(GOLDEN, "known_answers.json")) as f:
        return json.load(f)


def _text(c):
    return bytes.fromhex(c["text_hex"]) if "text_hex" in c else c["text"].encode("utf-8")


# ── reference-module goldens ────────────────────────────────────────────────

def test_vocab_matches_reference_vocab_js(ref):
    for inp, out in zip(ref["inputs"]["vocab_cases"], ref["outputs"]["vocab_cases"]):
        v = O.Vocab()
        ids = [v.add_merge(a, b) for a, b in inp["merges"]]
        assert ids == out["ids"], inp["name"]
        assert v.entries == out["entries"], inp["name"]
        assert v.strings == out["strings"], inp["name"]
        assert v.size == out["size"] and v.next_token_id == out["nextTokenId"]
        assert v.export() == out["export"], inp["name"]


def test_trie_compile_matches_reference_trie_js(ref):
    for inp, out in zip(ref["inputs"]["trie_cases"], ref["outputs"]["trie_cases"]):
        blob = O.compile_vocab_to_trie(inp["vocab"])
        assert blob.hex() == out["trie_hex"], inp["name"]
        hdr = O.parse_header(blob)
        assert hdr == out["header"]
        nodes, edges = O.parse_trie_buffers(blob, hdr)
        assert nodes.tolist() == out["nodes"]
        assert edges.tolist() == out["edges"]


def test_merge_order_encode_matches_reference_tokenizer_manager(ref):
    for inp, out in zip(ref["inputs"]["merge_encode_cases"], ref["outputs"]["merge_encode_cases"]):
        toks = O.encode_merge_order(inp["text"].encode("utf-8"), inp["model"]["merges"])
        assert toks == out["tokens"], inp["name"]


def test_survey_trie_shape(ref):
    out = ref["outputs"]["trie_cases"][0]
    assert out["name"] == "survey_the"
    assert out["header"]["nodeCount"] == 262 and out["header"]["edgeCount"] == 261
    assert len(bytes.fromhex(out["trie_hex"])) == 5260


# ── hand-derived known answers (kernel semantics) ───────────────────────────

def test_train_known_answers(ka):
    for c in ka["train"]:
        nid = c.get("next_token_id", 256)
        r = O.train(_text(c), c["target"], next_token_id=nid)
        assert [m for m in r["merges"]] == c["merges"], c["name"]
        if "early_stop" in c:
            assert r["early_stop"] == c["early_stop"], c["name"]
        if "final_stream" in c:
            assert r["symbols"].tolist() == c["final_stream"], c["name"]
        rx = O.train(_text(c), c["target"], compaction="exact", next_token_id=nid)
        if "merges_exact" in c:
            assert rx["merges"] == c["merges_exact"], c["name"]
        if "final_stream_exact" in c:
            assert rx["symbols"].tolist() == c["final_stream_exact"], c["name"]


def test_word_boundary_known_answers(ka):
    for c in ka["word_boundary"]:
        data = np.frombuffer(_text(c), np.uint8)
        assert O.heuristic_word_starts(data).astype(int).tolist() == c["ws"]


def _known_vocab(c):
    if "vocab_holes" in c:
        vh = c["vocab_holes"]
        voc = [[] for _ in range(vh["size"])]
        for k, v in vh["entries"].items():
            voc[int(k)] = v
        return voc
    return O.vocab_from_merges(c["merges"]).entries


def test_encode_known_answers(ka):
    for c in ka["encode"]:
        blob = O.compile_vocab_to_trie(_known_vocab(c))
        nodes, edges = O.parse_trie_buffers(blob, O.parse_header(blob))
        toks = O.encode_chunked(_text(c), nodes, edges, c["chunk_size"])
        assert toks.tolist() == c["tokens"], c["name"]


# ── brute-force cross-checks ────────────────────────────────────────────────

def _brute_train(data: bytes, target: int, compaction: str):
    """Literal per-position restatement with Python lists (independent of numpy code)."""
    ws = O.heuristic_word_starts(np.frombuffer(data, np.uint8)).tolist()
    A = [b | (0x10000 if w else 0) for b, w in zip(data, ws)]
    B = [0] * len(A)
    cur, oth, n, nxt, merges = A, B, len(A), 256, []
    while len(merges) < target - 256:
        cnt = {}
        for i in range(1, n):
            s0, s1 = cur[i - 1], cur[i]
            if s1 & 0x10000 or not (s0 & 0xFFFF) or not (s1 & 0xFFFF):
                continue
            p = ((s0 & 0xFFFF) << 16) | (s1 & 0xFFFF)
            cnt[p] = cnt.get(p, 0) + 1
        best = (0, 0)
        for p, c in cnt.items():
            if c > best[0] or (c == best[0] and p < best[1]):
                best = (c, p)
        if best[0] < 2 or nxt > 0xFFFF:
            break
        a, b = best[1] >> 16, best[1] & 0xFFFF
        snap = cur[:n]
        valid, rw = [True] * n, [False] * n
        for i in range(n):
            raw = snap[i]
            nxt_raw = snap[i + 1] if i + 1 < n else 0
            prv_raw = snap[i - 1] if i > 0 else 0
            if i + 1 < n and not nxt_raw & 0x10000 and raw & 0xFFFF == a and nxt_raw & 0xFFFF == b:
                rw[i] = True
            if i > 0 and not raw & 0x10000 and prv_raw & 0xFFFF == a and raw & 0xFFFF == b:
                valid[i] = False
        for i in range(n):
            if rw[i]:
                cur[i] = nxt | (snap[i] & 0x10000)
        new_n = sum(valid)
        d = 0
        for i in range(n):
            if valid[i]:
                if compaction == "exact" or i < new_n:
                    oth[d] = cur[i]
                d += 1
        merges.append([a, b, nxt, best[0]])
        nxt += 1
        cur, oth, n = oth, cur, new_n
    return merges, cur[:n]


@settings(max_examples=60, deadline=None)
@given(st.lists(st.sampled_from(list(b"aabbc \n.0")), min_size=0, max_size=60),
       st.integers(min_value=256, max_value=290), st.sampled_from(["reference", "exact"]))
def test_train_matches_bruteforce(chars, target, compaction):
    data = bytes(chars)
    if not data:
        with pytest.raises(ValueError):
            O.train(data, target)
        return
    r = O.train(data, target, compaction=compaction)
    bm, bs = _brute_train(data, target, compaction)
    assert r["merges"] == bm
    assert r["symbols"].tolist() == bs


def test_ws_bit_of_merged_token_is_first_symbols():
    # "xab xab": the merged 'ab' keeps the A-side word-start flag (train.wgsl:486-487)
    r = O.train(b"ab ab", 257, compaction="exact")
    assert r["merges"] == [[97, 98, 256, 2]]


def test_external_word_starts_override_heuristic():
    data = b"abab"
    ws = np.array([1, 0, 1, 0], np.uint8)          # 'ab' 'ab' as two words
    r = O.train(data, 300, word_starts=ws, compaction="exact")
    # (b,a) crosses a word start, so only (a,b)=2 counts
    assert r["merges"] == [[97, 98, 256, 2]]
    assert r["symbols"].tolist() == [256 | 0x10000, 256 | 0x10000]


def test_chunked_encode_roundtrip_on_byte_complete_vocab():
    # with all 256 bytes in the vocab, decode(encode(x)) == x for any x and chunk size
    rng = np.random.default_rng(5)
    data = bytes(rng.integers(0, 256, size=3000, dtype=np.uint8))
    merges = O.train(data, 320, compaction="exact")["merges"]
    voc = O.vocab_from_merges(merges).entries
    blob = O.compile_vocab_to_trie(voc)
    nodes, edges = O.parse_trie_buffers(blob, O.parse_header(blob))
    for cs in (1, 7, 512):
        toks = O.encode_chunked(data, nodes, edges, cs)
        assert O.decode(toks, voc) == data


# ── C restatement (oracle/bpe_oracle.c) agrees with the numpy restatement ──

def test_c_oracle_matches_numpy_oracle():
    import cpu_ref
    import sys, os
    from gpubpe import synth
    for kind, size, target in (("english", 40000, 700), ("multilingual", 30000, 500), ("code", 30000, 600)):
        data = getattr(synth, kind)(size, seed=size % 11)
        for exact in (False, True):
            a = O.train(data, target, compaction="exact" if exact else "reference")
            b = cpu_ref.train(data, target, exact=exact, threads=4)
            assert b["merges"] == a["merges"], (kind, exact)
            assert np.array_equal(b["symbols"], a["symbols"]), (kind, exact)
            assert b["tail_total"] == sum(a["tail_drops"])


def test_c_oracle_known_answers(ka):
    import cpu_ref
    for c in ka["train"]:
        nid = c.get("next_token_id", 256)
        r = cpu_ref.train(_text(c), c["target"], threads=2, next_token_id=nid)
        assert r["merges"] == c["merges"], c["name"]
        if "final_stream" in c:
            assert r["symbols"].tolist() == c["final_stream"], c["name"]


def test_c_oracle_encode_matches_python():
    import cpu_ref
    from gpubpe import synth
    train = synth.english(20000, seed=2)
    voc = O.vocab_from_merges(O.train(train, 600, compaction="exact")["merges"]).entries
    blob = O.compile_vocab_to_trie(voc)
    nodes, edges = O.parse_trie_buffers(blob, O.parse_header(blob))
    text = synth.english(30000, seed=3)
    for cs in (1, 5, 512):
        assert np.array_equal(cpu_ref.encode(text, nodes, edges, cs, threads=4),
                              O.encode_chunked(text, nodes, edges, cs))


def test_gpt4_pretokenizer_oracle_vs_reference_goldens():
    """oracle.gpt4_word_starts vs the reference pre_tokenizer.mjs (tests/golden/ref_pretok.json)."""
    d = json.load(open(os.path.join(GOLDEN, "ref_pretok.json")))
    for inp, out in zip(d["inputs"], d["outputs"]):
        b = bytes.fromhex(inp["hex"])
        assert out["bytes"] == inp["hex"]          # NFC input: bytes pass through
        exp = np.frombuffer(bytes.fromhex(out["word_starts"]), np.uint8)
        np.testing.assert_array_equal(O.gpt4_word_starts(b), exp, err_msg=inp["name"])
