"""Full-length GPU parity at the benchmark configurations, against committed
oracle fixtures (tests/golden/train_*.npz, encode_*.json; oracle/gen_golden_train.py).

Every merge [a, b, id, count] of a whole training run, the final stream length,
the reference compaction's stale-tail total and the sha256 of the final symbol
stream must equal the CPU restatement's.  Configurations:

* c1, c1x — C1 (BASELINE configs[0]): 256 KiB ASCII English, seed 1, 1K vocab,
            768 merges, reference and exact compaction
* c2      — 100 MiB English (the bench's C2 leg), 32K vocab, 32,512 merges
* en1g    — 1 GiB English @ 32K: the bench's headline workload
* code1g  — C5: 1 GiB code, 50K vocab (u32 symbols), GPT-4 rule word starts
            computed on the device (pre_tokenizer.mjs:226-292), 49,744 merges
* ml1g    — 1 GiB multilingual @ 32K
* ml1g64k — C4's rank-0 shard (1 GiB multilingual, seed 5) alone @ 64K (u32 symbols)
* c3      — C3's 32K vocab (100 MiB multilingual sample) trained on the GPU,
            then the chunked trie encode of 64 MiB and of 1 GiB multilingual
            text with it (token count and token-stream sha256)

The corpus sha256 in each fixture is checked first, so a numpy generator drift
on the box fails as a corpus mismatch, not as a parity failure.
"""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

import gen_golden_train as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from gpubpe import BPEEngine
    return BPEEngine(0).init()


def _sha(b) -> str:
    return hashlib.sha256(b).hexdigest()


def _train_full(eng, data: bytes, target: int, flags: int = 0):
    """One whole run through the stepwise C-ABI on HBM-resident input (as the
    bench runs it); returns merges [k, 4], stats, final stream (u32 LE)."""
    from gpubpe import _lib
    lib = _lib.load()
    ctx = eng.device
    d = C.c_void_p()
    _lib.check(lib.gbpe_device_alloc(ctx, len(data) + 64, C.byref(d)), ctx, "alloc")
    tr = C.c_void_p()
    try:
        _lib.check(lib.gbpe_memcpy_h2d(ctx, d, data, len(data)), ctx, "h2d")
        opts = _lib.TrainOpts(target_vocab_size=target, vocab_size=256, next_token_id=256, batch_size=128,
                              flags=flags, table_log2=0)
        _lib.check(lib.gbpe_trainer_create(ctx, d, len(data), None, 1, C.byref(opts), C.byref(tr)), ctx, "create")
        out = (C.c_uint32 * 512)()
        merges = []
        while True:
            nd, es = C.c_uint32(), C.c_uint32()
            _lib.check(lib.gbpe_trainer_step(tr, 128, out, C.byref(nd), C.byref(es)), ctx, "step")
            merges += list(out[: 4 * nd.value])
            if nd.value == 0 or es.value:
                break
        st = _lib.TrainerStats()
        lib.gbpe_trainer_stats_get(tr, C.byref(st))
        n = C.c_uint64()
        lib.gbpe_trainer_symbols(tr, None, 0, C.byref(n))
        syms = np.zeros(n.value, dtype="<u4")
        _lib.check(lib.gbpe_trainer_symbols(tr, syms.ctypes.data_as(_lib.u32p), n.value, C.byref(n)), ctx, "symbols")
    finally:
        if tr:
            lib.gbpe_trainer_destroy(tr)
        lib.gbpe_device_free(ctx, d)
    return np.array(merges, dtype=np.uint32).reshape(-1, 4), st, syms


def _check_train(eng, name: str):
    from gpubpe import _lib
    want, meta = G.load_train(name)
    data = G.corpus(meta["corpus"])
    assert _sha(data) == meta["corpus_sha256"], "corpus generator drift (numpy version?): not the fixture's input"
    flags = _lib.GBPE_TRAIN_GPT4_BOUNDARIES if meta["boundaries"] == "gpt4" else 0
    if meta.get("compaction") == "exact":
        flags |= _lib.GBPE_TRAIN_EXACT_COMPACTION
    got, st, syms = _train_full(eng, data, meta["target_vocab"], flags)
    assert got.shape == want.shape, (got.shape, want.shape)
    bad = np.flatnonzero((got != want).any(axis=1))
    assert bad.size == 0, f"first differing merge {bad[0]}: got {got[bad[0]].tolist()} want {want[bad[0]].tolist()}"
    assert int(st.symbol_count) == meta["final_n"]
    assert int(st.tail_dropped) == meta["tail_total"]
    assert bool(st.early_stop) == meta["early_stop"]
    assert _sha(syms.tobytes()) == meta["final_stream_sha256"]
    return st, syms


@pytest.mark.parametrize("name", ["c1", "c1x"])
def test_full_c1(eng, name):
    # C1 on the HIP path: every merge, the final stream and the stale-tail total
    st, _ = _check_train(eng, name)
    assert st.merges_done == 768 and st.bytes_per_symbol == 2


def test_full_c2_bench_corpus(eng):
    st, syms = _check_train(eng, "c2")
    assert st.sparse_merges > 30000 and st.bytes_per_symbol == 2


def test_full_en1g_headline(eng):
    st, _ = _check_train(eng, "en1g")
    assert st.sparse_merges > 30000


def test_full_code1g_c5_gpt4_u32(eng):
    st, _ = _check_train(eng, "code1g")
    assert st.bytes_per_symbol == 4


def test_full_ml1g(eng):
    _check_train(eng, "ml1g")


def test_full_ml1g64k_c4_shard(eng):
    # C4's rank-0 shard (1 GiB multilingual, seed 5) at C4's 64K vocab: ids past 0x7FFF
    # need the u32 layout, and the run ends at the 0xFFFF stop (train.wgsl:345)
    st, _ = _check_train(eng, "ml1g64k")
    assert st.bytes_per_symbol == 4


def _c3_tokenizer(eng):
    from gpubpe import TrieTokenizer, Vocab, compile_vocab_to_trie
    want, meta = G.load_train("c3vocab")
    voc = Vocab()
    for a, b, i, _ in want.tolist():
        assert voc.add_merge(a, b) == i
    blob = compile_vocab_to_trie(voc.entries)
    return TrieTokenizer(eng, blob, voc.entries), blob


def test_c3_vocab_train_and_encode_64m(eng):
    _check_train(eng, "c3vocab")
    tok, blob = _c3_tokenizer(eng)
    meta = json.load(open(os.path.join(G.GOLD, "encode_c3enc64m.json")))
    assert _sha(blob) == meta["trie_sha256"]           # product trie compile == oracle compile (trie.js)
    assert tok.chunk_size == meta["chunk_size"]         # tokenizer.js:67-68
    text = G.corpus(meta["corpus"])
    assert _sha(text) == meta["corpus_sha256"]
    ids = np.ascontiguousarray(tok.encode_bytes(text), dtype="<u4")
    assert ids.shape[0] == meta["n_tokens"]
    assert ids[:64].tolist() == meta["first_tokens"]
    assert _sha(ids.tobytes()) == meta["tokens_sha256"]


def test_c3_encode_1g(eng):
    tok, _ = _c3_tokenizer(eng)
    meta = json.load(open(os.path.join(G.GOLD, "encode_c3enc1g.json")))
    text = G.corpus(meta["corpus"])
    assert _sha(text) == meta["corpus_sha256"]
    ids = np.ascontiguousarray(tok.encode_bytes(text), dtype="<u4")
    assert ids.shape[0] == meta["n_tokens"]
    assert _sha(ids.tobytes()) == meta["tokens_sha256"]
