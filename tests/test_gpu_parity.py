"""GPU parity: the HIP path through the C-ABI vs the CPU oracle.

Bit-exact for everything (integer / byte / index work): merge lists
[a, b, id, count], final symbol streams, live pair counts, token ids.
"""
import ctypes as C

import numpy as np
import pytest

import bpe_oracle as O
from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from gpubpe import BPEEngine
    return BPEEngine(0).init()


def _train_native(eng, data: bytes, target: int, exact=False, word_starts=None, batch=128, next_id=256,
                  vocab_size=None, table_log2=0, max_steps=None, sparse=None):
    """Drive the stepwise C-ABI directly; returns merges, final stream, live pair counts, stats.
    sparse: None = the library's policy, "dense" = dense loop only, "early" = sector-sparse
    loop from the first step boundary where its zone fits."""
    from gpubpe import _lib
    lib = _lib.load()
    ctx = eng.device
    flags = _lib.GBPE_TRAIN_EXACT_COMPACTION if exact else 0
    flags |= {None: 0, "dense": _lib.GBPE_TRAIN_DENSE_ONLY, "early": _lib.GBPE_TRAIN_SPARSE_EARLY}[sparse]
    opts = _lib.TrainOpts(target_vocab_size=target, vocab_size=vocab_size or next_id, next_token_id=next_id,
                          batch_size=batch, flags=flags, table_log2=table_log2)
    tr = C.c_void_p()
    buf = C.create_string_buffer(data, len(data))
    ws = None
    if word_starts is not None:
        ws = np.ascontiguousarray(word_starts, dtype=np.uint8)
    _lib.check(lib.gbpe_trainer_create(ctx, buf, len(data), ws.ctypes.data_as(C.c_void_p) if ws is not None else None,
                                       0, C.byref(opts), C.byref(tr)), ctx, "create")
    merges, steps = [], 0
    try:
        out = (C.c_uint32 * (4 * batch))()
        while True:
            nd, es = C.c_uint32(), C.c_uint32()
            _lib.check(lib.gbpe_trainer_step(tr, batch, out, C.byref(nd), C.byref(es)), ctx, "step")
            merges += [list(out[4 * i:4 * i + 4]) for i in range(nd.value)]
            steps += 1
            if nd.value == 0 or es.value or (max_steps and steps >= max_steps):
                break
        n = C.c_uint64()
        lib.gbpe_trainer_symbols(tr, None, 0, C.byref(n))
        syms = np.zeros(n.value, np.uint32)
        _lib.check(lib.gbpe_trainer_symbols(tr, syms.ctypes.data_as(_lib.u32p), n.value, C.byref(n)), ctx, "symbols")
        cap = 1 << 22
        pids = np.zeros(cap, np.uint32)
        cnts = np.zeros(cap, np.uint32)
        npairs = C.c_uint64()
        _lib.check(lib.gbpe_trainer_pair_counts(tr, pids.ctypes.data_as(_lib.u32p), cnts.ctypes.data_as(_lib.u32p),
                                                cap, C.byref(npairs)), ctx, "pairs")
        order = np.argsort(pids[:npairs.value])
        st = _lib.TrainerStats()
        lib.gbpe_trainer_stats_get(tr, C.byref(st))
    finally:
        lib.gbpe_trainer_destroy(tr)
    return merges, syms, (pids[:npairs.value][order], cnts[:npairs.value][order]), st


def _assert_counts_match_stream(pairs, syms):
    up, uc = O.count_pairs(syms.astype(np.uint32))
    assert np.array_equal(pairs[0], up), "live pair set differs from a recount of the stream"
    assert np.array_equal(pairs[1].astype(np.int64), uc), "pair counts differ from a recount of the stream"


def _text(c):
    return bytes.fromhex(c["text_hex"]) if "text_hex" in c else c["text"].encode("utf-8")


def test_known_answers(eng):
    import json, os
    ka = json.load(open(os.path.join(GOLDEN, "known_answers.json")))
    for c in ka["train"]:
        nid = c.get("next_token_id", 256)
        for exact in (False, True):
            for batch in [128] + c.get("batches", []):   # small batches: the odd-batch ping-pong swap
                m, s, pairs, st = _train_native(eng, _text(c), c["target"], exact=exact, batch=batch, next_id=nid)
                want = c["merges_exact"] if exact and "merges_exact" in c else c["merges"]
                assert m == want, (c["name"], exact, batch)
                if "early_stop" in c:
                    assert bool(st.early_stop) == c["early_stop"], (c["name"], exact, batch)
                key = "final_stream_exact" if exact else "final_stream"
                if key in c:
                    assert s.tolist() == c[key], (c["name"], exact, batch)
                _assert_counts_match_stream(pairs, s)


@pytest.mark.parametrize("kind,size,target", [("english", 65536, 1024), ("multilingual", 65536, 700),
                                              ("code", 65536, 900), ("english", 300000, 2048)])
@pytest.mark.parametrize("exact", [False, True])
def test_train_matches_oracle(eng, kind, size, target, exact):
    from gpubpe import synth
    data = getattr(synth, kind)(size, seed=size % 97 + 3)
    ref = O.train(data, target, compaction="exact" if exact else "reference")
    m, s, pairs, st = _train_native(eng, data, target, exact=exact)
    assert m == ref["merges"]
    assert np.array_equal(s, ref["symbols"])
    _assert_counts_match_stream(pairs, s)
    if not exact:
        assert st.tail_dropped == sum(ref["tail_drops"])


@pytest.mark.parametrize("exact", [False, True])
def test_train_multitile_delta(eng, monkeypatch, exact):
    # GBPE_DEBUG=delta_mt=1: every dense merge runs k_delta_mt (8 tiles per workgroup,
    # the last workgroup partial), which the library otherwise keeps for >= 2048 tiles
    from gpubpe import synth
    monkeypatch.setenv("GBPE_DEBUG", "delta_mt=1")
    data = synth.english(300000, seed=41)
    ref = O.train(data, 1500, compaction="exact" if exact else "reference")
    m, s, pairs, st = _train_native(eng, data, 1500, exact=exact, sparse="dense")
    assert m == ref["merges"]
    assert np.array_equal(s, ref["symbols"])
    _assert_counts_match_stream(pairs, s)
    if not exact:
        assert st.tail_dropped == sum(ref["tail_drops"])


def test_u32_symbol_path(eng):
    # target > 32768 forces 32-bit symbols (bit 16 = word start)
    from gpubpe import synth
    data = synth.english(40000, seed=21)
    ref = O.train(data, 40000)
    m, s, pairs, st = _train_native(eng, data, 40000)
    assert st.bytes_per_symbol == 4
    assert m == ref["merges"] and np.array_equal(s, ref["symbols"])
    _assert_counts_match_stream(pairs, s)


def test_odd_batches_and_resumed_ids(eng):
    from gpubpe import synth
    data = synth.multilingual(50000, seed=5)
    ref = O.train(data, 700, next_token_id=300, vocab_size=300)
    m, s, pairs, _ = _train_native(eng, data, 700, batch=7, next_id=300, vocab_size=300)
    assert m == ref["merges"] and np.array_equal(s, ref["symbols"])
    _assert_counts_match_stream(pairs, s)


def test_external_word_starts(eng):
    from gpubpe import synth
    data = synth.code(60000, seed=9)
    rng = np.random.default_rng(3)
    ws = (rng.random(len(data)) < 0.2).astype(np.uint8)
    ws[0] = 1
    for exact in (False, True):
        ref = O.train(data, 800, word_starts=ws, compaction="exact" if exact else "reference")
        m, s, pairs, _ = _train_native(eng, data, 800, word_starts=ws, exact=exact)
        assert m == ref["merges"] and np.array_equal(s, ref["symbols"])
        _assert_counts_match_stream(pairs, s)


def test_table_rebuild_small_table(eng):
    # a tiny pair table forces rebuilds between steps; results must not change
    from gpubpe import synth
    data = synth.multilingual(120000, seed=13)
    ref = O.train(data, 1500)
    m, s, pairs, st = _train_native(eng, data, 1500, table_log2=15, batch=16)
    assert m == ref["merges"] and np.array_equal(s, ref["symbols"])
    _assert_counts_match_stream(pairs, s)


def test_table_grows_when_crowded(eng):
    # a 2^13-slot table outgrown by the live pairs is rebuilt larger (more than once);
    # results must not change, dense or with the sector-sparse loop entering later
    from gpubpe import synth
    data = synth.english(300000, seed=41)
    ref = O.train(data, 1200)
    for sparse in (None, "dense"):
        m, s, pairs, st = _train_native(eng, data, 1200, table_log2=13, batch=16, sparse=sparse)
        assert m == ref["merges"] and np.array_equal(s, ref["symbols"])
        _assert_counts_match_stream(pairs, s)
        assert st.table_slots >= 1 << 15, st.table_slots


def test_table_grows_inside_sparse_loop(eng, monkeypatch):
    # inside the sector-sparse loop a crowded table moves its live entries to a
    # larger one (k_rehash) instead of leaving the loop for a dense recount: same
    # merges and counts, fewer sparse -> dense exits than the recount path
    from gpubpe import synth
    data = synth.english(300000, seed=41)
    ref = O.train(data, 1200)
    exits = {}
    for rehash in ("1", "0"):
        monkeypatch.setenv("GBPE_DEBUG", f"rehash={rehash}")
        m, s, pairs, st = _train_native(eng, data, 1200, table_log2=13, batch=16, sparse="early")
        assert m == ref["merges"] and np.array_equal(s, ref["symbols"])
        _assert_counts_match_stream(pairs, s)
        assert st.table_slots >= 1 << 15, st.table_slots
        exits[rehash] = st.sparse_exits
    assert exits["1"] < exits["0"], exits


def test_random_bytes_and_runs(eng):
    rng = np.random.default_rng(17)
    for trial in range(6):
        alphabet = rng.choice(256, size=rng.integers(2, 6), replace=False).astype(np.uint8)
        n = int(rng.integers(1, 5000))
        data = bytes(rng.choice(alphabet, size=n))
        for exact in (False, True):
            ref = O.train(data, 400, compaction="exact" if exact else "reference")
            m, s, pairs, _ = _train_native(eng, data, 400, exact=exact)
            assert m == ref["merges"], (trial, exact)
            assert np.array_equal(s, ref["symbols"]), (trial, exact)
            _assert_counts_match_stream(pairs, s)


def test_empty_corpus_error(eng):
    from gpubpe import BPETrainer
    with pytest.raises(ValueError, match="empty"):
        BPETrainer(eng).train(b"", 300)


def test_trainer_api_and_persistent_vocab(eng):
    from gpubpe import BPETrainer, synth
    t = BPETrainer(eng)
    d1 = synth.english(30000, seed=1)
    r1 = t.train(d1, target_vocab_size=500)
    ref1 = O.train(d1, 500)
    assert r1["merges"] == [m[:3] for m in ref1["merges"]]
    assert r1["vocabSize"] == 256 + len(r1["merges"])
    # a second call continues numbering from the persisted vocab (trainer.js:136, 191, 208)
    d2 = synth.english(30000, seed=2)
    r2 = t.train(d2, target_vocab_size=700)
    ref2 = O.train(d2, 700, next_token_id=r1["vocabSize"], vocab_size=r1["vocabSize"])
    assert r2["merges"] == [m[:3] for m in ref2["merges"]]
    assert r2["vocabSize"] == r1["vocabSize"] + len(r2["merges"])
    v = O.vocab_from_merges(r1["merges"] + r2["merges"])
    assert t.export_vocab() == v.export()


def test_word_boundary_known_answers_gpu(eng):
    # the hand-traced byte-class cases (train.wgsl:111-185) through the device kernel
    import json, os
    from gpubpe import _lib
    lib = _lib.load()
    ka = json.load(open(os.path.join(GOLDEN, "known_answers.json")))
    for c in ka["word_boundary"]:
        data = bytes.fromhex(c["text_hex"]) if "text_hex" in c else c["text"].encode("utf-8")
        out = np.zeros(len(data), np.uint8)
        _lib.check(lib.gbpe_word_boundary(eng.device, data, len(data), out.ctypes.data_as(C.c_void_p)), eng.device, "wb")
        assert out.astype(int).tolist() == c["ws"], c["name"]


def test_word_boundary_kernel(eng):
    from gpubpe import _lib
    lib = _lib.load()
    rng = np.random.default_rng(4)
    data = bytes(rng.integers(0, 256, size=100000, dtype=np.uint8)) + b"Hi, you 42x\n  y"
    out = np.zeros(len(data), np.uint8)
    _lib.check(lib.gbpe_word_boundary(eng.device, data, len(data), out.ctypes.data_as(C.c_void_p)), eng.device, "wb")
    want = O.heuristic_word_starts(np.frombuffer(data, np.uint8)).astype(np.uint8)
    assert np.array_equal(out, want)


# ── encode ──────────────────────────────────────────────────────────────────

def _oracle_encode(vocab, text, cs):
    blob = O.compile_vocab_to_trie(vocab)
    nodes, edges = O.parse_trie_buffers(blob, O.parse_header(blob))
    return O.encode_chunked(text, nodes, edges, cs)


def test_encode_known_answers(eng):
    import json, os
    from gpubpe import TrieTokenizer
    ka = json.load(open(os.path.join(GOLDEN, "known_answers.json")))
    for c in ka["encode"]:
        if "vocab_holes" in c:
            vh = c["vocab_holes"]
            voc = [[] for _ in range(vh["size"])]
            for k, v in vh["entries"].items():
                voc[int(k)] = v
        else:
            voc = O.vocab_from_merges(c["merges"]).entries
        tok = TrieTokenizer.from_vocab(eng, voc, chunk_size=c["chunk_size"])
        assert tok.encode_bytes(_text(c)).tolist() == c["tokens"], c["name"]
        tok.destroy()


@pytest.mark.parametrize("cs", [None, 1, 7, 64, 512, 2048])
def test_encode_matches_oracle(eng, cs):
    from gpubpe import TrieTokenizer, synth
    train = synth.multilingual(80000, seed=31)
    vocab = O.vocab_from_merges(O.train(train, 1200, compaction="exact")["merges"]).entries
    text = synth.multilingual(150000, seed=32)
    tok = TrieTokenizer.from_vocab(eng, vocab, chunk_size=cs)
    got = tok.encode_bytes(text)
    want = _oracle_encode(vocab, text, tok.chunk_size)
    assert np.array_equal(got, want)
    assert tok.decode(got) == text
    tok.destroy()


@pytest.mark.parametrize("cs", [None, 7, 64])
def test_encode_host_pipeline_slices(eng, cs, monkeypatch):
    # gbpe_encode (host buffers) pipelines chunk-aligned slices with a second
    # readback thread; a tiny slice makes a 150 KB input dozens of slices, and the
    # tokens must equal one device pass (gbpe_encode_device) and the oracle
    from gpubpe import TrieTokenizer, synth
    train = synth.multilingual(80000, seed=31)
    vocab = O.vocab_from_merges(O.train(train, 1200, compaction="exact")["merges"]).entries
    text = synth.multilingual(150000, seed=33)
    tok = TrieTokenizer.from_vocab(eng, vocab, chunk_size=cs)
    want = _oracle_encode(vocab, text, tok.chunk_size)
    monkeypatch.setenv("GBPE_DEBUG", "encode_slice=4096")
    got = tok.encode_bytes(text)
    assert np.array_equal(got, want)
    monkeypatch.delenv("GBPE_DEBUG")
    assert np.array_equal(tok.encode_bytes(text), want)
    tok.destroy()


def test_encode_edge_cases(eng):
    from gpubpe import TrieTokenizer
    vocab = O.vocab_from_merges([[116, 104], [256, 101], [32, 257]]).entries
    tok = TrieTokenizer.from_vocab(eng, vocab)
    assert tok.encode_bytes(b"").tolist() == []
    assert tok.encode_bytes(b"t").tolist() == [116]
    for n in (1, 2, 3, 4, 5, 511, 512, 513, 1023, 1025):
        text = (b"the then " * 200)[:n]
        assert np.array_equal(tok.encode_bytes(text), _oracle_encode(vocab, text, tok.chunk_size)), n
    assert tok.decode([70000]) == bytes([0xEF, 0xBF, 0xBD])


def test_encode_wide_token_ids(eng):
    # token ids >= 65536 exercise the 32-bit scratch path
    from gpubpe import TrieTokenizer
    voc = [[b] for b in range(256)] + [[] for _ in range(70000)]
    voc[70100] = [97, 98, 99]
    voc[65600] = [97, 98]
    tok = TrieTokenizer.from_vocab(eng, voc, chunk_size=16)
    text = b"abcab xabc" * 50
    got = tok.encode_bytes(text)
    assert np.array_equal(got, _oracle_encode(voc, text, 16))
    assert 70100 in got.tolist()


def test_encode_v2_trie_parse(eng):
    # a v2 trie (8-byte nodes, 4-byte edges) is accepted (trie.js:140-141)
    import struct
    from gpubpe import TrieTokenizer
    nodes = [(0, 2, 0xFFFF), (0, 0, 97), (2, 1, 98), (0, 0, 300)]     # root->'a','b'; 'b'->'c'(300)
    edges = [(97, 1), (98, 2), (99, 3)]
    blob = struct.pack("<7I", 0x54524945, 2, len(nodes), len(edges), 2, 301, 0)
    blob += b"".join(struct.pack("<4H", fc, nc, tid, 0) for fc, nc, tid in nodes)
    blob += b"".join(struct.pack("<2H", s, t) for s, t in edges)
    tok = TrieTokenizer(eng, blob, chunk_size=512)
    assert tok.encode_bytes(b"abcbbx").tolist() == [97, 300, 98, 98, 120]


@pytest.mark.parametrize("exact", [False, True])
def test_train_large_vs_c_oracle(eng, exact):
    # 24 MiB: thousands of tiles, so the two-level tile prefix (group sums) and
    # multi-block stale-tail windows are exercised; checked against the C restatement
    import cpu_ref
    from gpubpe import synth
    data = synth.english(24 << 20, seed=77, fancy_punct=0.005)
    k = 300
    ref = cpu_ref.train(data, 256 + k, exact=exact, threads=16)
    m, s, pairs, st = _train_native(eng, data, 256 + k, exact=exact)
    assert m == ref["merges"]
    assert np.array_equal(s, ref["symbols"])
    _assert_counts_match_stream(pairs, s)
    if not exact:
        assert st.tail_dropped == ref["tail_total"]


@pytest.mark.parametrize("off", [0, 1, 7, 16])
@pytest.mark.parametrize("n", [40_000, 40_013])
def test_symbols_device_input_alignment(eng, off, n):
    """Trainer creation from a device pointer at any byte offset and any length: the
    16-byte symbol kernel (aligned input, whole vectors, a ragged last vector) and the
    byte-per-thread one (unaligned input) give the reference's merges and stream."""
    from gpubpe import _lib, synth
    lib = _lib.load()
    ctx = eng.device
    data = synth.english(n, seed=11)
    ref = O.train(data, 700)
    want = [list(m[:4]) for m in ref["merges"]]
    d = C.c_void_p()
    _lib.check(lib.gbpe_device_alloc(ctx, n + 64, C.byref(d)), ctx, "alloc")
    try:
        pad = bytes([0x41]) * off
        _lib.check(lib.gbpe_memcpy_h2d(ctx, d, pad + data, n + off), ctx, "h2d")
        opts = _lib.TrainOpts(target_vocab_size=700, vocab_size=256, next_token_id=256, batch_size=128,
                              flags=0, table_log2=0)
        tr = C.c_void_p()
        _lib.check(lib.gbpe_trainer_create(ctx, C.c_void_p(d.value + off), n, None, 1, C.byref(opts), C.byref(tr)),
                   ctx, "create")
        try:
            merges, out = [], (C.c_uint32 * 512)()
            while True:
                nd, es = C.c_uint32(), C.c_uint32()
                _lib.check(lib.gbpe_trainer_step(tr, 128, out, C.byref(nd), C.byref(es)), ctx, "step")
                merges += [list(out[4 * i:4 * i + 4]) for i in range(nd.value)]
                if nd.value == 0 or es.value:
                    break
            nn = C.c_uint64()
            lib.gbpe_trainer_symbols(tr, None, 0, C.byref(nn))
            syms = np.zeros(nn.value, np.uint32)
            _lib.check(lib.gbpe_trainer_symbols(tr, syms.ctypes.data_as(_lib.u32p), nn.value, C.byref(nn)), ctx, "sym")
        finally:
            lib.gbpe_trainer_destroy(tr)
    finally:
        lib.gbpe_device_free(ctx, d)
    assert [m[:4] for m in merges] == [m[:4] for m in want]
    assert np.array_equal(syms, np.asarray(ref["symbols"], dtype=np.uint32))
