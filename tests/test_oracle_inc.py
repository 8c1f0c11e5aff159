"""The incremental restatement (oracle/bpe_oracle_inc.c) that produces the
full-length fixtures must equal the full-recount restatement (oracle/bpe_oracle.c,
the reference algorithm per merge) merge-for-merge, symbol-for-symbol and in the
stale-tail total, in both compaction modes, with heuristic and external word
starts, on runs, random bytes, and ids reaching the 0xFFFF stop (train.wgsl:345).
Also: the committed fixtures are well-formed, and the first C2 fixture merges
are re-derived here by the full recount.  CPU only."""
import numpy as np
import pytest

import bpe_oracle as O
import cpu_ref


def _same(data, target, **kw):
    a = cpu_ref.train(data, target, **kw)
    b = cpu_ref.train_inc(data, target, **kw)
    assert a["merges"] == b["merges"]
    assert np.array_equal(a["symbols"], b["symbols"])
    assert a["tail_total"] == b["tail_total"] and a["early_stop"] == b["early_stop"]
    return a


@pytest.mark.parametrize("exact", [False, True])
def test_inc_english_c1(exact):
    from gpubpe import synth
    r = _same(synth.english(262144, seed=1), 1024, exact=exact)
    assert len(r["merges"]) == 768


@pytest.mark.parametrize("name", ["c1", "c1x"])
def test_c1_fixture_is_the_full_recount(name):
    # the committed C1 fixtures (GPU test + bench leg) equal the reference algorithm
    # restated as a full recount per merge (oracle/bpe_oracle.c)
    import hashlib
    import gen_golden_train as G
    want, meta = G.load_train(name)
    data = G.corpus(meta["corpus"])
    assert hashlib.sha256(data).hexdigest() == meta["corpus_sha256"]
    r = cpu_ref.train(data, meta["target_vocab"], exact=meta["compaction"] == "exact")
    assert np.array_equal(np.array(r["merges"], dtype=np.uint32), want)
    assert r["tail_total"] == meta["tail_total"] and int(r["symbols"].shape[0]) == meta["final_n"]
    syms = np.ascontiguousarray(r["symbols"], dtype="<u4")
    assert hashlib.sha256(syms.tobytes()).hexdigest() == meta["final_stream_sha256"]


def test_inc_multilingual_and_code_gpt4():
    from gpubpe import synth
    _same(synth.multilingual(1 << 19, seed=4), 2000)
    code = synth.code(1 << 19, seed=6)
    ws = cpu_ref.gpt4_word_starts_ascii(code)
    assert np.array_equal(ws[:100000], O.gpt4_word_starts(code[:100000]))
    _same(code, 2000, word_starts=ws)


def test_inc_known_answers_runs_random():
    for data in (b"aaaa", b"aaa aaa", b"aaaaaaa bbbb aaaa ab" * 500, b"\x00a\x00a\x00aa"):
        _same(data, 300)
    rng = np.random.default_rng(0)
    for k in range(4):
        alpha = rng.choice(256, size=2 + k, replace=False).astype(np.uint8)
        _same(bytes(rng.choice(alpha, size=30000)), 1200, exact=bool(k & 1))


def test_inc_id_limit_stop():
    from gpubpe import synth
    r = _same(synth.english(100000, seed=3), 66000, next_token_id=65000)
    assert r["early_stop"] and r["merges"][-1][2] == 0xFFFF


def test_fixtures_well_formed():
    import gen_golden_train as G
    for name in ("c2", "c3vocab"):
        m, meta = G.load_train(name)
        assert m.shape == (meta["n_merges"], 4)
        assert np.array_equal(m[:, 2], 256 + np.arange(m.shape[0]))
        assert (m[:, 3] >= 2).all()


def test_c2_fixture_head_by_full_recount():
    import gen_golden_train as G
    m, meta = G.load_train("c2")
    data = G.corpus(meta["corpus"])
    import hashlib
    assert hashlib.sha256(data).hexdigest() == meta["corpus_sha256"]
    r = cpu_ref.train(data, 32768, max_merges=12, want_symbols=False)
    assert r["merges"] == m[:12].tolist()
