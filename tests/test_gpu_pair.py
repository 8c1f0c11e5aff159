"""GPU parity of paired k_body launches against the CPU oracle.

A launch runs two merges when the table's top two pairs P1 > P2 are token-disjoint
(P2 is then provably the argmax after P1), and — under the reference compaction —
when the stale window merge 1 appends cannot lift another pair over P2 or change
P2's count (zone_two's verdict).  These cases force the sector-sparse loop on early
so the late (zone_one) form, where launches pair, runs from the first steps, and
check every merge [a, b, id, count], the final stream and the live pair counts in
both compaction modes, on corpora with same-symbol runs (a == b), count ties, token
0 and external word starts; and that the pairing itself happened (paired_merges),
and that GBPE_DEBUG=pair=0 (one merge per launch) gives the same results.
"""
import numpy as np
import pytest

import bpe_oracle as O
from test_gpu_parity import _train_native, _assert_counts_match_stream

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from gpubpe import BPEEngine
    return BPEEngine(0).init()


def _corpus(kind):
    from gpubpe import synth
    rng = np.random.default_rng(71)
    if kind == "english":
        return synth.english(200000, seed=43)
    if kind == "runs":   # same-symbol runs (a == b collapses) inside words
        words = [b"aa", b"aaaa", b"zzz", b"abab", b"baaab", b"zzzzzz", b"ab", b"ba"]
        return b" ".join(words[i] for i in rng.integers(0, len(words), 30000))
    if kind == "ties":   # every word equally frequent: many equal counts, the pid tie-break decides
        words = [bytes(rng.choice(list(b"abcdefghij"), size=int(rng.integers(2, 6)))) for _ in range(400)]
        return b" ".join(words * 40)
    if kind == "nul":    # token 0 never pairs (train.wgsl:395-399)
        d = bytearray(synth.english(80000, seed=47))
        for i in rng.integers(0, len(d), 3000):
            d[i] = 0
        return bytes(d)
    raise ValueError(kind)


@pytest.mark.parametrize("kind,target,batch", [("english", 1800, 128), ("runs", 600, 16), ("ties", 900, 32),
                                               ("nul", 1200, 64)])
@pytest.mark.parametrize("exact", [False, True])
def test_paired_launches_match_oracle(eng, kind, target, batch, exact):
    data = _corpus(kind)
    ref = O.train(data, target, compaction="exact" if exact else "reference")
    m, s, pairs, st = _train_native(eng, data, target, exact=exact, batch=batch, sparse="early")
    assert st.sparse_merges > 0
    assert m == ref["merges"]
    assert np.array_equal(s, ref["symbols"])
    _assert_counts_match_stream(pairs, s)
    if not exact:
        assert st.tail_dropped == sum(ref["tail_drops"])
    if kind == "english":
        assert st.paired_merges > 0   # the case the test exists for


def test_paired_external_word_starts_and_u32(eng):
    from gpubpe import synth
    code = synth.code(90000, seed=11)
    ws = (np.random.default_rng(5).random(len(code)) < 0.15).astype(np.uint8)
    ws[0] = 1
    for exact in (False, True):
        ref = O.train(code, 1000, word_starts=ws, compaction="exact" if exact else "reference")
        m, s, pairs, st = _train_native(eng, code, 1000, word_starts=ws, exact=exact, batch=32, sparse="early")
        assert m == ref["merges"] and np.array_equal(s, ref["symbols"])
        _assert_counts_match_stream(pairs, s)
    data = synth.english(60000, seed=23)   # a 40K vocab: u32 symbols
    ref = O.train(data, 40000)
    m, s, pairs, st = _train_native(eng, data, 40000, batch=64, sparse="early")
    assert st.bytes_per_symbol == 4
    assert m == ref["merges"] and np.array_equal(s, ref["symbols"])
    _assert_counts_match_stream(pairs, s)


def test_pairing_off_gives_the_same_run(eng, monkeypatch):
    from gpubpe import synth
    data = synth.multilingual(150000, seed=17)
    on = _train_native(eng, data, 1500, batch=128, sparse="early")
    monkeypatch.setenv("GBPE_DEBUG", "pair=0")
    off = _train_native(eng, data, 1500, batch=128, sparse="early")
    assert on[3].paired_merges > 0 and off[3].paired_merges == 0
    assert on[0] == off[0] and np.array_equal(on[1], off[1])
    assert on[3].tail_dropped == off[3].tail_dropped


def test_paired_random_corpora(eng):
    """Property test over random corpora: a small random alphabet (2-7 letters, so
    same-symbol runs and count ties abound), Zipf-weighted random words, token-0
    bytes in some, both compaction modes and several step sizes — every merge, the
    final stream and every live pair count equal the oracle's, and pairing happens."""
    paired = 0
    for seed in range(8):
        rng = np.random.default_rng(1000 + seed)
        alpha = rng.choice(list(b"abcdefghijklmnop"), size=int(rng.integers(2, 8)), replace=False)
        nv = int(rng.integers(300, 2000))
        vocab = [bytes(rng.choice(alpha, size=int(n)).tolist()) for n in rng.integers(1, 9, size=nv)]
        p = 1.0 / np.arange(1, nv + 1) ** rng.uniform(0.8, 1.3)
        words = rng.choice(nv, size=int(rng.integers(12000, 24000)), p=p / p.sum())
        data = bytearray(b" ".join(vocab[i] for i in words))
        if seed % 3 == 0:   # token 0 never pairs (train.wgsl:395-399)
            for i in rng.integers(0, len(data), len(data) // 200):
                data[i] = 0
        data = bytes(data)
        exact = bool(seed & 1)
        target = 256 + int(rng.integers(300, 1200))
        batch = int(rng.choice([16, 64, 128]))
        ref = O.train(data, target, compaction="exact" if exact else "reference")
        m, s, pairs, st = _train_native(eng, data, target, exact=exact, batch=batch, sparse="early")
        assert m == ref["merges"], f"seed {seed}"
        assert np.array_equal(s, ref["symbols"]), f"seed {seed}"
        _assert_counts_match_stream(pairs, s)
        if not exact:
            assert st.tail_dropped == sum(ref["tail_drops"]), f"seed {seed}"
        paired += st.paired_merges
    assert paired > 0
