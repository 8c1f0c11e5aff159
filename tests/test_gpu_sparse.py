"""GPU parity of the sector-sparse merge loop against the CPU oracle.

The sparse loop re-lays the stream out as word-aligned sectors plus a dense
zone that carries the reference's compaction quirk (train.wgsl:605-607 + 698/727).
These cases force it on early (GBPE_TRAIN_SPARSE_EARLY, small batches so the
layout changes at many step boundaries) and check bit-exact merges
[a, b, id, count], final streams and live pair counts in both compaction modes.
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


@pytest.mark.parametrize("kind,size,target,batch", [("english", 65536, 1024, 16), ("multilingual", 65536, 700, 5),
                                                    ("code", 65536, 900, 32), ("english", 300000, 2048, 128)])
@pytest.mark.parametrize("exact", [False, True])
def test_sparse_matches_oracle(eng, kind, size, target, batch, exact):
    from gpubpe import synth
    data = getattr(synth, kind)(size, seed=size % 97 + 3)
    ref = O.train(data, target, compaction="exact" if exact else "reference")
    m, s, pairs, st = _train_native(eng, data, target, exact=exact, batch=batch, sparse="early")
    assert st.sparse_enters >= 1 and st.sparse_merges > 0
    assert m == ref["merges"]
    assert np.array_equal(s, ref["symbols"])
    _assert_counts_match_stream(pairs, s)
    if not exact:
        assert st.tail_dropped == sum(ref["tail_drops"])


def test_sparse_u32_and_external_word_starts(eng):
    from gpubpe import synth
    data = synth.english(40000, seed=21)
    ref = O.train(data, 40000)
    m, s, pairs, st = _train_native(eng, data, 40000, batch=64, sparse="early")
    assert st.bytes_per_symbol == 4 and st.sparse_merges > 0
    assert m == ref["merges"] and np.array_equal(s, ref["symbols"])
    _assert_counts_match_stream(pairs, s)
    code = synth.code(60000, seed=9)
    ws = (np.random.default_rng(3).random(len(code)) < 0.2).astype(np.uint8)
    ws[0] = 1
    for exact in (False, True):
        ref = O.train(code, 800, word_starts=ws, compaction="exact" if exact else "reference")
        m, s, pairs, st = _train_native(eng, code, 800, word_starts=ws, exact=exact, batch=8, sparse="early")
        assert st.sparse_merges > 0
        assert m == ref["merges"] and np.array_equal(s, ref["symbols"])
        _assert_counts_match_stream(pairs, s)


def test_sparse_zone_aborts_and_reentry(eng, monkeypatch):
    # the smallest zone the invariant allows (5 mc): merges outgrow it, the loop
    # returns to dense mid-step and re-enters later; results must not change
    from gpubpe import synth
    monkeypatch.setenv("GBPE_DEBUG", "zt=5")
    data = synth.multilingual(120000, seed=13)
    ref = O.train(data, 1500)
    m, s, pairs, st = _train_native(eng, data, 1500, batch=16, sparse="early", table_log2=15)
    assert st.sparse_merges > 0 and st.sparse_exits >= 1
    assert m == ref["merges"] and np.array_equal(s, ref["symbols"])
    _assert_counts_match_stream(pairs, s)


def test_sparse_runs_and_random_bytes(eng):
    rng = np.random.default_rng(29)
    for trial in range(6):
        alphabet = rng.choice(256, size=rng.integers(2, 6), replace=False).astype(np.uint8)
        n = int(rng.integers(2000, 20000))
        data = bytes(rng.choice(alphabet, size=n))
        for exact in (False, True):
            ref = O.train(data, 400, compaction="exact" if exact else "reference")
            m, s, pairs, _ = _train_native(eng, data, 400, exact=exact, batch=4, sparse="early")
            assert m == ref["merges"], (trial, exact)
            assert np.array_equal(s, ref["symbols"]), (trial, exact)
            _assert_counts_match_stream(pairs, s)


@pytest.mark.parametrize("exact", [False, True])
def test_sparse_default_policy_large_vs_c_oracle(eng, exact):
    # 24 MiB with the library's own policy: dense first, sector-sparse once the
    # counts fall; checked against the C restatement
    import cpu_ref
    from gpubpe import synth
    data = synth.english(24 << 20, seed=77, fancy_punct=0.005)
    k = 1200
    ref = cpu_ref.train(data, 256 + k, exact=exact, threads=16)
    m, s, pairs, st = _train_native(eng, data, 256 + k, exact=exact)
    assert st.sparse_merges > 0
    assert m == ref["merges"]
    assert np.array_equal(s, ref["symbols"])
    _assert_counts_match_stream(pairs, s)
    if not exact:
        assert st.tail_dropped == ref["tail_total"]


def test_sparse_vs_dense_full_c2(eng):
    # BASELINE C2 at full size, the bench's own corpus (100 MiB English, seed 2,
    # 0.5 % 3-byte punctuation; all 32,512 merges to a 32K vocab): the library's
    # policy (dense, then sector-sparse) and the dense loop alone must each equal
    # the committed oracle fixture (tests/golden/train_c2.npz, every merge), and
    # agree with each other on the final stream and every live pair count
    import gen_golden_train as G
    want, meta = G.load_train("c2")
    data = G.corpus(meta["corpus"])
    m1, s1, p1, st1 = _train_native(eng, data, 32768)
    m2, s2, p2, st2 = _train_native(eng, data, 32768, sparse="dense")
    assert st1.sparse_merges > 30000 and st2.sparse_merges == 0
    assert m1 == want.tolist()
    assert m2 == want.tolist()
    assert s1.shape[0] == meta["final_n"]
    assert np.array_equal(s1, s2)
    assert np.array_equal(p1[0], p2[0]) and np.array_equal(p1[1], p2[1])
    _assert_counts_match_stream(p1, s1)
    assert st1.tail_dropped == st2.tail_dropped == meta["tail_total"]


@pytest.mark.parametrize("table_log2", [14, 15, 18, 20])
def test_sparse_wide_refresh_workgroups(eng, monkeypatch, table_log2):
    # late k_refresh grids take up to 256 table blocks per workgroup (TPB: C5's
    # 2^25 slots give 512 partial maxima per selection instead of 2,048); rfl=1
    # with a late threshold above every zone forces the widest form from the first
    # step: the grid is ceil(blocks / 256), so 2^18 slots (1,024 blocks) -> 4
    # workgroups of 256, 2^20 -> 16 x 256; 2^14 (64 blocks) is the narrow form's
    # largest workgroup and 2^15 (128 blocks, one workgroup) the wide form's
    # smallest (the boundary at 64 vs 65+ blocks per workgroup)
    from gpubpe import synth
    monkeypatch.setenv("GBPE_DEBUG", "rfl=1,rflz=100000000")
    data = synth.english(300000, seed=41)
    ref = O.train(data, 2048)
    m, s, pairs, st = _train_native(eng, data, 2048, batch=32, sparse="early", table_log2=table_log2)
    assert st.sparse_merges > 0
    assert m == ref["merges"] and np.array_equal(s, ref["symbols"])
    _assert_counts_match_stream(pairs, s)
