"""Word-lexicon build on the GPU: the word table sized from a sample of the
distinct words, and its rebuild at full size when the sample misleads.

The corpus opens with 4.3M copies of one word (so the 4M-word sample sees one
distinct word and sizes the table for a few), then 20M words drawn from a pool
of 2M: the estimated table overflows, the build reruns at full size, and the
lexicon run must give the same merges as the run without a lexicon
(in-place sectors), which the full-length fixture tests pin against the oracle.
"""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from gpubpe import BPEEngine
    return BPEEngine(0).init()


def _train(eng, d, n, merges, env):
    from gpubpe import _lib
    lib = _lib.load()
    ctx = eng.device
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)   # read at trainer creation (GBPE_DEBUG lex_check at every build)
    tr = C.c_void_p()
    try:
        opts = _lib.TrainOpts(target_vocab_size=256 + merges, vocab_size=256, next_token_id=256, batch_size=128,
                              flags=0, table_log2=0)
        _lib.check(lib.gbpe_trainer_create(ctx, d, n, None, 1, C.byref(opts), C.byref(tr)), ctx, "create")
        out, got = (C.c_uint32 * 512)(), []
        while True:
            nd, es = C.c_uint32(), C.c_uint32()
            _lib.check(lib.gbpe_trainer_step(tr, 128, out, C.byref(nd), C.byref(es)), ctx, "step")
            got += [tuple(out[4 * i:4 * i + 4]) for i in range(nd.value)]
            if nd.value == 0 or es.value:
                break
        st = _lib.TrainerStats()
        lib.gbpe_trainer_stats_get(tr, C.byref(st))
    finally:
        if tr.value:
            lib.gbpe_trainer_destroy(tr)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return got, st


def test_word_table_estimate_short(eng):
    from gpubpe import _lib
    lib = _lib.load()
    ctx = eng.device
    rng = np.random.default_rng(5)
    pool = rng.integers(97, 123, size=(2_000_000, 7), dtype=np.uint8)
    words = np.empty((20_000_000, 8), np.uint8)
    words[:, 0] = 32
    words[:, 1:] = pool[rng.integers(0, pool.shape[0], size=words.shape[0])]
    data = b" a" * 4_300_000 + words.tobytes()
    n = len(data)
    d = C.c_void_p()
    _lib.check(lib.gbpe_device_alloc(ctx, n + 64, C.byref(d)), ctx, "alloc")
    try:
        _lib.check(lib.gbpe_memcpy_h2d(ctx, d, data, n), ctx, "h2d")
        lex, st = _train(eng, d, n, 300, {"GBPE_DEBUG": "lexicon=1,lex_check=1"})
        ref, _ = _train(eng, d, n, 300, {"GBPE_DEBUG": "lexicon=0"})
    finally:
        lib.gbpe_device_free(ctx, d)
    assert st.lexicon_builds >= 1 and st.lexicon_fallbacks == 0
    assert st.lexicon_entries > (1 << 20)   # more distinct words than the estimated table held
    assert len(lex) == 300 and lex == ref
