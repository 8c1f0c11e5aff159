"""Checkpoint / resume through the C-ABI (gbpe_trainer_export_state →
gbpe_trainer_create_from_state, gpubpe/checkpoint.py): one trainer runs `split`
merges and exports its (current, previous) streams; a second trainer created
from that state finishes the run.  Merges and the final stream equal the
oracle's uninterrupted run (oracle/bpe_oracle.py, snapshot semantics of
train.wgsl:433-520 with the compaction quirk of train.wgsl:605-607 + 698/727)."""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "gpu-bpe_amd"))

import bpe_oracle as O  # noqa: E402
from gpubpe import synth  # noqa: E402

pytestmark = pytest.mark.gpu

RESUME = [("ref", False, 300), ("exact", True, 300), ("ref_first", False, 0), ("ref_late", False, 1100)]


@pytest.mark.parametrize("name,exact,split", RESUME, ids=[r[0] for r in RESUME])
def test_gpu_export_state_resume(name, exact, split):
    from gpubpe import _lib
    from gpubpe.checkpoint import ResumedTrainer, export_state
    lib = _lib.load()
    ctx = C.c_void_p()
    _lib.check(lib.gbpe_ctx_create(0, C.byref(ctx)), ctx, "ctx")
    data = synth.english(400_000, seed=31)
    vocab = 1800
    exp = O.train(data, vocab, compaction="exact" if exact else "reference")
    try:
        opts = _lib.TrainOpts(target_vocab_size=vocab, vocab_size=256, next_token_id=256, batch_size=128,
                              flags=_lib.GBPE_TRAIN_EXACT_COMPACTION if exact else 0, table_log2=0)
        t = C.c_void_p()
        buf = C.create_string_buffer(data, len(data))
        _lib.check(lib.gbpe_trainer_create(ctx, buf, len(data), None, 0, C.byref(opts), C.byref(t)), ctx, "create")
        got = []
        out = (C.c_uint32 * 512)()
        while len(got) < split:
            nd, es = C.c_uint32(), C.c_uint32()
            _lib.check(lib.gbpe_trainer_step(t, min(128, split - len(got)), out, C.byref(nd), C.byref(es)), ctx, "step")
            got += [list(out[4 * i: 4 * i + 4]) for i in range(nd.value)]
        cur, prev = export_state(lib, ctx, t)
        lib.gbpe_trainer_destroy(t)
        assert cur.shape[0] == exp["n_history"][split]
        assert prev.shape[0] == (exp["n_history"][split - 1] if split else cur.shape[0])
        single = ResumedTrainer(lib, ctx, cur, prev, vocab, 256 + split, exact=exact)
        while len(got) < len(exp["merges"]):
            m, early = single.step(128)
            got += m
            if early or not m:
                break
        assert got == exp["merges"]
        np.testing.assert_array_equal(single.symbols(), exp["symbols"])
        single.close()
    finally:
        lib.gbpe_ctx_destroy(ctx)
