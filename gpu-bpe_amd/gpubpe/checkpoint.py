"""Checkpoint / resume of a training run through the C-ABI.

The reference keeps no mid-training checkpoint (only the final model
JSON, training-manager.js:173-224).  A trainer's state is its current stream and
its previous stream — the ping-pong buffer the compaction quirk reads stale
symbols from (train.wgsl:605-607 + 698/727) — both in the reference u32 layout
(bit 16 = word start): gbpe_trainer_export_state writes them, and
gbpe_trainer_create_from_state continues a run from them bit-exactly
(tests/test_gpu_resume.py)."""
from __future__ import annotations

import ctypes as C

import numpy as np

BATCH_SIZE = 128


def state_lens(lib, ctx, t):
    """(current, previous) stream lengths of a trainer (gbpe_trainer_export_state, no copy)."""
    from . import _lib
    n, npv = C.c_uint64(), C.c_uint64()
    _lib.check(lib.gbpe_trainer_export_state(t, None, 0, C.byref(n), None, 0, C.byref(npv), 0), ctx, "export_state")
    return int(n.value), int(npv.value)


def export_state(lib, ctx, t):
    """(current, previous) stream of a trainer as host u32 arrays."""
    from . import _lib
    n, npv = state_lens(lib, ctx, t)
    cur = np.zeros(max(1, n), np.uint32)
    prev = np.zeros(max(1, npv), np.uint32)
    a, b = C.c_uint64(), C.c_uint64()
    _lib.check(lib.gbpe_trainer_export_state(t, cur.ctypes.data_as(C.c_void_p), n, C.byref(a),
                                             prev.ctypes.data_as(C.c_void_p), npv, C.byref(b), 0),
               ctx, "export_state")
    return cur[:n], prev[:npv]


def export_state_device(lib, ctx, t, cur_ptr: int, prev_ptr: int, cap_cur: int, cap_prev: int):
    """The same into device buffers (HBM to HBM)."""
    from . import _lib
    a, b = C.c_uint64(), C.c_uint64()
    _lib.check(lib.gbpe_trainer_export_state(t, C.c_void_p(cur_ptr), cap_cur, C.byref(a), C.c_void_p(prev_ptr),
                                             cap_prev, C.byref(b), 1), ctx, "export_state")
    return int(a.value), int(b.value)


class ResumedTrainer:
    """A trainer continuing from an exported (current, previous) stream pair
    (gbpe_trainer_create_from_state) with the single-GPU policy."""

    def __init__(self, lib, ctx, cur, prev, target_vocab: int, next_id: int, exact: bool = False, flags: int = 0,
                 table_log2: int = 0, batch: int = BATCH_SIZE):
        from . import _lib
        self.lib, self.ctx, self._lib = lib, ctx, _lib
        flags |= _lib.GBPE_TRAIN_EXACT_COMPACTION if exact else 0
        self.opts = _lib.TrainOpts(target_vocab_size=target_vocab, vocab_size=next_id, next_token_id=next_id,
                                   batch_size=batch, flags=flags, table_log2=table_log2)
        t = C.c_void_p()
        if hasattr(cur, "data_ptr"):   # torch tensors (int32 / uint32 view) already in HBM
            cur, prev = cur.contiguous(), prev.contiguous()
            assert cur.is_cuda and prev.is_cuda and cur.element_size() == 4 and prev.element_size() == 4
            args = (C.c_void_p(cur.data_ptr()), cur.numel(), C.c_void_p(prev.data_ptr()), prev.numel(), 1)
        else:
            cur = np.ascontiguousarray(cur, dtype=np.uint32)
            prev = np.ascontiguousarray(prev, dtype=np.uint32)
            args = (cur.ctypes.data_as(C.c_void_p), cur.shape[0], prev.ctypes.data_as(C.c_void_p), prev.shape[0], 0)
        _lib.check(lib.gbpe_trainer_create_from_state(ctx, *args, C.byref(self.opts), C.byref(t)), ctx,
                   "create_from_state")
        self.t = t
        self.batch = batch
        self._out = (C.c_uint32 * (4 * batch))()

    def step(self, max_merges):
        nd, es = C.c_uint32(), C.c_uint32()
        self._lib.check(self.lib.gbpe_trainer_step(self.t, min(max_merges, self.batch), self._out, C.byref(nd),
                                                   C.byref(es)), self.ctx, "single step")
        return [list(self._out[4 * i: 4 * i + 4]) for i in range(nd.value)], bool(es.value)

    def symbols(self):
        n = C.c_uint64()
        self._lib.check(self.lib.gbpe_trainer_symbols(self.t, None, 0, C.byref(n)), self.ctx, "symbols")
        out = np.zeros(max(1, n.value), np.uint32)
        self._lib.check(self.lib.gbpe_trainer_symbols(self.t, out.ctypes.data_as(C.POINTER(C.c_uint32)), n.value,
                                                      C.byref(n)), self.ctx, "symbols")
        return out[: n.value]

    def stats(self):
        st = self._lib.TrainerStats()
        self.lib.gbpe_trainer_stats_get(self.t, C.byref(st))
        return st

    def close(self):
        if self.t:
            self.lib.gbpe_trainer_destroy(self.t)
            self.t = None
