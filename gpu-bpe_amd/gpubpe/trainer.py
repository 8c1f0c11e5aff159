"""BPETrainer — the reference's training API (src/bpe/trainer.js:125-371)
over the native HIP merge loop.

``train(input, target_vocab_size=4096, pre_tokenizer=None, word_starts=None,
on_progress=None)`` returns ``{vocab, vocabStrings, vocabSize, merges,
trainingTime}`` like trainer.js:328-334; ``merges`` are ``[a, b, id]``.
The Vocab persists across ``train()`` calls on one instance
(trainer.js:136, 191).  ``pre_tokenizer`` may be any object with a
``pre_tokenize_bytes(bytes) -> {"bytes", "wordStarts"}`` method (the
reference's PreTokenizer.preTokenizeBytes contract, trainer.js:64-80);
``word_starts`` passes a byte mask directly.
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np

from . import _lib
from .vocab import Vocab

BATCH_SIZE = 128


def _fmt_duration(s: float) -> str:
    if s < 60:
        return f"{s:.1f}s"
    m, r = int(s // 60), round(s % 60)
    return f"{m}m {r}s" if r > 0 else f"{m}m"


class BPETrainer:
    def __init__(self, engine, exact_compaction: bool = False, batch_size: int = BATCH_SIZE):
        self._engine = engine
        self._vocab = Vocab()
        self._flags = _lib.GBPE_TRAIN_EXACT_COMPACTION if exact_compaction else 0
        self._batch = batch_size
        self.last_stats = None

    @property
    def vocab(self) -> Vocab:
        return self._vocab

    def train(self, data, target_vocab_size: int = 4096, pre_tokenizer=None, word_starts=None, on_progress=None):
        if isinstance(data, str):
            data = data.encode("utf-8")
        data = bytes(data)
        if pre_tokenizer is not None and word_starts is None:
            r = pre_tokenizer.pre_tokenize_bytes(data)
            if len(r["bytes"]) or not len(data):
                data, word_starts = bytes(r["bytes"]), np.asarray(r["wordStarts"], dtype=np.uint8)
        if len(data) == 0:
            raise ValueError("No symbols to train on — corpus is empty after pre-processing")
        ws = None
        if word_starts is not None:
            ws = np.ascontiguousarray(np.asarray(word_starts, dtype=np.uint8))
            if ws.shape[0] != len(data):
                raise ValueError("word_starts length must equal the byte length")
        lib = _lib.load()
        ctx = self._engine.device
        opts = _lib.TrainOpts(target_vocab_size=target_vocab_size, vocab_size=self._vocab.size,
                              next_token_id=self._vocab.next_token_id, batch_size=self._batch,
                              flags=self._flags, table_log2=0)
        needed = max(0, target_vocab_size - self._vocab.size)
        tr = C.c_void_p()
        buf = C.create_string_buffer(data, len(data))
        wsp = ws.ctypes.data_as(C.c_void_p) if ws is not None else None
        _lib.check(lib.gbpe_trainer_create(ctx, buf, len(data), wsp, 0, C.byref(opts), C.byref(tr)), ctx, "train")
        merges = []
        t0 = time.perf_counter()
        try:
            batch = (C.c_uint32 * (4 * self._batch))()
            done_total, stop = 0, False
            while done_total < needed and not stop:
                nd, es = C.c_uint32(), C.c_uint32()
                _lib.check(lib.gbpe_trainer_step(tr, self._batch, batch, C.byref(nd), C.byref(es)), ctx, "train step")
                for i in range(nd.value):
                    a, b = batch[4 * i], batch[4 * i + 1]
                    nid = self._vocab.add_merge(a, b)          # trainer.js:270-276
                    merges.append([a, b, nid])
                done_total += nd.value
                stop = bool(es.value)
                if on_progress is not None:
                    el = time.perf_counter() - t0
                    st = _lib.TrainerStats()
                    lib.gbpe_trainer_stats_get(tr, C.byref(st))
                    on_progress({
                        "mergeIndex": done_total, "totalMerges": needed,
                        "mergeString": self._vocab.strings[-1] if nd.value else "—",
                        "bestCount": batch[4 * (nd.value - 1) + 3] if nd.value else 0,
                        "symbolCount": int(st.symbol_count),
                        "mergesPerSecond": done_total / el if el > 0 else 0.0,
                    })
                if nd.value == 0 and not stop:
                    break
            st = _lib.TrainerStats()
            lib.gbpe_trainer_stats_get(tr, C.byref(st))
            self.last_stats = {f: getattr(st, f) for f, _ in _lib.TrainerStats._fields_}
        finally:
            lib.gbpe_trainer_destroy(tr)
        total = time.perf_counter() - t0
        return {
            "vocab": self._vocab.entries,
            "vocabStrings": self._vocab.strings,
            "vocabSize": self._vocab.size,
            "merges": merges,
            "trainingTime": _fmt_duration(total),
        }

    def export_vocab(self) -> str:
        return self._vocab.export()
