"""GpuPreTokenizer — the reference's PreTokenizer (src/wasm/pre_tokenizer.mjs:402-509)
on the device.

``pre_tokenize_bytes(bytes)`` / ``pre_tokenize(text)`` return
``{"bytes": ..., "wordStarts": ...}`` like preTokenizeBytes / preTokenize; the
word starts come from gbpe_pretokenize_gpt4 (GPT-4 rules, findWordBoundaries
:226-292).  Input must already be NFC (the reference normalises first; NFC
text is unchanged by that step).  ``BPETrainer.train(pre_tokenizer=...)``
accepts it like the reference trainer accepts its PreTokenizer (trainer.js:62-99).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib


class GpuPreTokenizer:
    def __init__(self, engine):
        self._engine = engine

    def pre_tokenize_bytes(self, raw) -> dict:
        data = bytes(raw)
        ws = np.zeros(len(data), dtype=np.uint8)
        if data:
            lib = _lib.load()
            ctx = self._engine.device
            buf = C.create_string_buffer(data, len(data))
            _lib.check(lib.gbpe_pretokenize_gpt4(ctx, buf, len(data), ws.ctypes.data_as(C.c_void_p)), ctx,
                       "pretokenize")
        return {"bytes": data, "wordStarts": ws}

    def pre_tokenize(self, text: str) -> dict:
        return self.pre_tokenize_bytes(text.encode("utf-8"))

    # reference spelling
    preTokenizeBytes = pre_tokenize_bytes
    preTokenize = pre_tokenize
