"""MergeEncoder — TokenizerManager.encode (src/bpe/tokenizer/tokenizer-manager.js:13-61)
on the device: the learned merges applied in rank order to the whole byte
string, through gbpe_bpe_upload / gbpe_bpe_encode."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib


class MergeEncoder:
    def __init__(self, engine, merges):
        self._engine = engine
        self._merges = [list(m[:3]) for m in merges]
        lib = _lib.load()
        arr = np.ascontiguousarray(np.asarray(self._merges, dtype=np.uint32).reshape(-1, 3))
        h = C.c_void_p()
        _lib.check(lib.gbpe_bpe_upload(engine.device, arr.ctypes.data_as(_lib.u32p), arr.shape[0], C.byref(h)),
                   engine.device, "bpe upload")
        self._h = h

    def encode_bytes(self, data) -> np.ndarray:
        data = bytes(data)
        lib = _lib.load()
        ctx = self._engine.device
        out = np.empty(max(1, len(data)), dtype=np.uint32)
        n = C.c_uint64()
        buf = C.create_string_buffer(data, len(data)) if data else None
        _lib.check(lib.gbpe_bpe_encode(ctx, self._h, buf, len(data), out.ctypes.data_as(_lib.u32p), out.shape[0],
                                       C.byref(n)), ctx, "bpe encode")
        return out[: n.value].copy()

    def encode(self, text) -> dict:
        """{tokens, text} like TokenizerManager.encode's result (tokenizer-manager.js:60)."""
        data = text.encode("utf-8") if isinstance(text, str) else bytes(text)
        return {"tokens": self.encode_bytes(data).tolist(), "text": text}

    def destroy(self):
        if self._h:
            _lib.load().gbpe_bpe_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:  # noqa: BLE001
            pass
