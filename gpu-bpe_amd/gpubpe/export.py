"""Model JSON and DXFT export — the reference's training-manager.js:173-224
(downloadModel / loadFromJSON) and export-controller.js:191-248 (.bin v2).

* ``model_json(model)``: ``{"version": 1, "vocabSize", "vocab", "merges"}`` as
  compact JSON, byte-identical to JSON.stringify of the same object.
* ``load_model_json(data)``: validates and rebuilds ``vocabStrings`` with a
  non-fatal UTF-8 decode (TextDecoder('utf-8', {fatal: false})).
* ``dxft_bin(tokens, vocab_size, vocab_export)``: u32 [0x44584654 'DXFT',
  vocabSize, tokenCount, jsonLen] + tokens + JSON bytes (gbpe_dxft_pack).
* ``export_dxft(tokenizer, files, vocab_export)``: the export pipeline — files
  joined with "\\n\\n", GPU trie encode, pack.
"""
from __future__ import annotations

import ctypes as C
import json

import numpy as np

from . import _lib


def model_json(model: dict) -> str:
    data = {"version": 1, "vocabSize": model["vocabSize"], "vocab": model["vocab"],
            "merges": [list(m[:3]) for m in model["merges"]]}
    return json.dumps(data, separators=(",", ":"))


def load_model_json(data) -> dict:
    obj = json.loads(data) if isinstance(data, (str, bytes, bytearray)) else data
    if not obj.get("vocab") or "merges" not in obj or obj.get("merges") is None:
        raise ValueError("Invalid vocabulary file: missing vocab or merges")
    vocab = obj["vocab"]
    strings = [bytes(b).decode("utf-8", errors="replace") if b else "" for b in vocab]
    return {"vocab": vocab, "vocabStrings": strings, "vocabSize": len(vocab), "merges": obj["merges"]}


def dxft_bin(tokens, vocab_size: int, vocab_export) -> bytes:
    toks = np.ascontiguousarray(np.asarray(tokens, dtype=np.uint32))
    js = b"" if vocab_export is None else (
        vocab_export.encode() if isinstance(vocab_export, str) else json.dumps(vocab_export, separators=(",", ":")).encode())
    lib = _lib.load()
    need = C.c_uint64()
    jb = C.create_string_buffer(js, len(js)) if js else None
    _lib.check(lib.gbpe_dxft_pack(toks.ctypes.data_as(C.c_void_p), toks.shape[0], vocab_size, jb, len(js), None, 0,
                                  C.byref(need)), None, "dxft")
    out = (C.c_uint8 * need.value)()
    _lib.check(lib.gbpe_dxft_pack(toks.ctypes.data_as(C.c_void_p), toks.shape[0], vocab_size, jb, len(js), out,
                                  need.value, C.byref(need)), None, "dxft")
    return bytes(out)


def export_dxft(tokenizer, files, vocab_export=None, model=None) -> bytes:
    """export-controller.js:191-248: join files with "\\n\\n", encode on the GPU, pack."""
    merged = b"\n\n".join(bytes(f) for f in files)
    tokens = tokenizer.encode_bytes(merged)
    if vocab_export is None and model is not None:
        vocab_export = {"version": 1, "vocabSize": model["vocabSize"], "vocab": model["vocab"],
                        "merges": [list(m[:3]) for m in model["merges"]]}
    if vocab_export is not None and isinstance(vocab_export, dict) and vocab_export.get("vocab") is not None:
        vocab_size = len(vocab_export["vocab"])
    elif model is not None:
        vocab_size = model["vocabSize"]
    else:
        vocab_size = 256
    return dxft_bin(tokens, vocab_size, vocab_export)
