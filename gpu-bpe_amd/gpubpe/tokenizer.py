"""TrieTokenizer — the reference's encode API (src/bpe/tokenizer/tokenizer.js)
over the native chunked trie walk.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .trie import compile_vocab_to_trie, parse_header, parse_trie_buffers

DEFAULT_CHUNK_SIZE = 512
UTF8_REPLACEMENT = bytes([0xEF, 0xBF, 0xBD])


class TrieTokenizer:
    def __init__(self, engine, trie_data: bytes, vocab=None, chunk_size: int | None = None):
        self._engine = engine
        self._vocab = vocab if vocab is not None else [[i] for i in range(256)]
        hdr = parse_header(trie_data)
        nodes, edges = parse_trie_buffers(trie_data, hdr)
        self.node_count = hdr["nodeCount"]
        self.edge_count = hdr["edgeCount"]
        self.max_token_len = hdr["maxTokenLen"]
        adaptive = max(DEFAULT_CHUNK_SIZE, min(2048, hdr["maxTokenLen"] * 8))   # tokenizer.js:67-68
        self.chunk_size = chunk_size if chunk_size is not None else adaptive
        if self.chunk_size <= 0:
            raise ValueError("chunk_size must be positive")
        lib = _lib.load()
        ctx = engine.device
        self._trie = C.c_void_p()
        nodes = np.ascontiguousarray(nodes, dtype=np.uint32)
        edges = np.ascontiguousarray(edges, dtype=np.uint32)
        _lib.check(lib.gbpe_trie_upload(ctx, nodes.ctypes.data_as(_lib.u32p), self.node_count,
                                        edges.ctypes.data_as(_lib.u32p), self.edge_count, C.byref(self._trie)),
                   ctx, "trie upload")

    @classmethod
    def from_vocab(cls, engine, vocab, chunk_size: int | None = None) -> "TrieTokenizer":
        return cls(engine, compile_vocab_to_trie(vocab), vocab, chunk_size)

    def encode_bytes(self, data) -> np.ndarray:
        data = bytes(data)
        n = len(data)
        if n == 0:
            return np.zeros(0, dtype=np.uint32)
        lib = _lib.load()
        ctx = self._engine.device
        out = np.empty(n, dtype=np.uint32)      # at most one token per byte
        n_out = C.c_uint64()
        buf = C.create_string_buffer(data, n)
        _lib.check(lib.gbpe_encode(ctx, self._trie, buf, n, self.chunk_size, out.ctypes.data_as(_lib.u32p), n,
                                   C.byref(n_out)), ctx, "encode")
        return out[: n_out.value].copy()

    def decode(self, tokens) -> bytes:
        out = bytearray()
        for t in tokens:
            t = int(t)
            out.extend(self._vocab[t] if t < len(self._vocab) else UTF8_REPLACEMENT)
        return bytes(out)

    def destroy(self):
        if getattr(self, "_trie", None):
            _lib.load().gbpe_trie_free(self._trie)
            self._trie = None
