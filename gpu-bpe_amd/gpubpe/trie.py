"""Trie compile / parse — behaviour of the reference src/bpe/tokenizer/trie.js.

Binary format v3 (trie.js:10-13, 167-206): 28-byte header
[magic 'TRIE', version, nodeCount, edgeCount, maxTokenLen, vocabSize, flags],
12-byte nodes {firstChild, numChildren, tokenId}, 8-byte edges
{symbol u8 + 3 pad, targetNode}.  BFS node order, children sorted by byte,
a later duplicate byte string overwrites the token id (trie.js:44-57).
v2 (8-byte nodes, 4-byte edges) is accepted on parse (trie.js:140-141).
"""
from __future__ import annotations

import struct

import numpy as np

TRIE_MAGIC = 0x54524945
TRIE_VERSION = 3
HEADER_SIZE = 28
INVALID_TOKEN = 0xFFFFFFFF


def compile_vocab_to_trie(vocab) -> bytes:
    """compileVocabToTrie (trie.js:39-98) through the library's native compiler
    (gbpe_trie_compile): vocab[i] = byte list of token id i."""
    import ctypes as C

    from . import _lib
    lib = _lib.load()
    lens = np.fromiter((len(v) if v else 0 for v in vocab), dtype=np.uint64, count=len(vocab))
    offs = np.zeros(len(vocab) + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    flat = np.fromiter((b for v in vocab if v for b in v), dtype=np.uint8, count=int(offs[-1]))
    need = C.c_uint64()
    _lib.check(lib.gbpe_trie_compile(flat.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(_lib.u64p), len(vocab),
                                     None, 0, C.byref(need)), None, "trie compile")
    out = (C.c_uint8 * need.value)()
    _lib.check(lib.gbpe_trie_compile(flat.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(_lib.u64p), len(vocab),
                                     out, need.value, C.byref(need)), None, "trie compile")
    return bytes(out)


def parse_header(data: bytes) -> dict:
    if len(data) < HEADER_SIZE:
        raise ValueError("Truncated trie data")
    magic, version, nc, ec, mtl = struct.unpack_from("<5I", data, 0)
    if magic != TRIE_MAGIC:
        raise ValueError("Invalid trie magic: 0x%x" % magic)
    if version not in (2, 3):
        raise ValueError("Unsupported trie version: %d" % version)
    return {"version": version, "nodeCount": nc, "edgeCount": ec, "maxTokenLen": mtl}


def parse_trie_buffers(data: bytes, header: dict):
    """→ (nodes uint32[3*N], edges uint32[2*E]) exactly as trie.js:209-249."""
    v, nc, ec = header["version"], header["nodeCount"], header["edgeCount"]
    per_node, per_edge = (12, 8) if v == 3 else (8, 4)
    if len(data) < HEADER_SIZE + nc * per_node + ec * per_edge:
        raise ValueError("Truncated trie data")
    o = HEADER_SIZE
    if v == 3:
        nodes = np.frombuffer(data, dtype="<u4", count=3 * nc, offset=o).astype(np.uint32)
        e = np.frombuffer(data, dtype="<u4", count=2 * ec, offset=o + 12 * nc).reshape(-1, 2)
        edges = np.stack([e[:, 0] & 0xFF, e[:, 1]], axis=1).astype(np.uint32).reshape(-1)
    else:
        raw = np.frombuffer(data, dtype="<u2", count=4 * nc, offset=o).reshape(-1, 4).astype(np.uint32)
        tid = np.where(raw[:, 2] == 0xFFFF, INVALID_TOKEN, raw[:, 2]).astype(np.uint32)
        nodes = np.stack([raw[:, 0], raw[:, 1], tid], axis=1).astype(np.uint32).reshape(-1)
        e = np.frombuffer(data, dtype="<u2", count=2 * ec, offset=o + 8 * nc).reshape(-1, 2).astype(np.uint32)
        edges = np.stack([e[:, 0] & 0xFF, e[:, 1]], axis=1).astype(np.uint32).reshape(-1)
    return np.ascontiguousarray(nodes), np.ascontiguousarray(edges)
