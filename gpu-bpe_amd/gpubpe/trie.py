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
from collections import deque

import numpy as np

TRIE_MAGIC = 0x54524945
TRIE_VERSION = 3
HEADER_SIZE = 28
INVALID_TOKEN = 0xFFFFFFFF


class _Node:
    __slots__ = ("kids", "tid")

    def __init__(self):
        self.kids = {}
        self.tid = INVALID_TOKEN


def compile_vocab_to_trie(vocab) -> bytes:
    root = _Node()
    max_len = 0
    for tid, seq in enumerate(vocab):
        if not seq:
            continue
        node = root
        for byte in seq:
            nxt = node.kids.get(byte)
            if nxt is None:
                nxt = node.kids[byte] = _Node()
            node = nxt
        node.tid = tid
        max_len = max(max_len, len(seq))
    nodes = []          # (firstChild, numChildren, tokenId) in BFS order
    edges = []          # (symbol, target)
    order = deque([root])
    next_index = 1
    while order:
        node = order.popleft()
        first = len(edges)
        for sym in sorted(node.kids):
            edges.append((sym, next_index))
            next_index += 1
            order.append(node.kids[sym])
        nodes.append((first, len(node.kids), node.tid))
    head = struct.pack("<7I", TRIE_MAGIC, TRIE_VERSION, len(nodes), len(edges), max_len, len(vocab), 0)
    nb = np.asarray(nodes, dtype="<u4").reshape(-1, 3).tobytes()
    eb = np.zeros((len(edges), 2), dtype="<u4")
    if edges:
        eb[:] = np.asarray(edges, dtype="<u4")
    return head + nb + eb.tobytes()


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
