"""ctypes wrapper of oracle/bpe_oracle.c — TEST / BENCH INFRASTRUCTURE ONLY.

The C restatement of the reference algorithm (full recount every merge,
snapshot merge, reference compaction) for inputs too large for the numpy
oracle, and the `cpu_baseline` leg of bench.py.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "lib", "libbpe_oracle.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", HERE], check=True, capture_output=True)
        _lib = C.CDLL(LIB)
        _lib.oracle_train.restype = C.c_int
        _lib.oracle_train.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                      C.c_uint32, C.c_int, C.c_void_p, C.POINTER(C.c_uint32),
                                      C.POINTER(C.c_uint32), C.c_void_p, C.POINTER(C.c_uint64),
                                      C.POINTER(C.c_uint64)]
        _lib.oracle_encode.restype = C.c_uint64
        _lib.oracle_encode.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_int,
                                       C.c_void_p]
        _lib.oracle_max_threads.restype = C.c_int
        _lib.oracle_train_inc.restype = C.c_int
        _lib.oracle_train_inc.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                          C.c_int, C.c_uint32, C.c_void_p, C.POINTER(C.c_uint32),
                                          C.POINTER(C.c_uint32), C.c_void_p, C.POINTER(C.c_uint64),
                                          C.POINTER(C.c_uint64)]
        _lib.oracle_gpt4_ws_ascii.restype = C.c_int
        _lib.oracle_gpt4_ws_ascii.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
    return _lib


def max_threads() -> int:
    return load().oracle_max_threads()


def train(data: bytes, target: int, word_starts=None, next_token_id: int = 256, vocab_size: int | None = None,
          exact: bool = False, max_merges: int = 0, threads: int = 0, want_symbols: bool = True):
    lib = load()
    n = len(data)
    if n == 0:
        raise ValueError("No symbols to train on — corpus is empty after pre-processing")
    vs = next_token_id if vocab_size is None else vocab_size
    needed = max(0, target - vs)
    if max_merges:
        needed = min(needed, max_merges)
    merges = np.zeros(4 * max(needed, 1), np.uint32)
    syms = np.zeros(n, np.uint32) if want_symbols else None
    nm, es, fn, tail = C.c_uint32(), C.c_uint32(), C.c_uint64(), C.c_uint64()
    buf = np.frombuffer(data, np.uint8)
    ws = None if word_starts is None else np.ascontiguousarray(word_starts, dtype=np.uint8)
    rc = lib.oracle_train(buf.ctypes.data, n, ws.ctypes.data if ws is not None else None, target, vs, next_token_id,
                          1 if exact else 0, max_merges, threads, merges.ctypes.data, C.byref(nm), C.byref(es),
                          syms.ctypes.data if syms is not None else None, C.byref(fn), C.byref(tail))
    if rc != 0:
        raise RuntimeError(f"oracle_train failed ({rc})")
    return {"merges": merges[:4 * nm.value].reshape(-1, 4).tolist(),
            "symbols": syms[:fn.value] if syms is not None else None,
            "early_stop": bool(es.value), "tail_total": int(tail.value), "final_n": int(fn.value)}


def train_inc(data: bytes, target: int, word_starts=None, next_token_id: int = 256, vocab_size: int | None = None,
              exact: bool = False, max_merges: int = 0, want_symbols: bool = True):
    """Same contract as train(): the incremental restatement (bpe_oracle_inc.c,
    linked-list stream + occurrence lists + lazy heap), for full-length runs on
    corpora where the full recount would take hours.  Checked against train()
    by tests/test_oracle_inc.py."""
    lib = load()
    n = len(data)
    if n == 0:
        raise ValueError("No symbols to train on — corpus is empty after pre-processing")
    vs = next_token_id if vocab_size is None else vocab_size
    needed = max(0, target - vs)
    if max_merges:
        needed = min(needed, max_merges)
    merges = np.zeros(4 * max(needed, 1), np.uint32)
    syms = np.zeros(n, np.uint32) if want_symbols else None
    nm, es, fn, tail = C.c_uint32(), C.c_uint32(), C.c_uint64(), C.c_uint64()
    buf = np.frombuffer(data, np.uint8)
    ws = None if word_starts is None else np.ascontiguousarray(word_starts, dtype=np.uint8)
    rc = lib.oracle_train_inc(buf.ctypes.data, n, ws.ctypes.data if ws is not None else None, target, vs,
                              next_token_id, 1 if exact else 0, max_merges, merges.ctypes.data, C.byref(nm),
                              C.byref(es), syms.ctypes.data if syms is not None else None, C.byref(fn),
                              C.byref(tail))
    if rc != 0:
        raise RuntimeError(f"oracle_train_inc failed ({rc})")
    return {"merges": merges[:4 * nm.value].reshape(-1, 4).tolist(),
            "symbols": syms[:fn.value] if syms is not None else None,
            "early_stop": bool(es.value), "tail_total": int(tail.value), "final_n": int(fn.value)}


def gpt4_word_starts_ascii(data: bytes) -> np.ndarray:
    """GPT-4 rule word starts (bpe_oracle.gpt4_word_starts) for ASCII-only
    input, in C; the 128 classes come from bpe_oracle.pt_classify."""
    import bpe_oracle as O
    lib = load()
    cls = np.array([O.pt_classify(c) for c in range(128)], dtype=np.uint8)
    buf = np.frombuffer(data, np.uint8)
    out = np.zeros(len(data), np.uint8)
    if lib.oracle_gpt4_ws_ascii(buf.ctypes.data, len(data), cls.ctypes.data, out.ctypes.data) != 0:
        raise ValueError("gpt4_word_starts_ascii: non-ASCII input")
    return out


def encode(data: bytes, nodes: np.ndarray, edges: np.ndarray, chunk: int, threads: int = 0, count_only=False):
    lib = load()
    buf = np.frombuffer(data, np.uint8)
    nodes = np.ascontiguousarray(nodes, np.uint32)
    edges = np.ascontiguousarray(edges, np.uint32)
    if count_only:
        return int(lib.oracle_encode(buf.ctypes.data, len(data), nodes.ctypes.data, nodes.shape[0] // 3,
                                     edges.ctypes.data, chunk, threads, None))
    out = np.zeros(max(1, len(data)), np.uint32)
    k = lib.oracle_encode(buf.ctypes.data, len(data), nodes.ctypes.data, nodes.shape[0] // 3, edges.ctypes.data, chunk,
                          threads, out.ctypes.data)
    return out[:k]
