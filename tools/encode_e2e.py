#!/usr/bin/env python3
"""End-to-end (host bytes -> host tokens) encode rate of the C3 workload
(diagnostic): gbpe_encode on 1 GiB multilingual text with the bench's 32K vocab;
prints {gbps_e2e, ms, tokens} for `reps` runs (best)."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gpu-bpe_amd"))
import numpy as np  # noqa: E402
import bench  # noqa: E402
from gpubpe import _lib, compile_vocab_to_trie, parse_header, parse_trie_buffers  # noqa: E402
from gpubpe.vocab import Vocab  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    lib = _lib.load()
    ctx = C.c_void_p()
    _lib.check(lib.gbpe_ctx_create(0, C.byref(ctx)), None, "ctx")
    sample = bench.make_corpus({"gen": "multilingual", "n": 104_857_600, "seed": 4})
    d = bench.device_buffer(lib, ctx, sample)
    merges, _ = bench.train_run(lib, ctx, d, len(sample), 32768)
    lib.gbpe_device_free(ctx, d)
    voc = Vocab()
    for a, b in merges[:, :2].tolist():
        voc.add_merge(a, b)
    blob = compile_vocab_to_trie(voc.entries)
    hdr = parse_header(blob)
    nodes, edges = parse_trie_buffers(blob, hdr)
    text = bench.make_corpus({"gen": "multilingual", "n": 1 << 30, "seed": 3})
    n = len(text)
    trie = C.c_void_p()
    _lib.check(lib.gbpe_trie_upload(ctx, nodes.ctypes.data_as(_lib.u32p), hdr["nodeCount"],
                                    edges.ctypes.data_as(_lib.u32p), hdr["edgeCount"], C.byref(trie)), ctx, "trie")
    cs = max(512, min(2048, hdr["maxTokenLen"] * 8))
    out = np.empty(n, dtype=np.uint32)
    n_out = C.c_uint64()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        _lib.check(lib.gbpe_encode(ctx, trie, text, n, cs, out.ctypes.data_as(_lib.u32p), n, C.byref(n_out)), ctx, "enc")
        ts.append(time.perf_counter() - t0)
    print(json.dumps({"gbps_e2e": n / 1e9 / min(ts), "ms": [round(1e3 * t, 2) for t in ts], "tokens": int(n_out.value)}))
    lib.gbpe_trie_free(trie)
    lib.gbpe_ctx_destroy(ctx)


if __name__ == "__main__":
    main()
