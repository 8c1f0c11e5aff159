#!/usr/bin/env python3
"""One C3 encode window for profiling (diagnostic): the bench's C3 vocab (32K,
trained on the GPU on the 100 MiB multilingual sample, seed 4), then `reps`
encodes of 1 GiB multilingual text (seed 3), device-resident.  Prints one JSON
line {bytes, tokens, chunk_size, reps, ms_walk, ms_scan, ms_compact} (means; the minimum walk; sha256 prefix of the tokens).  argv[2]: another libgpubpe.so (A/B builds)."""
import ctypes as C
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gpu-bpe_amd"))
import numpy as np  # noqa: E402
import bench  # noqa: E402
from gpubpe import _lib, compile_vocab_to_trie, parse_header, parse_trie_buffers  # noqa: E402
from gpubpe.vocab import Vocab  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    lib = _lib.load(sys.argv[2] if len(sys.argv) > 2 else None)
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
    d_in = bench.device_buffer(lib, ctx, text)
    d_out = C.c_void_p()
    _lib.check(lib.gbpe_device_alloc(ctx, 4 * n + 64, C.byref(d_out)), ctx, "alloc")
    n_out = C.c_uint64()
    ms = []
    for _ in range(reps):
        _lib.check(lib.gbpe_encode_device(ctx, trie, d_in, n, cs, d_out, n, C.byref(n_out)), ctx, "encode")
        w, sc, cp = C.c_double(), C.c_double(), C.c_double()
        lib.gbpe_encode_last_timing(ctx, C.byref(w), C.byref(sc), C.byref(cp))
        ms.append((w.value, sc.value, cp.value))
    lib.gbpe_synchronize(ctx)
    host = np.empty(int(n_out.value), np.uint32)
    _lib.check(lib.gbpe_memcpy_d2h(ctx, host.ctypes.data_as(C.c_void_p), d_out, 4 * host.shape[0]), ctx, "d2h")
    digest = hashlib.sha256(host.tobytes()).hexdigest()[:16]
    del host
    m = np.mean(np.array(ms), axis=0)
    print(json.dumps({"bytes": n, "tokens": int(n_out.value), "chunk_size": cs, "reps": reps,
                      "ms_walk": m[0], "ms_scan": m[1], "ms_compact": m[2],
                      "ms_walk_min": float(np.min(np.array(ms)[:, 0])), "sha256_16": digest, "lib": sys.argv[2] if len(sys.argv) > 2 else None}),
          flush=True)
    lib.gbpe_device_free(ctx, d_in)
    lib.gbpe_device_free(ctx, d_out)
    lib.gbpe_trie_free(trie)
    lib.gbpe_ctx_destroy(ctx)


if __name__ == "__main__":
    main()
