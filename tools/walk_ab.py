#!/usr/bin/env python3
"""A/B of trie-walk variants in one process (diagnostic): the bench's C3 vocab
(32K, trained on the GPU on the 100 MiB multilingual sample, seed 4), then for
each GBPE_WALK_R value `reps` encodes of 1 GiB multilingual text (seed 3) and of
256 MiB English / code, device-resident.  Every variant's tokens must equal the
first variant's.  Prints one JSON line per (corpus, variant)."""
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
    variants = sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "16", "32"]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
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
    trie = C.c_void_p()
    _lib.check(lib.gbpe_trie_upload(ctx, nodes.ctypes.data_as(_lib.u32p), hdr["nodeCount"],
                                    edges.ctypes.data_as(_lib.u32p), hdr["edgeCount"], C.byref(trie)), ctx, "trie")
    auto_cs = max(512, min(2048, hdr["maxTokenLen"] * 8))
    for spec in ({"gen": "multilingual", "n": 1 << 30, "seed": 3}, {"gen": "english", "n": 1 << 28, "seed": 5},
                 {"gen": "code", "n": 1 << 28, "seed": 6}):
        text = bench.make_corpus(spec)
        n = len(text)
        d_in = bench.device_buffer(lib, ctx, text)
        d_out = C.c_void_p()
        _lib.check(lib.gbpe_device_alloc(ctx, 4 * n + 64, C.byref(d_out)), ctx, "alloc")
        for cs in (auto_cs, 64):
            want = None
            for v in variants:
                os.environ[os.environ.get("AB_VAR", "GBPE_WALK_NT")] = v
                n_out = C.c_uint64()
                ms = []
                for _ in range(reps):
                    _lib.check(lib.gbpe_encode_device(ctx, trie, d_in, n, cs, d_out, n, C.byref(n_out)), ctx, "encode")
                    w, sc, cp = C.c_double(), C.c_double(), C.c_double()
                    lib.gbpe_encode_last_timing(ctx, C.byref(w), C.byref(sc), C.byref(cp))
                    ms.append(w.value)
                toks = np.empty(n_out.value, np.uint32)
                _lib.check(lib.gbpe_memcpy_d2h(ctx, toks.ctypes.data_as(C.c_void_p), d_out, toks.nbytes), ctx, "d2h")
                h = hashlib.sha256(toks.tobytes()).hexdigest()[:16]
                if want is None:
                    want = h
                print(json.dumps({"corpus": spec["gen"], "bytes": n, "cs": cs, "walk_r": v, "tokens": int(n_out.value),
                                  "sha": h, "equal": h == want, "ms_walk_min": min(ms),
                                  "ms_walk_med": float(np.median(ms))}), flush=True)
                if h != want:
                    sys.exit(f"walk variant {v} differs on {spec['gen']} cs={cs}")
        lib.gbpe_device_free(ctx, d_in)
        lib.gbpe_device_free(ctx, d_out)
    lib.gbpe_trie_free(trie)
    lib.gbpe_ctx_destroy(ctx)


if __name__ == "__main__":
    main()
