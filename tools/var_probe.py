#!/usr/bin/env python3
"""Run-to-run variance probe (diagnostic): whole 1 GiB headline runs, (a) in one
context with its pooled buffers reused, (b) each in a fresh context with a fresh
corpus buffer (new device allocations every run).  Prints one JSON line."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gpu-bpe_amd"))
import bench  # noqa: E402
from gpubpe import _lib  # noqa: E402


def one(lib, ctx, d, n):
    t0 = time.perf_counter()
    m, st = bench.train_run(lib, ctx, d, n, 32768)
    return round(time.perf_counter() - t0, 4), int(m.shape[0])


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    lib = _lib.load()
    data = bench.make_corpus({"gen": "english", "n": 1 << 30, "seed": 2, "fancy_punct": 0.005})
    res = {"reuse": [], "fresh": []}
    ctx = C.c_void_p()
    _lib.check(lib.gbpe_ctx_create(0, C.byref(ctx)), None, "ctx")
    d = bench.device_buffer(lib, ctx, data)
    for _ in range(reps):
        res["reuse"].append(one(lib, ctx, d, len(data)))
        print("reuse", res["reuse"][-1], file=sys.stderr, flush=True)
    lib.gbpe_device_free(ctx, d)
    lib.gbpe_ctx_destroy(ctx)
    for _ in range(reps):
        ctx = C.c_void_p()
        _lib.check(lib.gbpe_ctx_create(0, C.byref(ctx)), None, "ctx")
        d = bench.device_buffer(lib, ctx, data)
        one(lib, ctx, d, len(data))   # (the new buffers' first run)
        res["fresh"].append(one(lib, ctx, d, len(data)))
        print("fresh", res["fresh"][-1], file=sys.stderr, flush=True)
        lib.gbpe_device_free(ctx, d)
        lib.gbpe_ctx_destroy(ctx)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
