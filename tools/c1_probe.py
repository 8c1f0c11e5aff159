#!/usr/bin/env python3
"""C1 probe (diagnostic): the bench's C1 run (256 KiB ASCII @ 1K vocab), three
times, with the trainer's stats (dense / sparse merges) and per-step times."""
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


def main():
    lib = _lib.load()
    ctx = C.c_void_p()
    _lib.check(lib.gbpe_ctx_create(0, C.byref(ctx)), None, "ctx")
    data = bench.make_corpus({"gen": "english", "n": 262_144, "seed": 1})
    d = bench.device_buffer(lib, ctx, data)
    for rep in range(3):
        steps = []
        t0 = time.perf_counter()
        m, st = bench.train_run(lib, ctx, d, len(data), 1024, steps_out=steps)
        dt = time.perf_counter() - t0
        print(json.dumps({"rep": rep, "s": round(dt, 5), "merges": int(m.shape[0]), "sparse_merges": int(st.sparse_merges),
                          "sparse_enters": int(st.sparse_enters), "steps_ms": [round(s * 1e3, 2) for _, s in steps]}), flush=True)
    lib.gbpe_device_free(ctx, d)
    lib.gbpe_ctx_destroy(ctx)


if __name__ == "__main__":
    main()
