#!/usr/bin/env python3
"""Exploration run (diagnostic, not part of the product): full training runs of
the 1 GiB configurations through the C-ABI, with per-step wall times and the
trainer's stats, and the merge list dumped to gpurun_out/ for offline
comparison with the CPU oracle fixtures.

    python tools/explore_1g.py en1g ml1g code1g
"""
import ctypes as C
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-bpe_amd"))
import numpy as np  # noqa: E402
from gpubpe import _lib, synth  # noqa: E402

CONFIGS = {
    "c2": (lambda: synth.english(104_857_600, seed=2, fancy_punct=0.005), 32768, 0),
    "en1g": (lambda: synth.english(1 << 30, seed=2, fancy_punct=0.005), 32768, 0),
    "ml1g": (lambda: synth.multilingual(1 << 30, seed=3), 32768, 0),
    "code1g": (lambda: synth.code(1 << 30, seed=6), 50000, _lib.GBPE_TRAIN_GPT4_BOUNDARIES),
}


def main():
    lib = _lib.load()
    ctx = C.c_void_p()
    _lib.check(lib.gbpe_ctx_create(0, C.byref(ctx)), None, "ctx")
    out_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    reps = int(os.environ.get("EXPLORE_REPS", "1"))
    max_steps = int(os.environ.get("EXPLORE_MAX_STEPS", "0"))   # 0 = the whole run
    for name in sys.argv[1:]:
        gen, vocab, flags = CONFIGS[name]
        t = time.time()
        data = gen()
        sha = hashlib.sha256(data).hexdigest()
        print(f"[{name}] corpus {len(data)} B sha256 {sha[:16]} in {time.time() - t:.1f}s", flush=True)
        d = C.c_void_p()
        _lib.check(lib.gbpe_device_alloc(ctx, len(data) + 64, C.byref(d)), ctx, "alloc")
        _lib.check(lib.gbpe_memcpy_h2d(ctx, d, data, len(data)), ctx, "h2d")
        for rep in range(reps):
            opts = _lib.TrainOpts(target_vocab_size=vocab, vocab_size=256, next_token_id=256, batch_size=128,
                                  flags=flags, table_log2=0)
            tr = C.c_void_p()
            lib.gbpe_synchronize(ctx)
            t0 = time.perf_counter()
            _lib.check(lib.gbpe_trainer_create(ctx, d, len(data), None, 1, C.byref(opts), C.byref(tr)), ctx, "create")
            t1 = time.perf_counter()
            out = (C.c_uint32 * 512)()
            merges, steps = [], []
            while True:
                nd, es = C.c_uint32(), C.c_uint32()
                ts = time.perf_counter()
                _lib.check(lib.gbpe_trainer_step(tr, 128, out, C.byref(nd), C.byref(es)), ctx, "step")
                steps.append(time.perf_counter() - ts)
                merges += list(out[: 4 * nd.value])
                if len(steps) % 32 == 0:
                    print(f"[{name}] step {len(steps)} merges {len(merges) // 4} "
                          f"{time.perf_counter() - t1:.2f}s", flush=True)
                if nd.value == 0 or es.value or (max_steps and len(steps) >= max_steps):
                    break
            t2 = time.perf_counter()
            st = _lib.TrainerStats()
            lib.gbpe_trainer_stats_get(tr, C.byref(st))
            t3 = time.perf_counter()
            lib.gbpe_trainer_destroy(tr)
            lib.gbpe_synchronize(ctx)
            t4 = time.perf_counter()
            m = np.array(merges, dtype=np.uint32).reshape(-1, 4)
            np.save(os.path.join(out_dir, f"explore_{name}_merges.npy"), m)
            sd = {f: getattr(st, f) for f, _ in _lib.TrainerStats._fields_}
            st_ms = np.array(steps) * 1e3
            res = {"name": name, "rep": rep, "n": len(data), "sha256": sha, "merges": int(m.shape[0]),
                   "create_s": t1 - t0, "loop_s": t2 - t1, "destroy_s": t4 - t3, "merges_per_s_loop": m.shape[0] / (t2 - t1),
                   "merges_per_s_total": m.shape[0] / (t2 - t0),
                   "step_ms_first10": [round(x, 2) for x in st_ms[:10]],
                   "step_ms_by_32": [round(float(st_ms[i:i + 32].sum()), 1) for i in range(0, len(st_ms), 32)],
                   "stats": sd, "last_merge": m[-1].tolist() if len(m) else None}
            print(json.dumps(res), flush=True)
        lib.gbpe_device_free(ctx, d)
    lib.gbpe_ctx_destroy(ctx)


if __name__ == "__main__":
    main()
