#!/usr/bin/env python3
"""A/B of library builds (diagnostic): alternating complete training runs of
the named configurations with each libgpubpe.so, every run's merge list
compared with its committed oracle fixture.

    python tools/ab_libs.py gpu-bpe_amd/lib/A/libgpubpe.so gpu-bpe_amd/lib/B/libgpubpe.so:GBPE_X=0 -- en1g c2 code1g

(a library may carry environment settings after a colon, separated by "@", so
that a GBPE_DEBUG value can hold commas: lib.so:GBPE_DEBUG=zt=4,subk=8@X=1)

Each library runs in its own child process (one .so per process); the runs
alternate A, B, A, B so drift on the box hits both alike.  AB_TABLE_LOG2 sets
the trainer's table_log2 option (0 = sized by the trainer).
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import ctypes as C, json, os, sys, time
sys.path.insert(0, os.path.join(sys.argv[1], "gpu-bpe_amd"))
import numpy as np
from gpubpe import _lib, synth
CONF = {
    "c1": (lambda: synth.english(262_144, seed=1), 1024, 0),
    "c2": (lambda: synth.english(104_857_600, seed=2, fancy_punct=0.005), 32768, 0),
    "en1g": (lambda: synth.english(1 << 30, seed=2, fancy_punct=0.005), 32768, 0),
    "ml1g": (lambda: synth.multilingual(1 << 30, seed=3), 32768, 0),
    "code1g": (lambda: synth.code(1 << 30, seed=6), 50000, _lib.GBPE_TRAIN_GPT4_BOUNDARIES),
    "ml1g64k": (lambda: synth.multilingual(1 << 30, seed=5), 65536, 0),   # bench.py's C4 shard (u32)
}
lib = _lib.load(sys.argv[2])
ctx = C.c_void_p()
_lib.check(lib.gbpe_ctx_create(0, C.byref(ctx)), None, "ctx")
reps = int(sys.argv[3])
for name in sys.argv[4:]:
    gen, vocab, flags = CONF[name]
    cache = os.path.join(os.environ.get("TMPDIR", "/tmp"), "gbpe_ab_corpus_" + name + ".bin")
    if os.path.exists(cache):   # (generated once per box: every child of the A/B reads it back)
        data = open(cache, "rb").read()
    else:
        data = gen()
        with open(cache + ".part", "wb") as f:
            f.write(data)
        os.replace(cache + ".part", cache)
    fx = np.load(os.path.join(sys.argv[1], "tests", "golden", "train_" + name + ".npz"))["merges"]
    d = C.c_void_p()
    _lib.check(lib.gbpe_device_alloc(ctx, len(data) + 64, C.byref(d)), ctx, "alloc")
    _lib.check(lib.gbpe_memcpy_h2d(ctx, d, data, len(data)), ctx, "h2d")
    for rep in range(reps + 1):   # the first run warms up
        opts = _lib.TrainOpts(target_vocab_size=vocab, vocab_size=256, next_token_id=256, batch_size=128,
                              flags=flags, table_log2=int(os.environ.get("AB_TABLE_LOG2", "0")))
        tr = C.c_void_p()
        lib.gbpe_synchronize(ctx)
        t0 = time.perf_counter()
        _lib.check(lib.gbpe_trainer_create(ctx, d, len(data), None, 1, C.byref(opts), C.byref(tr)), ctx, "create")
        out = (C.c_uint32 * 512)()
        merges = []
        t4k = None
        while True:
            nd, es = C.c_uint32(), C.c_uint32()
            _lib.check(lib.gbpe_trainer_step(tr, 128, out, C.byref(nd), C.byref(es)), ctx, "step")
            merges += list(out[: 4 * nd.value])
            if t4k is None and len(merges) >= 4 * 4096:
                t4k = time.perf_counter()
            if nd.value == 0 or es.value:
                break
        t1 = time.perf_counter()
        sbuf = (C.c_char * 1024)()   # (room for a library built against another stats layout)
        st = _lib.TrainerStats.from_buffer(sbuf)
        lib.gbpe_trainer_stats_get(tr, C.byref(st))
        lib.gbpe_trainer_destroy(tr)
        m = np.array(merges, dtype=np.uint32).reshape(-1, 4)
        eq = m.shape == fx.shape and bool((m == fx).all())
        if rep:
            print(json.dumps({"name": name, "s": round(t1 - t0, 4), "s_first4k": round((t4k or t1) - t0, 4),
                              "merges": int(m.shape[0]), "equal": eq,
                              "sparse_exits": int(st.sparse_exits),
                              "table_slots": int(st.table_slots), "max_live_pairs": int(st.max_live_pairs),
                              "paired": int(getattr(st, "paired_merges", 0))}), flush=True)
        if not eq:
            print(json.dumps({"name": name, "error": "merges differ from the fixture"}), flush=True)
            sys.exit(3)
    lib.gbpe_device_free(ctx, d)
lib.gbpe_ctx_destroy(ctx)
"""


def main():
    i = sys.argv.index("--")
    libs, names = sys.argv[1:i], sys.argv[i + 1:]
    reps = int(os.environ.get("AB_REPS", "2"))
    rounds = int(os.environ.get("AB_ROUNDS", "2"))
    res = {}
    for r in range(rounds):
        for lp in libs:   # "path" or "path:ENV=V@ENV2=V2"
            path, _, envs = lp.partition(":")
            env = dict(os.environ)
            env.update(kv.split("=", 1) for kv in envs.split("@") if kv)
            p = subprocess.run([sys.executable, "-c", CHILD, ROOT, os.path.abspath(path), str(reps)] + names,
                               capture_output=True, text=True, timeout=600, env=env)
            for line in p.stdout.splitlines():
                j = json.loads(line)
                if "error" in j:
                    print(lp, j, flush=True)
                    print(p.stderr[-3000:], flush=True)
                    sys.exit(3)
                res.setdefault((lp, j["name"]), []).append(j["s"])
                print(lp, line, flush=True)
            if p.returncode:
                print(lp, "rc", p.returncode, p.stderr[-2000:], flush=True)
                sys.exit(p.returncode)
            if os.environ.get("AB_STDERR"):   # the children's diagnostics (GBPE_DEBUG=htime=1: [pair], [htime])
                for line in p.stderr.splitlines():
                    if line.startswith("["):
                        print(lp, line, flush=True)
            print(f"round {r} {lp} done", flush=True)
    for (lp, name), v in sorted(res.items(), key=lambda kv: (kv[0][1], kv[0][0])):
        print(f"{name:8s} {lp:50s} min {min(v):.4f} s  all {[round(x, 4) for x in v]}")


if __name__ == "__main__":
    main()
