#!/usr/bin/env python3
"""Benchmark: BPE merges/sec (+ tokenize GB/s) on MI355X through the C-ABI.

Workload (BASELINE.json configs[1]): 32K-vocab training
on 104,857,600 bytes of synthetic English UTF-8 (seed 2), heuristic word
boundaries, reference compaction semantics.  A "step" is one batch of 128
merges (the reference's GPU round trip, training-pipeline.js:13); the timed
region covers trainer creation on the HBM-resident corpus (symbol widening,
word boundaries, initial pair count) plus K steps.  `value` = merges / s.

Secondary leg (configs[2], C3): chunked trie encode of 1 GiB synthetic
multilingual text with a 32K vocab trained on a 100 MiB sample (seed 4).

Multi-GPU (--gpus N under torch.distributed.run): N>1 is not yet sharded
(SURVEY §8(e) training needs a per-merge count exchange, planned); each rank
runs the same single-GPU workload as an independent replica and the line
reports `"parallelism": "replicas"`.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gpu-bpe_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_env():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("LOCAL_RANK", "0"))


class Dist:
    """barrier / max over ranks via torch.distributed (gloo on host — the
    timing collectives carry a few bytes, no data path)."""

    def __init__(self, world):
        self.world = world
        self.pg = None
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x: float) -> float:
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())


def device_buffer(lib, ctx, data: bytes):
    from gpubpe import _lib
    p = C.c_void_p()
    _lib.check(lib.gbpe_device_alloc(ctx, len(data) + 64, C.byref(p)), ctx, "alloc")
    _lib.check(lib.gbpe_memcpy_h2d(ctx, p, data, len(data)), ctx, "h2d")
    return p


def run_train(lib, ctx, d_bytes, n, vocab, steps, flags, batch=128):
    """Create a trainer on HBM-resident bytes and run up to `steps` batches."""
    from gpubpe import _lib
    opts = _lib.TrainOpts(target_vocab_size=vocab, vocab_size=256, next_token_id=256, batch_size=batch,
                          flags=flags, table_log2=0)
    tr = C.c_void_p()
    _lib.check(lib.gbpe_trainer_create(ctx, d_bytes, n, None, 1, C.byref(opts), C.byref(tr)), ctx, "trainer_create")
    merges = 0
    done_steps = 0
    stop = False
    out = (C.c_uint32 * (4 * batch))()
    last = []
    dump = [] if os.environ.get("BENCH_DUMP_MERGES") and flags else None
    while done_steps < steps and not stop:
        nd, es = C.c_uint32(), C.c_uint32()
        _lib.check(lib.gbpe_trainer_step(tr, batch, out, C.byref(nd), C.byref(es)), ctx, "trainer_step")
        merges += nd.value
        done_steps += 1
        stop = bool(es.value) or nd.value == 0
        if nd.value:
            last = list(out[4 * (nd.value - 1): 4 * nd.value])
            if dump is not None:
                dump += list(out[: 4 * nd.value])
    if dump is not None:   # diagnostic: per-merge (a, b, id, count) of the timed run
        import numpy as np
        np.save(os.environ["BENCH_DUMP_MERGES"], np.array(dump, dtype=np.uint32).reshape(-1, 4))
    return tr, merges, done_steps, stop, last


def first_merges(lib, ctx, data: bytes, vocab: int, k: int):
    from gpubpe import _lib
    d = device_buffer(lib, ctx, data)
    opts = _lib.TrainOpts(target_vocab_size=vocab, vocab_size=256, next_token_id=256, batch_size=128, flags=0,
                          table_log2=0)
    tr = C.c_void_p()
    _lib.check(lib.gbpe_trainer_create(ctx, d, len(data), None, 1, C.byref(opts), C.byref(tr)), ctx, "create")
    out = (C.c_uint32 * (4 * 128))()
    got = []
    while len(got) < k:
        nd, es = C.c_uint32(), C.c_uint32()
        _lib.check(lib.gbpe_trainer_step(tr, min(128, k - len(got)), out, C.byref(nd), C.byref(es)), ctx, "step")
        got += [list(out[4 * i: 4 * i + 4]) for i in range(nd.value)]
        if nd.value == 0 or es.value:
            break
    lib.gbpe_trainer_destroy(tr)
    lib.gbpe_device_free(ctx, d)
    return got


def train_leg(args, lib, ctx, dist, rank):
    from gpubpe import _lib, synth
    n = args.train_bytes
    t = time.time()
    data = synth.english(n, seed=2, fancy_punct=0.005)
    log(f"[bench] C2 corpus {n} B generated in {time.time() - t:.1f}s")
    d = device_buffer(lib, ctx, data)
    # warmup: W batches on a 8 MiB prefix (code paths, allocator, caches)
    if args.warmup > 0:
        tr, _, _, _, _ = run_train(lib, ctx, d, min(n, 8 << 20), args.vocab, args.warmup, 0)
        lib.gbpe_trainer_destroy(tr)
    lib.gbpe_synchronize(ctx)
    dist.barrier()
    lib.gbpe_synchronize(ctx)
    t0 = time.perf_counter()
    tr, merges, steps, stop, last = run_train(lib, ctx, d, n, args.vocab, args.steps, 0)
    lib.gbpe_synchronize(ctx)
    t1 = time.perf_counter()
    dist.barrier()
    st = _lib.TrainerStats()
    lib.gbpe_trainer_stats_get(tr, C.byref(st))
    lib.gbpe_trainer_destroy(tr)
    wall = dist.max(t1 - t0)
    # roofline pass: the same run again with HIP events around every launch (the
    # event markers add inter-kernel gaps, so they stay out of the timed run)
    sk = _lib.TrainerStats()
    if not args.no_kernel_timing:
        tr2, _, _, _, _ = run_train(lib, ctx, d, n, args.vocab, args.steps, _lib.GBPE_TRAIN_TIMING)
        lib.gbpe_trainer_stats_get(tr2, C.byref(sk))
        lib.gbpe_trainer_destroy(tr2)
    lib.gbpe_device_free(ctx, d)
    res = {
        "merges": merges, "steps": steps, "early_stop": stop, "wall_s": wall,
        "final_symbols": int(st.symbol_count), "bytes_per_symbol": int(st.bytes_per_symbol),
        "stream_bytes": int(st.stream_bytes_moved), "ms_stream_kernels": sk.ms_merge,
        "ms_select": sk.ms_select, "ms_refresh": sk.ms_other,
        "ms_delta": sk.ms_delta, "ms_compact": sk.ms_compact, "timed_merges": int(sk.timed_merges),
        "tail_dropped": int(st.tail_dropped), "max_live_pairs": int(st.max_live_pairs),
        "last_merge": last,
    }
    return data, res


def encode_leg(args, lib, ctx, dist, rank):
    """C3: train a 32K vocab on a 100 MiB multilingual sample (seed 4), then
    encode 1 GiB multilingual text (seed 3) with the chunked trie walk."""
    from gpubpe import _lib, synth, compile_vocab_to_trie, parse_header, parse_trie_buffers
    from gpubpe.vocab import Vocab
    t = time.time()
    sample = synth.multilingual(args.vocab_sample_bytes, seed=4)
    d = device_buffer(lib, ctx, sample)
    opts = _lib.TrainOpts(target_vocab_size=args.vocab, vocab_size=256, next_token_id=256, batch_size=128, flags=0,
                          table_log2=0)
    tr = C.c_void_p()
    _lib.check(lib.gbpe_trainer_create(ctx, d, len(sample), None, 1, C.byref(opts), C.byref(tr)), ctx, "create")
    voc = Vocab()
    out = (C.c_uint32 * 512)()
    while True:
        nd, es = C.c_uint32(), C.c_uint32()
        _lib.check(lib.gbpe_trainer_step(tr, 128, out, C.byref(nd), C.byref(es)), ctx, "step")
        for i in range(nd.value):
            voc.add_merge(out[4 * i], out[4 * i + 1])
        if nd.value == 0 or es.value:
            break
    lib.gbpe_trainer_destroy(tr)
    lib.gbpe_device_free(ctx, d)
    blob = compile_vocab_to_trie(voc.entries)
    hdr = parse_header(blob)
    nodes, edges = parse_trie_buffers(blob, hdr)
    log(f"[bench] C3 vocab {voc.size} tokens, trie {hdr['nodeCount']} nodes in {time.time() - t:.1f}s")
    t = time.time()
    text = synth.multilingual(args.encode_bytes, seed=3)
    n = len(text)
    log(f"[bench] C3 corpus {n} B generated in {time.time() - t:.1f}s")
    trie = C.c_void_p()
    _lib.check(lib.gbpe_trie_upload(ctx, nodes.ctypes.data_as(_lib.u32p), hdr["nodeCount"],
                                    edges.ctypes.data_as(_lib.u32p), hdr["edgeCount"], C.byref(trie)), ctx, "trie")
    cs = max(512, min(2048, hdr["maxTokenLen"] * 8))            # tokenizer.js:67-68
    d_in = device_buffer(lib, ctx, text)
    d_out = C.c_void_p()
    _lib.check(lib.gbpe_device_alloc(ctx, 4 * n + 64, C.byref(d_out)), ctx, "alloc out")
    n_out = C.c_uint64()
    _lib.check(lib.gbpe_encode_device(ctx, trie, d_in, n, cs, d_out, n, C.byref(n_out)), ctx, "encode warmup")
    reps = 3
    kms = []
    dist.barrier()
    lib.gbpe_synchronize(ctx)
    t0 = time.perf_counter()
    for _ in range(reps):
        _lib.check(lib.gbpe_encode_device(ctx, trie, d_in, n, cs, d_out, n, C.byref(n_out)), ctx, "encode")
        w, sc, cp = C.c_double(), C.c_double(), C.c_double()
        lib.gbpe_encode_last_timing(ctx, C.byref(w), C.byref(sc), C.byref(cp))
        kms.append((w.value, sc.value, cp.value))
    lib.gbpe_synchronize(ctx)
    wall = dist.max((time.perf_counter() - t0) / reps)
    T = int(n_out.value)
    k_walk = float(np.mean([k[0] for k in kms]))
    k_all = float(np.mean([sum(k) for k in kms]))
    # end-to-end host -> tokens -> host (the reference's MB/s definition, export-controller.js:210-213)
    host_out = np.empty(n, dtype=np.uint32)
    t0 = time.perf_counter()
    _lib.check(lib.gbpe_encode(ctx, trie, text, n, cs, host_out.ctypes.data_as(_lib.u32p), n, C.byref(n_out)),
               ctx, "encode e2e")
    e2e = time.perf_counter() - t0
    tokens = host_out[: n_out.value]
    lib.gbpe_device_free(ctx, d_in)
    lib.gbpe_device_free(ctx, d_out)
    lib.gbpe_trie_free(trie)
    alg = n + 4 * T
    res = {
        "workload": "C3: chunked greedy trie encode of 1,073,741,824 B multilingual UTF-8 (seed 3), 32K vocab "
                    f"trained on a {args.vocab_sample_bytes} B sample (seed 4), chunk {cs}",
        "bytes": n, "tokens": T, "chunk_size": cs,
        "gbps_kernels": round(n / 1e9 / (k_all / 1e3), 2),
        "gbps_device_wall": round(n / 1e9 / wall, 2),
        "gbps_end_to_end": round(n / 1e9 / e2e, 2),
        "ms_walk": round(k_walk, 3), "ms_scan": round(float(np.mean([k[1] for k in kms])), 3),
        "ms_compact": round(float(np.mean([k[2] for k in kms])), 3),
        "roofline": {"bound": "hbm", "kernel": "k_trie_walk + k_chunk_scan + k_chunk_compact",
                     "achieved": round(alg / 1e9 / (k_all / 1e3), 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(alg / 1e9 / (k_all / 1e3) / HBM_PEAK_GBPS, 4), "algorithmic_bytes": alg,
                     "traffic": None},
    }
    return text, nodes, edges, cs, tokens, res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=254, help="timed batches of 128 merges (254 = full 32K vocab)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--vocab", type=int, default=32768)
    ap.add_argument("--train-bytes", type=int, default=104_857_600)
    ap.add_argument("--encode-bytes", type=int, default=1 << 30)
    ap.add_argument("--vocab-sample-bytes", type=int, default=104_857_600)
    ap.add_argument("--no-encode", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true", help="skip the HIP-event roofline pass")
    ap.add_argument("--cpu-merges", type=int, default=0, help="CPU baseline merges (0 = auto, ~10-30 s)")
    args = ap.parse_args()

    rank, world, local = dist_env()
    dist = Dist(world)
    from gpubpe import _lib
    lib = _lib.load()
    ctx = C.c_void_p()
    rc = lib.gbpe_ctx_create(local if world > 1 else 0, C.byref(ctx))
    if rc != 0:
        raise SystemExit(f"gbpe_ctx_create failed ({rc}): no MI355X visible")

    data, tr = train_leg(args, lib, ctx, dist, rank)
    total_merges = dist.sum(tr["merges"]) if world > 1 else tr["merges"]
    value = total_merges / tr["wall_s"]
    ms_stream = tr["ms_stream_kernels"]
    achieved = (tr["stream_bytes"] / 1e9) / (ms_stream / 1e3) if ms_stream > 0 else None
    line = {
        "metric": "BPE merges/sec + tokenize GB/s, 1 GiB UTF-8 @ 32K vocab, 1/2/4/8 MI355X",
        "value": round(value, 1),
        "unit": "merges/s",
        "n_gpus": world,
        "steps": tr["steps"],
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * tr["wall_s"] / max(1, tr["steps"]), 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": f"u{8 * tr['bytes_per_symbol']}",
        "data": "synthetic (seeded Zipf English-like corpus, gpubpe.synth)",
        "config": {"workload": "C2: 32K-vocab BPE train on 104,857,600 B English UTF-8 (seed 2), heuristic "
                               "word boundaries, reference compaction; step = 128 merges",
                   "train_bytes": args.train_bytes, "target_vocab": args.vocab,
                   "merges_timed": tr["merges"], "early_stop": tr["early_stop"],
                   "parallelism": "single" if world == 1 else "replicas"},
        "roofline": {
            "bound": "hbm",
            "kernel": "stream pass per merge: k_delta + k_compact",
            "achieved": round(achieved, 1) if achieved else None,
            "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4) if achieved else None,
            "algorithmic_bytes": tr["stream_bytes"],
            "traffic": None,
        },
        "train_detail": tr,
    }

    pmc = os.path.join(ROOT, "profiles", "r1_pmc_traffic.json")
    if os.path.exists(pmc) and args.train_bytes == 104_857_600 and tr["bytes_per_symbol"] == 2:
        # HBM bytes per merge of k_delta + k_compact from the committed rocprofv3 --pmc
        # passes (FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction), on the first merges of
        # this same workload; scaled to the per-merge algorithmic bytes of this run
        p = json.load(open(pmc))
        ratio = p["traffic_over_algorithmic"]
        line["roofline"]["traffic"] = round(ratio * tr["stream_bytes"] / max(1, tr["merges"]))
        line["roofline"]["traffic_unit"] = "bytes/merge (k_delta + k_compact)"
        line["roofline"]["traffic_over_algorithmic"] = round(ratio, 4)
        line["roofline"]["traffic_sample"] = (f"profiles/r1_pmc_traffic.json: first {p['merges']} merges, "
                                              f"FETCH_SIZE and WRITE_SIZE passes")

    enc = None
    if not args.no_encode:
        enc = encode_leg(args, lib, ctx, dist, rank)
        line["tokenize"] = enc[-1]

    if rank == 0 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import cpu_ref
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
        k = args.cpu_merges or 256
        t = time.perf_counter()
        r = cpu_ref.train(data, args.vocab, max_merges=k, threads=threads, want_symbols=False)
        dt = time.perf_counter() - t
        line["cpu_baseline"] = {"value": round(len(r["merges"]) / dt, 3), "unit": "merges/s", "cores": threads,
                                "kind": "port",
                                "sample": f"first {len(r['merges'])} merges of the same C2 corpus, full pair "
                                          f"recount per merge (reference algorithm, oracle/bpe_oracle.c), {dt:.1f}s"}
        # full-size parity: the GPU run's first k merges equal the CPU restatement's
        g = first_merges(lib, ctx, data, args.vocab, len(r["merges"]))
        line["parity"] = {"train_first_merges_equal": g == r["merges"], "train_merges_checked": len(r["merges"])}
        if enc is not None:
            text, nodes, edges, cs, tokens, er = enc
            t = time.perf_counter()
            ref_tokens = cpu_ref.encode(text, nodes, edges, cs, threads=threads)
            dt = time.perf_counter() - t
            er["cpu_baseline"] = {"value": round(len(text) / 1e9 / dt, 3), "unit": "GB/s", "cores": threads,
                                  "kind": "port", "sample": f"full {len(text)} B encode, chunked greedy trie walk "
                                                            f"(oracle/bpe_oracle.c), {dt:.1f}s"}
            line["parity"]["encode_tokens_equal"] = bool(np.array_equal(tokens, ref_tokens))
            line["parity"]["encode_tokens_checked"] = int(len(ref_tokens))
    if rank == 0:
        print(json.dumps(line), flush=True)
    lib.gbpe_ctx_destroy(ctx)


if __name__ == "__main__":
    main()
