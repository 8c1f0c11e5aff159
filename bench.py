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

Multi-GPU (--gpus N under torch.distributed.run, one rank per GPU): sharded
training (gpubpe.sharded).  Each rank holds a 104,857,600-byte
English shard (seed 2 + rank, newline-terminated so shard starts are word
starts) and the ranks train ONE global 32K vocab over the N-shard corpus,
bit-exact to a single-stream run, with one RCCL all-gather of a fixed-size
exchange record per merge.  Weak scaling: `value` = shard-merges/s = N x
global merges / max wall (one merge applied to one 100 MiB shard is the unit
of work at every N).  The encode leg runs one 1 GiB corpus per rank (seed
3 + rank, no collective) and reports the total.
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
TILE_SYMS = 8192
METRIC = "BPE merges/sec + tokenize GB/s, 1 GiB UTF-8 @ 32K vocab, 1/2/4/8 MI355X"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_env():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("LOCAL_RANK", "0"))


class Dist:
    """Process groups: the default group carries the sharded trainer's data path
    (RCCL = backend "nccl" over xGMI; GBPE_SHARD_TRANSPORT=gloo stages records
    through host memory instead); a gloo group carries the timing scalars
    (barrier / max / sum of a few bytes)."""

    def __init__(self, world, local, force=False):
        local = int(os.environ.get("GBPE_BENCH_DEVICE", local))   # rehearsal: several ranks on one GPU
        self.world = world
        self.transport = os.environ.get("GBPE_SHARD_TRANSPORT", "nccl")
        if world > 1 or force:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29571")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            import torch
            import torch.distributed as dist
            torch.cuda.set_device(local)
            if self.transport == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            else:
                dist.init_process_group("gloo")
            self.dist = dist
            self.host = dist.new_group(backend="gloo")

    def barrier(self):
        if hasattr(self, "host"):
            self.dist.barrier(group=self.host)

    def max(self, x: float) -> float:
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.host)
        return float(t.item())

    def sum(self, x: float) -> float:
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.host)
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
        "sparse": {"merges": int(st.sparse_merges), "enters": int(st.sparse_enters), "exits": int(st.sparse_exits),
                   "sectors": int(st.sparse_sectors), "zone_at_entry": int(st.sparse_zone)},
        # by mode, from the HIP-event pass: the dense merges' stream kernels and the
        # sector-sparse merges' k_body (+ multi-tile zone passes); bytes actually moved
        "dense_merges": int(sk.timed_merges - sk.sparse_merges), "dense_bytes": int(sk.dense_bytes),
        "ms_dense": sk.ms_dense, "sparse_merges": int(sk.sparse_merges), "body_bytes": int(sk.body_bytes),
        "zone_bytes": int(sk.zone_bytes), "ms_body": sk.ms_body, "ms_sparse": sk.ms_sparse,
        "body_bytes_run": int(st.body_bytes),   # the timed run's k_body bytes (PMC comparisons)
    }
    return data, res


def shard_corpus(args, rank):
    from gpubpe import synth
    data = synth.english(args.train_bytes, seed=2 + rank, fancy_punct=0.005)
    return data[:-1] + b"\n"          # shard starts stay word starts in the global stream


_COMM = {}   # one RCCL communicator per process, created in the warmup (outside the timed region)


def run_sharded(args, lib, ctx, dist, rank, world, d, n, steps, table_log2):
    import torch
    from gpubpe.sharded import GpuShardBackend, ShardedTrainer
    be = GpuShardBackend(lib, ctx, d, None, rank, world, args.vocab, input_on_device=True, n=n,
                         table_log2=table_log2, cap_extra=max(TILE_SYMS, n // 4),
                         stream=torch.cuda.current_stream().cuda_stream)
    tr = ShardedTrainer(be, dist.dist, device="cuda", staged=dist.transport != "nccl")
    tr.setup()
    if dist.transport == "nccl" and os.environ.get("GBPE_SHARD_LOOP", "native") == "native" and \
            _COMM.get("ok", True):
        # whole steps inside the library: RCCL all-gather on its own stream; every
        # rank must agree, else all fall back to the host loop
        ok = 1.0
        try:
            _COMM["c"] = tr.attach_native_comm(_COMM.get("c"))
            be.owns_comm = False
        except Exception as e:  # noqa: BLE001
            log(f"[bench] rank {rank}: native step loop unavailable ({e}); using the host loop")
            ok = 0.0
        if world > 1:
            ok = -dist.max(-ok)   # min over ranks
        if ok < 1.0:
            tr.native = False
            be.comm = None
            _COMM["ok"] = False
    merges, done_steps, early = [], 0, False
    needed = min(args.vocab - 256, 128 * steps)     # stalled steps are redone: count merges, not steps
    while len(merges) < needed and not early:
        got, early = tr.step(min(128, needed - len(merges)))
        merges += got
        done_steps += 1
    return be, tr, merges, done_steps, early


def train_leg_sharded(args, lib, ctx, dist, rank, world):
    """C2-size shard per rank, one global vocab (weak scaling)."""
    t = time.time()
    data = shard_corpus(args, rank)
    log(f"[bench] rank {rank}: shard {len(data)} B generated in {time.time() - t:.1f}s")
    d = device_buffer(lib, ctx, data)
    n = len(data)
    table_log2 = 23
    if args.warmup > 0:   # RCCL communicators, code paths: W steps on an 8 MiB prefix of every shard
        be, _, _, _, _ = run_sharded(args, lib, ctx, dist, rank, world, d, min(n, 8 << 20), args.warmup, table_log2)
        be.close()
    lib.gbpe_synchronize(ctx)
    dist.barrier()
    lib.gbpe_synchronize(ctx)
    t0 = time.perf_counter()
    be, tr, merges, steps, early = run_sharded(args, lib, ctx, dist, rank, world, d, n, args.steps, table_log2)
    lib.gbpe_synchronize(ctx)
    t1 = time.perf_counter()
    dist.barrier()
    st = be.stats()
    be.close()
    lib.gbpe_device_free(ctx, d)
    wall = dist.max(t1 - t0)
    stream_bytes = int(dist.sum(float(st.stream_bytes_moved)))
    res = {
        "merges": len(merges), "steps": steps, "early_stop": early, "wall_s": wall,
        "final_symbols_rank": int(st.symbol_count), "bytes_per_symbol": int(st.bytes_per_symbol),
        "stream_bytes": stream_bytes, "stalls": tr.stalls, "record_caps": [tr.C, tr.Cw],
        "transport": dist.transport + (" (native step loop)" if tr.native else " (host loop)"), "last_merge": merges[-1] if merges else [],
        "tail_dropped": int(st.tail_dropped),
    }
    return data, merges, res


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
    text = synth.multilingual(args.encode_bytes, seed=3 + rank)   # one corpus per rank (no collective)
    n = len(text)
    log(f"[bench] C3 corpus {n} B generated in {time.time() - t:.1f}s")
    trie = C.c_void_p()
    _lib.check(lib.gbpe_trie_upload(ctx, nodes.ctypes.data_as(_lib.u32p), hdr["nodeCount"],
                                    edges.ctypes.data_as(_lib.u32p), hdr["edgeCount"], C.byref(trie)), ctx, "trie")
    cs = max(512, min(2048, hdr["maxTokenLen"] * 8))            # tokenizer.js:67-68
    nrec = C.c_uint32()
    lib.gbpe_trie_info(trie, C.byref(nrec), None, None)
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
        "bytes": n, "tokens": T, "chunk_size": cs, "trie_nodes": int(hdr["nodeCount"]),
        "trie_records": int(nrec.value),
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
    if dist.world > 1:   # weak scaling: every rank encodes its own 1 GiB
        res["ranks"] = dist.world
        res["gbps_kernels_total"] = round(dist.sum(res["gbps_kernels"]), 2)
        res["gbps_device_wall_total"] = round(dist.sum(n) / 1e9 / wall, 2)
    return text, nodes, edges, cs, tokens, res


def train_roofline(tr):
    """Roofline of the dominant training kernel, from the HIP-event pass.

    Sector-sparse merges (most of the run) spend their time in k_body; its bytes are
    what it actually moved (candidate extents and signatures, sector symbols read and
    rewritten, the one-workgroup zone pass).  The dense merges' stream kernels are
    reported beside it with the SURVEY §8(d) bytes s*(2N_i + N_{i+1}).  The SURVEY
    formula over the whole run and its wall time is also given as the bandwidth a
    dense loop would need to match this merge rate (it is not credited as moved)."""
    dense = None
    if tr.get("ms_dense", 0) > 0:
        a = tr["dense_bytes"] / 1e9 / (tr["ms_dense"] / 1e3)
        dense = {"kernel": "k_delta + k_compact (dense merges)", "merges": tr["dense_merges"],
                 "achieved": round(a, 1), "frac": round(a / HBM_PEAK_GBPS, 4), "algorithmic_bytes": tr["dense_bytes"],
                 "ms": round(tr["ms_dense"], 2)}
    equiv = tr["stream_bytes"] / 1e9 / tr["wall_s"]
    if tr.get("ms_body", 0) > 0 and tr.get("sparse_merges", 0) > 0:
        a = tr["body_bytes"] / 1e9 / (tr["ms_body"] / 1e3)
        roof = {"bound": "hbm", "kernel": "k_body (sector-sparse merge pass, one launch per merge)",
                "achieved": round(a, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(a / HBM_PEAK_GBPS, 4),
                "algorithmic_bytes": tr["body_bytes"],
                "bytes_per_launch": round(tr["body_bytes"] / tr["sparse_merges"]),
                "us_per_launch": round(1e3 * tr["ms_body"] / tr["sparse_merges"], 2),
                "launches": tr["sparse_merges"], "traffic": None,
                "note": "latency-bound by design: a late merge touches ~100 sectors, so it moves kilobytes, "
                        "not the stream; frac is low because the loop avoids the bytes, not because it wastes them"}
    else:
        a = dense["achieved"] if dense else None
        roof = {"bound": "hbm", "kernel": "stream pass per merge: k_delta + k_compact", "achieved": a,
                "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(a / HBM_PEAK_GBPS, 4) if a else None,
                "algorithmic_bytes": tr["dense_bytes"], "traffic": None}
    roof["dense_stream"] = dense
    roof["dense_equivalent"] = {"gbps": round(equiv, 1), "frac": round(equiv / HBM_PEAK_GBPS, 4),
                                "bytes": tr["stream_bytes"],
                                "meaning": "SURVEY s*(2N_i+N_{i+1}) over all merges / wall: the HBM rate a "
                                           "full-stream-per-merge loop would need for this merge rate"}
    return roof


def single_line(args, tr):
    value = tr["merges"] / tr["wall_s"]
    return {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "merges/s",
        "n_gpus": 1,
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
                   "merges_timed": tr["merges"], "early_stop": tr["early_stop"], "parallelism": "single"},
        "roofline": train_roofline(tr),
        "train_detail": tr,
    }


def sharded_line(args, lib, ctx, dist, rank, world):
    data, merges, tr = train_leg_sharded(args, lib, ctx, dist, rank, world)
    value = world * tr["merges"] / tr["wall_s"]
    achieved = tr["stream_bytes"] / 1e9 / tr["wall_s"]
    line = {
        "metric": METRIC,
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
        "data": "synthetic (seeded Zipf English-like corpus per shard, gpubpe.synth)",
        "config": {"workload": f"C2 x {world}: one global 32K-vocab BPE train over {world} shards of "
                               f"{args.train_bytes:,} B English UTF-8 (seeds 2..{1 + world}), heuristic word "
                               "boundaries, reference compaction, bit-exact to one stream; value = shard-merges/s "
                               "(global merges x shards / wall); step = 128 merges",
                   "train_bytes_per_rank": args.train_bytes, "target_vocab": args.vocab,
                   "merges_timed": tr["merges"], "early_stop": tr["early_stop"],
                   "parallelism": f"shard{world} ({tr['transport']} all-gather per merge)"},
        "roofline": {
            "bound": "hbm",
            "kernel": "whole sharded loop (algorithmic stream bytes of all ranks / wall)",
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS * world, "unit": "GB/s",
            "frac": round(achieved / (HBM_PEAK_GBPS * world), 4),
            "algorithmic_bytes": tr["stream_bytes"], "traffic": None,
        },
        "train_detail": tr,
    }
    if rank == 0 and not args.no_parity:
        # the first merges equal a single-GPU run on the concatenated corpus
        full = b"".join(shard_corpus(args, r) for r in range(world))
        k = min(128, len(merges))
        g = first_merges(lib, ctx, full, args.vocab, k)
        line["parity"] = {"sharded_vs_single_stream_first_merges_equal": g == merges[:k], "merges_checked": k}
    return line, data


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
    ap.add_argument("--no-parity", action="store_true", help="N>1: skip the single-stream parity check")
    ap.add_argument("--sharded", action="store_true", help="use the sharded trainer even at N=1 (RCCL rehearsal)")
    args = ap.parse_args()

    rank, world, local = dist_env()
    dist = Dist(world, local, force=args.sharded)
    from gpubpe import _lib
    lib = _lib.load()
    ctx = C.c_void_p()
    rc = lib.gbpe_ctx_create(int(os.environ.get("GBPE_BENCH_DEVICE", local)) if world > 1 else 0, C.byref(ctx))
    if rc != 0:
        raise SystemExit(f"gbpe_ctx_create failed ({rc}): no MI355X visible")

    if world > 1 or args.sharded:
        line, data = sharded_line(args, lib, ctx, dist, rank, world)
    else:
        data, tr = train_leg(args, lib, ctx, dist, rank)
        line = single_line(args, tr)

    pmc = os.path.join(ROOT, "profiles", "r1_pmc_kbody.json")
    if world == 1 and not args.sharded and os.path.exists(pmc) and args.train_bytes == 104_857_600 and \
            tr["bytes_per_symbol"] == 2 and "bytes_per_launch" in line["roofline"]:
        # HBM bytes per k_body launch from the committed rocprofv3 --pmc passes
        # (FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction) of this same workload
        p = json.load(open(pmc))
        line["roofline"]["traffic"] = round(p["hbm_bytes_per_launch"])
        line["roofline"]["traffic_unit"] = "bytes/launch (k_body)"
        line["roofline"]["traffic_over_algorithmic"] = round(p["hbm_bytes_per_launch"] / p["algorithmic_bytes_per_launch"], 4)
        line["roofline"]["traffic_sample"] = (f"profiles/r1_pmc_kbody.json: {p['launches']} k_body launches, "
                                              f"FETCH_SIZE and WRITE_SIZE passes")

    enc = None
    if not args.no_encode:
        enc = encode_leg(args, lib, ctx, dist, rank)
        line["tokenize"] = enc[-1]

    if world == 1 and not args.sharded and not args.no_cpu:
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
    if _COMM.get("c"):
        lib.gbpe_comm_destroy(_COMM["c"])
    lib.gbpe_ctx_destroy(ctx)


if __name__ == "__main__":
    main()
