#!/usr/bin/env python3
"""Benchmark: BPE merges/sec (+ tokenize GB/s) on MI355X through the C-ABI.

Headline workload (BASELINE.json metric: "1 GiB UTF-8 @ 32K vocab"): 32K-vocab
BPE training on 1,073,741,824 bytes of synthetic English-like UTF-8 (seed 2,
0.5 % 3-byte punctuation), heuristic word boundaries (train.wgsl:87-186),
reference compaction semantics.  A "step" is one complete training run on the
HBM-resident corpus: trainer creation (symbol widening, word boundaries, the
initial pair count) plus all 32,512 merges (every 128-merge host round trip of
trainer.js:225-335).  `value` = merges of the K timed runs / their wall time.

Secondary legs (same JSON line):
  * c1: BASELINE configs[0] (1K vocab on 256 KiB ASCII, seed 1), full runs, with
    the full 768-merge CPU run on 1 core and on the CPU share beside it;
  * c2: BASELINE configs[1] (100 MiB English, seed 2, 32K vocab), full runs;
  * tokenize (configs[2], C3): chunked trie encode of 1 GiB multilingual text
    with a 32K vocab trained on a 100 MiB sample (seed 4);
  * c4_shard: C4's rank-0 shard (1 GiB multilingual, seed 5) trained alone at
    C4's 64K vocab, u32 symbols, run to the 0xFFFF id stop (configs[3] per rank);
  * ml1g: the metric's "1 GiB UTF-8 @ 32K" on multi-byte text: 1 GiB
    multilingual (seed 3) at 32K vocab, against its fixture;
  * c5: configs[4], 1 GiB code at 50K vocab with GPT-4 rule word starts
    computed on the device (u32 symbols); both against their oracle fixtures;
  * cpu_baseline: the reference algorithm restated on the CPU
    (oracle/bpe_oracle.c: full pair recount every merge), a bounded sample of
    the same workload on the box's CPU share and on 1 core;
  * parity: the timed runs' merge list against the committed oracle fixture
    (tests/golden/train_en1g.npz, all 32,512 merges), the encode tokens against
    the fixture and the CPU restatement.

Multi-GPU (--gpus N under torch.distributed.run, one rank per GPU):
  * training (the default N > 1 line): one 1 GiB corpus, one vocabulary (strong
    scaling: the total work is fixed), cut at word starts into one piece per
    rank; every GPU runs its piece's first pass (symbols, word starts, pair
    counts, word lexicon), the lexicons go to the last rank, which runs the merge
    chain — it is sequential, every merge's argmax needs the previous merge's
    counts, and one merge costs less than an exchange between GPUs; `value` =
    merges / max wall over ranks.  `--replicated` instead runs the complete
    training on every rank (no exchange), reported beside the hand-over anyway;
  * C4 (N = 8): one 64K vocabulary over 8 x 1 GiB multilingual shards through the
    same hand-over, checked after the timed run: the root's live pair counts
    against a device recount of the final stream rebuilt from every rank's
    occurrence list (`counts_equal_recount`);
  * tokenize: the one 1 GiB C3 input cut into chunk-aligned slices, one per rank
    (gpubpe/split_encode.py): GB/s = input bytes / max wall over ranks; the
    tokens are gathered to rank 0 and checked against the fixture.
"""
from __future__ import annotations

import argparse
import ctypes as C
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gpu-bpe_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
# latency constants of MI355X_MICROARCH.md (one lane, idle chip): a dependent global
# load that hits the Infinity Cache (~545 cycles at 2.4 GHz), and a dependent kernel
# boundary on one stream (price list row "boundary")
HOP_US = 0.227
BOUNDARY_US = 1.45
# the dependent global hops of one late sector-sparse merge (DESIGN §8 "latency
# floor"): k_body, then k_refresh, each waits for the one before, and each launch
# waits for the previous one (two kernel boundaries per merge)
KBODY_HOPS = ("state + partial maxima (selection)", "bitmap rows of a and b", "candidate extents + signatures",
              "candidate sector symbols + multiplicities", "pair-table probe (flush)", "count adds landed")
KREFRESH_HOPS = ("dirty flags + state snapshot", "dirty blocks' slots (re-max)", "partial maxima stored")
TILE_SYMS = 8192
METRIC = "BPE merges/sec + tokenize GB/s, 1 GiB UTF-8 @ 32K vocab, 1/2/4/8 MI355X"
HEADLINE = {"gen": "english", "n": 1 << 30, "seed": 2, "fancy_punct": 0.005}
C2 = {"gen": "english", "n": 104_857_600, "seed": 2, "fancy_punct": 0.005}
PMC_FILE = os.path.join(ROOT, "profiles", "r6", "pmc_kbody.json")
ROCPROF_EN1G = os.path.join(ROOT, "profiles", "r6", "en1g_kernel_stats.csv")
ENC_PMC_FILE = os.path.join(ROOT, "profiles", "r6", "pmc_encode.json")
CAL_NOTE = ("FETCH_SIZE x2: tools/micro/fetch_cal.hip measured 64 counter bytes per distinct 128-B line for "
            "16-B streaming reads and 4-, 8- and 16-B one-per-line gathers alike (profiles/r3_fetch_calibration.json), "
            "so every read line moves 128 B; WRITE_SIZE counts 32-B granules (4-B scattered stores and atomics: 32 B "
            "per line, whole-line stores 128 B)")
GOLD = os.path.join(ROOT, "tests", "golden")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_env():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("LOCAL_RANK", "0"))


def make_corpus(spec: dict) -> bytes:
    from gpubpe import synth
    if spec["gen"] == "english":
        return synth.english(spec["n"], seed=spec["seed"], fancy_punct=spec.get("fancy_punct", 0.0))
    if spec["gen"] == "multilingual":
        return synth.multilingual(spec["n"], seed=spec["seed"])
    return synth.code(spec["n"], seed=spec["seed"])


class _stdout_to_stderr:
    """fd 1 -> fd 2 for the duration (native libraries' prints included)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


class Dist:
    """Process groups: the default group carries the lexicon hand-over's data
    path (RCCL = backend "nccl" over xGMI; GBPE_SHARD_TRANSPORT=gloo stages it
    through host memory instead); a gloo group carries the timing scalars."""

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
            with _stdout_to_stderr():   # gloo prints its connection banner on stdout: keep stdout the one JSON line
                if self.transport == "nccl":
                    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
                else:
                    dist.init_process_group("gloo")
                self.dist = dist
                self.host = dist.new_group(backend="gloo")
                self.dist.barrier(group=self.host)   # (the gloo pairs connect here)

    def barrier(self):
        if hasattr(self, "host"):
            self.dist.barrier(group=self.host)

    def _reduce(self, x: float, op) -> float:
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=op, group=self.host)
        return float(t.item())

    def max(self, x: float) -> float:
        return x if self.world == 1 else self._reduce(x, self.dist.ReduceOp.MAX)

    def sum(self, x: float) -> float:
        return x if self.world == 1 else self._reduce(x, self.dist.ReduceOp.SUM)


def device_buffer(lib, ctx, data: bytes):
    from gpubpe import _lib
    p = C.c_void_p()
    _lib.check(lib.gbpe_device_alloc(ctx, len(data) + 64, C.byref(p)), ctx, "alloc")
    _lib.check(lib.gbpe_memcpy_h2d(ctx, p, data, len(data)), ctx, "h2d")
    return p


def train_run(lib, ctx, d_bytes, n, vocab, flags=0, max_merges=0, batch=128, pairs_out=None, steps_out=None):
    """One training run on HBM-resident bytes: create + every step.  Returns
    (merges [k, 4] uint32, stats).  pairs_out (a list): the live pair ids at the
    end are appended to it (the reference-table estimate; never in a timed run).
    steps_out (a list): (merges, seconds) of every step call is appended to it."""
    from gpubpe import _lib
    opts = _lib.TrainOpts(target_vocab_size=vocab, vocab_size=256, next_token_id=256, batch_size=batch,
                          flags=flags, table_log2=0)
    tr = C.c_void_p()
    _lib.check(lib.gbpe_trainer_create(ctx, d_bytes, n, None, 1, C.byref(opts), C.byref(tr)), ctx, "trainer_create")
    out = (C.c_uint32 * (4 * batch))()
    merges = []
    try:
        while True:
            k = batch if not max_merges else min(batch, max_merges - len(merges) // 4)
            nd, es = C.c_uint32(), C.c_uint32()
            ts = time.perf_counter()
            _lib.check(lib.gbpe_trainer_step(tr, k, out, C.byref(nd), C.byref(es)), ctx, "trainer_step")
            if steps_out is not None:
                steps_out.append((nd.value, time.perf_counter() - ts))
            merges += out[: 4 * nd.value]
            if nd.value == 0 or es.value or (max_merges and len(merges) // 4 >= max_merges):
                break
        st = _lib.TrainerStats()
        lib.gbpe_trainer_stats_get(tr, C.byref(st))
        if pairs_out is not None:
            cnt = C.c_uint64()
            lib.gbpe_trainer_pair_counts(tr, None, None, 0, C.byref(cnt))
            pids = np.zeros(max(1, cnt.value), np.uint32)
            cts = np.zeros(max(1, cnt.value), np.uint32)
            _lib.check(lib.gbpe_trainer_pair_counts(tr, pids.ctypes.data_as(_lib.u32p), cts.ctypes.data_as(_lib.u32p),
                                                    cnt.value, C.byref(cnt)), ctx, "pair_counts")
            pairs_out.append(pids[: cnt.value])
    finally:
        lib.gbpe_trainer_destroy(tr)
    return np.array(merges, dtype=np.uint32).reshape(-1, 4), st


def fixture(name: str):
    p = os.path.join(GOLD, f"train_{name}.npz")
    if not os.path.exists(p):
        return None, None
    z = np.load(p, allow_pickle=False)
    return z["merges"], json.loads(str(z["meta"]))


def timed_runs(args, lib, ctx, dist, d, n, vocab, steps, warmup, flags=0, pairs_out=None):
    """W untimed + K timed full runs, barrier + sync on both sides of the timed ones
    (the last untimed run also hands its final live pairs to pairs_out)."""
    for w in range(warmup):
        train_run(lib, ctx, d, n, vocab, flags=flags, pairs_out=pairs_out if w == warmup - 1 else None)
    lib.gbpe_synchronize(ctx)
    dist.barrier()
    lib.gbpe_synchronize(ctx)
    t0 = time.perf_counter()
    total, last, st, create_s, run_s = 0, None, None, 0.0, []
    for _ in range(steps):
        tr0 = time.perf_counter()
        last, st = train_run(lib, ctx, d, n, vocab, flags=flags)   # (its last step call synchronises)
        run_s.append(round(time.perf_counter() - tr0, 4))
        total += last.shape[0]
        create_s += st.ms_create / 1e3
    lib.gbpe_synchronize(ctx)
    t1 = time.perf_counter()
    dist.barrier()
    st.create_s_total = create_s   # (the timed runs' trainer creation, host wall)
    st.run_s = run_s               # (each timed run's host wall, this rank)
    log(f"[bench] timed runs (s): {run_s}")
    return dist.max(t1 - t0), total, last, st


def ref_table(st, pairs):
    """the reference's 2^21-slot table against this run's pair sets."""
    from gpubpe import reftable
    return reftable.report(int(st.max_live_pairs), pairs[0] if pairs else None)


def train_detail(st, sk):
    """Per-run stats of a timed run (st) and of the HIP-event run (sk)."""
    return {
        "final_symbols": int(st.symbol_count), "bytes_per_symbol": int(st.bytes_per_symbol),
        "stream_bytes": int(st.stream_bytes_moved), "tail_dropped": int(st.tail_dropped),
        "max_live_pairs": int(st.max_live_pairs), "table_slots": int(st.table_slots),
        "sparse": {"merges": int(st.sparse_merges), "enters": int(st.sparse_enters), "exits": int(st.sparse_exits),
                   "sectors": int(st.sparse_sectors), "zone_at_entry": int(st.sparse_zone),
                   "paired_merges": int(getattr(st, "paired_merges", 0))},
        "ms_create": round(st.ms_create, 3),
        "run_s": getattr(st, "run_s", None),
        "events": None if sk is None else {
            "merges": int(sk.timed_merges), "dense_merges": int(sk.timed_merges - sk.sparse_merges),
            "dense_bytes": int(sk.dense_bytes), "ms_dense": sk.ms_dense,
            "sparse_merges": int(sk.sparse_merges), "paired_merges": int(getattr(sk, "paired_merges", 0)),
            "body_bytes": int(sk.body_bytes), "zone_bytes": int(sk.zone_bytes),
            "ms_body": sk.ms_body, "ms_sparse": sk.ms_sparse, "ms_select": sk.ms_select, "ms_refresh": sk.ms_other,
            "ms_delta": sk.ms_delta, "ms_compact": sk.ms_compact},
    }


def _rocprof_kernel(prefix: str):
    """(calls, total ns) of the kernels whose name starts with `prefix` in the
    committed rocprofv3 --stats summary of one full headline run."""
    import csv
    calls, ns = 0, 0.0
    if os.path.exists(ROCPROF_EN1G):
        for r in csv.DictReader(open(ROCPROF_EN1G)):
            name = r["Name"].replace("void ", "", 1).replace("(anonymous namespace)::", "")
            if name.startswith(prefix):
                calls += int(r["Calls"])
                ns += float(r["TotalDurationNs"])
    return calls, ns


def train_roofline(det, wall_per_run):
    """Roofline of the dominant training kernel from the HIP-event run.

    The sparse merges run in k_body, one launch per merge.  Each kernel's bytes are the ones it moves (candidate extents and signatures,
    sector symbols read and rewritten, the zone pass) — pair-table traffic
    excluded as in SURVEY §8(d).  The kernel with the larger share of the run's
    device time is the roofline kernel; the other is reported beside it.  The
    SURVEY formula over the whole run and its wall time is given as the bandwidth
    a stream-per-merge loop would need to match this merge rate (not credited)."""
    ev = det["events"]
    dense = None
    if ev and ev["ms_dense"] > 0:
        a = ev["dense_bytes"] / 1e9 / (ev["ms_dense"] / 1e3)
        dense = {"kernel": "k_delta + k_compact (dense merges)", "merges": ev["dense_merges"], "achieved": round(a, 1),
                 "frac": round(a / HBM_PEAK_GBPS, 4), "algorithmic_bytes": ev["dense_bytes"],
                 "ms": round(ev["ms_dense"], 2)}
    equiv = det["stream_bytes"] / 1e9 / wall_per_run

    def kern(name, byts, ms, launches, merges, prefix, desc):
        if not ev or ms <= 0 or launches <= 0:
            return None
        a = byts / 1e9 / (ms / 1e3)
        k = {"bound": "hbm", "kernel": desc, "achieved": round(a, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
             "frac": round(a / HBM_PEAK_GBPS, 4), "traffic": None,
             "algorithmic_bytes_per_launch": round(byts / launches), "us_per_launch": round(1e3 * ms / launches, 2),
             "launches": launches, "merges": merges, "ms_per_run": round(ms, 2),
             "timing": "HIP events around every launch of one extra full run of the same workload (events add "
                       "inter-kernel gaps, so they stay out of the timed runs)"}
        calls, ns = _rocprof_kernel(prefix)
        if calls:
            k["rocprof_us_per_launch"] = round(ns / calls / 1e3, 2)
            k["rocprof_launches"] = calls
            k["rocprof_achieved_with_rocprof_time"] = round(k["algorithmic_bytes_per_launch"] / (ns / calls), 1)
            k["rocprof_window"] = os.path.relpath(ROCPROF_EN1G, ROOT)
            k["rocprof_note"] = ("from a run under rocprofv3 --kernel-trace, which runs a few percent slower than the "
                                 "untraced timed runs (kernel-busy time above the untraced wall), so these per-launch "
                                 "times are slightly inflated")
        return k

    body = kern("body", ev["body_bytes"], ev["ms_body"], ev["sparse_merges"] - ev.get("paired_merges", 0),
                ev["sparse_merges"], "k_body<",
                "k_body (sector-sparse merge pass over the word lexicon, one launch per merge or two: paired "
                "launches, DESIGN §2f)") if ev else None
    cand = [k for k in (body,) if k]
    roof = max(cand, key=lambda k: k["ms_per_run"]) if cand else {
        "bound": "hbm", "kernel": None, "achieved": None, "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": None,
        "traffic": None}
    roof = dict(roof)
    roof["note"] = ("latency-bound by design: the body is one copy of every distinct word (DESIGN §2c), so a merge "
                    "moves the few sectors holding its pair, kilobytes, not the stream; the loop avoids the bytes "
                    "rather than streaming them")
    other = [k for k in cand if k["kernel"] != roof.get("kernel")]
    if other:
        roof["other_kernel"] = other[0]
    # latency floor: a late merge is a chain of dependent round
    # trips, not bytes; the floor counts them at the guide's idle-chip latencies
    floor_kernel = len(KBODY_HOPS) * HOP_US
    floor_merge = (len(KBODY_HOPS) + len(KREFRESH_HOPS)) * HOP_US + 2 * BOUNDARY_US
    lf = {"k_body_hops": list(KBODY_HOPS), "k_refresh_hops": list(KREFRESH_HOPS), "hop_us": HOP_US,
          "boundary_us": BOUNDARY_US, "k_body_us": round(floor_kernel, 3), "us_per_merge": round(floor_merge, 3),
          "meaning": "dependent Infinity-Cache round trips (~545 cycles each) of one late merge — k_body's and "
                     "k_refresh's — plus two kernel boundaries; achieved / floor says how far the chain is from its "
                     "own bound, as frac does for bytes"}
    if roof.get("us_per_launch"):
        lf["k_body_achieved_us"] = roof["us_per_launch"]
        lf["k_body_achieved_over_floor"] = round(roof["us_per_launch"] / floor_kernel, 2)
    if det.get("late_window"):
        w = det["late_window"]
        lf["late_window"] = w
        lf["late_achieved_over_floor"] = round(w["us_per_merge"] / floor_merge, 2)
    roof["latency_floor"] = lf
    roof["dense_stream"] = dense
    roof["dense_equivalent"] = {"gbps": round(equiv, 1), "frac": round(equiv / HBM_PEAK_GBPS, 4),
                                "bytes": det["stream_bytes"],
                                "meaning": "SURVEY s*(2N_i+N_{i+1}) over all merges / wall per run: the HBM rate a "
                                           "full-stream-per-merge loop would need for this merge rate"}
    if os.path.exists(PMC_FILE):
        p = json.load(open(PMC_FILE))
        kn = (roof.get("kernel") or "").split(" ")[0]
        if p.get("workload") == "en1g-full-run" and p.get("kernel", "k_body") == kn:
            roof["traffic"] = round(p["hbm_bytes_per_launch"])
            roof["traffic_unit"] = f"bytes/launch ({kn})"
            roof["traffic_over_algorithmic"] = round(p["traffic_over_algorithmic"], 4)
            roof["traffic_window"] = (f"{os.path.relpath(PMC_FILE, ROOT)}: rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and "
                                      f"WRITE_SIZE passes over one full run of this workload ({p['launches']} {kn} "
                                      f"launches); algorithmic bytes from the same run")
            roof["traffic_calibration"] = CAL_NOTE
    return roof


def single_gpu_roofline(args, lib, ctx, d, n):
    """The N = 1 line's roofline on this GPU (N > 1 lines, rank 0): one HIP-event
    run and one per-step-timed run of the headline workload."""
    from gpubpe import _lib
    _, sk = train_run(lib, ctx, d, n, args.vocab, flags=_lib.GBPE_TRAIN_TIMING)
    steps = []
    t0 = time.perf_counter()
    last, st = train_run(lib, ctx, d, n, args.vocab, steps_out=steps)
    wall = time.perf_counter() - t0
    det = train_detail(st, sk)
    done, late_m, late_s = 0, 0, 0.0
    for m, sec in steps:
        if done >= 16384:
            late_m += m
            late_s += sec
        done += m
    if late_m:
        det["late_window"] = {"merges_from": 16384, "merges": late_m, "us_per_merge": round(1e6 * late_s / late_m, 3)}
    roof = train_roofline(det, wall)
    roof["measured"] = "rank 0 of this run, alone on its GPU: one HIP-event run and one step-timed run of the headline"
    return roof


def headline_leg(args, lib, ctx, dist):
    t = time.time()
    data = make_corpus(HEADLINE)
    log(f"[bench] headline corpus {len(data)} B generated in {time.time() - t:.1f}s")
    d = device_buffer(lib, ctx, data)
    n = len(data)
    pairs = []
    wall, total, last, st = timed_runs(args, lib, ctx, dist, d, n, args.vocab, args.steps, args.warmup,
                                       pairs_out=pairs)
    sk = None
    if not args.no_kernel_timing:
        from gpubpe import _lib
        _, sk = train_run(lib, ctx, d, n, args.vocab, flags=_lib.GBPE_TRAIN_TIMING)
    steps = []   # one more untimed run with per-step host walls: the late-merge window's cost per merge
    train_run(lib, ctx, d, n, args.vocab, steps_out=steps)
    lib.gbpe_device_free(ctx, d)
    det = train_detail(st, sk)
    det["reference_rate"] = {
        "value": round(total / (wall - st.create_s_total), 1), "unit": "merges/s",
        "create_ms_per_run": round(1e3 * st.create_s_total / max(1, args.steps), 3),
        "definition": "the reference's merges/s = merges / t_loop (trainer.js:230, 291-292, 324-326): the timed "
                      "wall minus trainer creation (symbols, word starts and the first pair count); t_loop excludes "
                      "the symbols and word starts but includes the first count (every reference merge recounts, "
                      "training-pipeline.js:190), so this rate is an upper bound of the reference definition by the "
                      "first count's share of create_ms_per_run (~1.2 ms); `value` keeps all of creation inside"}
    done, late_m, late_s = 0, 0, 0.0
    for m, sec in steps:
        if done >= 16384:
            late_m += m
            late_s += sec
        done += m
    if late_m:
        det["late_window"] = {"merges_from": 16384, "merges": late_m, "us_per_merge": round(1e6 * late_s / late_m, 3),
                              "timing": "host wall of every gbpe_trainer_step call (128 merges, one sync) of one "
                                        "untimed run"}
    # SURVEY §8(d) N_i: the stream length before each merge, logged per 128-merge step
    n_i = n - np.concatenate([[0], np.cumsum(last[:, 3].astype(np.int64))])
    det["n_i_per_step"] = {"every": 128, "values": [int(v) for v in n_i[::128]], "final": int(n_i[-1])}
    det["reference_table"] = ref_table(st, pairs)
    det["merges_per_run"] = int(last.shape[0])
    det["last_merge"] = last[-1].tolist() if last.shape[0] else []
    parity = {}
    want, meta = fixture("en1g")
    if want is not None and args.vocab == 32768:
        parity["train_fixture"] = "tests/golden/train_en1g.npz (oracle/bpe_oracle_inc.c)"
        parity["train_corpus_sha256_equal"] = hashlib.sha256(data).hexdigest() == meta["corpus_sha256"]
        parity["train_merges_equal_fixture"] = bool(last.shape == want.shape and np.array_equal(last, want))
        parity["train_merges_checked"] = int(want.shape[0])
        parity["train_final_symbols_equal"] = int(st.symbol_count) == meta["final_n"]
    return data, wall, total, last, det, parity


def c2_leg(args, lib, ctx, dist):
    data = make_corpus(C2)
    d = device_buffer(lib, ctx, data)
    pairs = []
    wall, total, last, st = timed_runs(args, lib, ctx, dist, d, len(data), args.vocab, 3, 1, pairs_out=pairs)
    lib.gbpe_device_free(ctx, d)
    want, _ = fixture("c2")
    res = {"workload": "C2 (BASELINE configs[1]): 32K-vocab train on 104,857,600 B English UTF-8 (seed 2), full runs",
           "value": round(total / wall, 1), "unit": "merges/s", "runs": 3, "merges_per_run": int(last.shape[0]),
           "ms_per_run": round(1e3 * wall / 3, 2), "reference_table": ref_table(st, pairs)}
    if want is not None:
        res["merges_equal_fixture"] = bool(last.shape == want.shape and np.array_equal(last, want))
    if not args.no_cpu:
        # the stronger CPU comparator: the whole C2 run by the
        # incremental restatement of the reference algorithm (the fixtures' generator)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import cpu_ref
        t0 = time.perf_counter()
        r = cpu_ref.train_inc(data, args.vocab, want_symbols=False)
        dt = time.perf_counter() - t0
        m = np.array(r["merges"], dtype=np.uint32).reshape(-1, 4)
        res["cpu_incremental"] = {
            "value": round(m.shape[0] / dt, 1), "unit": "merges/s", "seconds": round(dt, 2), "cores": 1,
            "kind": "port", "merges": int(m.shape[0]),
            "sample": "the whole C2 run (32,512 merges), incremental restatement (oracle/bpe_oracle_inc.c: linked-list "
                      "stream, per-pair occurrence lists, lazy max-heap), one thread",
            "merges_equal_fixture": bool(want is not None and m.shape == want.shape and np.array_equal(m, want)),
            "gpu_over_cpu": round((total / wall) / (m.shape[0] / dt), 1)}
    return data, res


def config_leg(args, lib, ctx, dist, name, data, vocab, flags, workload, runs=2):
    """A secondary training configuration on its own fixture's corpus: 1 untimed +
    `runs` timed full runs, every merge of the last one checked against the fixture."""
    want, meta = fixture(name)
    d = device_buffer(lib, ctx, data)
    pairs = []
    wall, total, last, st = timed_runs(args, lib, ctx, dist, d, len(data), vocab, runs, 1, flags, pairs_out=pairs)
    lib.gbpe_device_free(ctx, d)
    res = {"workload": workload, "value": round(total / wall, 1), "unit": "merges/s", "runs": runs,
           "merges_per_run": int(last.shape[0]), "ms_per_run": round(1e3 * wall / runs, 2),
           "bytes_per_symbol": int(st.bytes_per_symbol), "early_stop": bool(st.early_stop),
           "sparse": {"enters": int(st.sparse_enters), "exits": int(st.sparse_exits),
                      "dense_merges": int(st.merges_done - st.sparse_merges),
                      "lexicon_builds": int(st.lexicon_builds), "lexicon_fallbacks": int(st.lexicon_fallbacks)},
           "reference_table": ref_table(st, pairs)}
    if want is not None:
        res["corpus_sha256_equal"] = hashlib.sha256(data).hexdigest() == meta["corpus_sha256"]
        res["merges_equal_fixture"] = bool(last.shape == want.shape and np.array_equal(last, want))
        res["fixture"] = f"tests/golden/train_{name}.npz"
    return res


def c1_leg(args, lib, ctx, dist):
    """C1 (BASELINE configs[0]): 1K vocab on 256 KiB ASCII English (seed 1), 768
    merges, heuristic word boundaries.  GPU: full runs on HBM-resident input,
    every merge checked against tests/golden/train_c1.npz.  CPU (BASELINE.md's
    plan): the same full run by the reference algorithm restated on the host
    (oracle/bpe_oracle.c, full recount per merge) on 1 core and on the CPU share.
    The reference itself needs a WebGPU adapter; none exists on the box
    (profiles/r3_webgpu_probe.txt: no Vulkan ICD, Dawn, wgpu or browser)."""
    want, meta = fixture("c1")
    data = make_corpus({"gen": "english", "n": 262_144, "seed": 1})
    d = device_buffer(lib, ctx, data)
    runs = 20
    wall, total, last, st = timed_runs(args, lib, ctx, dist, d, len(data), 1024, runs, 2)
    lib.gbpe_device_free(ctx, d)
    res = {"workload": "C1 (BASELINE configs[0]): 1K-vocab train on 262,144 B ASCII English (seed 1), 768 merges, "
                       "heuristic word boundaries, reference compaction; full runs on the HBM-resident corpus",
           "value": round(total / wall, 1), "unit": "merges/s", "runs": runs, "merges_per_run": int(last.shape[0]),
           "ms_per_run": round(1e3 * wall / runs, 3),
           "webgpu_reference": "not runnable: no WebGPU implementation on the box (profiles/r3_webgpu_probe.txt)"}
    if want is not None:
        res["corpus_sha256_equal"] = hashlib.sha256(data).hexdigest() == meta["corpus_sha256"]
        res["merges_equal_fixture"] = bool(last.shape == want.shape and np.array_equal(last, want))
        res["fixture"] = "tests/golden/train_c1.npz"
    if not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import cpu_ref
        share = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
        cpu = {}
        for cores in (1, share):
            t0 = time.perf_counter()
            r = cpu_ref.train(data, 1024, threads=cores, want_symbols=False)
            dt = time.perf_counter() - t0
            cpu[str(cores)] = {"merges_per_s": round(len(r["merges"]) / dt, 1), "seconds": round(dt, 3),
                               "merges_equal_fixture": bool(want is not None and np.array_equal(
                                   np.array(r["merges"], dtype=np.uint32), want))}
        res["cpu_baseline"] = {"kind": "port", "sample": "the full 768-merge run, full pair recount per merge "
                                                         "(oracle/bpe_oracle.c, OpenMP)", "cores": cpu,
                               "nproc": os.cpu_count()}
    return res


def encode_leg(args, lib, ctx, dist, rank):
    """C3: train a 32K vocab on a 100 MiB multilingual sample (seed 4), then
    encode 1 GiB multilingual text (seed 3) with the chunked trie walk."""
    from gpubpe import _lib, compile_vocab_to_trie, parse_header, parse_trie_buffers
    from gpubpe.vocab import Vocab
    t = time.time()
    sample = make_corpus({"gen": "multilingual", "n": args.vocab_sample_bytes, "seed": 4})
    d = device_buffer(lib, ctx, sample)
    merges, _ = train_run(lib, ctx, d, len(sample), args.vocab)
    lib.gbpe_device_free(ctx, d)
    voc = Vocab()
    for a, b in merges[:, :2].tolist():
        voc.add_merge(a, b)
    blob = compile_vocab_to_trie(voc.entries)
    hdr = parse_header(blob)
    nodes, edges = parse_trie_buffers(blob, hdr)
    log(f"[bench] C3 vocab {voc.size} tokens, trie {hdr['nodeCount']} nodes in {time.time() - t:.1f}s")
    t = time.time()
    text = make_corpus({"gen": "multilingual", "n": args.encode_bytes, "seed": 3})
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
    reps = 5
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
    e2e = []
    for _ in range(2):
        t0 = time.perf_counter()
        _lib.check(lib.gbpe_encode(ctx, trie, text, n, cs, host_out.ctypes.data_as(_lib.u32p), n, C.byref(n_out)),
                   ctx, "encode e2e")
        e2e.append(time.perf_counter() - t0)
    tokens = host_out[: n_out.value]
    lib.gbpe_device_free(ctx, d_in)
    lib.gbpe_device_free(ctx, d_out)
    lib.gbpe_trie_free(trie)
    alg = n + 4 * T
    res = {
        "workload": "C3: chunked greedy trie encode of 1,073,741,824 B multilingual UTF-8 (seed 3), 32K vocab "
                    f"trained on the GPU on a {args.vocab_sample_bytes} B sample (seed 4), chunk {cs}",
        "bytes": n, "tokens": T, "chunk_size": cs, "trie_nodes": int(hdr["nodeCount"]),
        "trie_records": int(nrec.value),
        "gbps_kernels": round(n / 1e9 / (k_all / 1e3), 2),
        "gbps_device_wall": round(n / 1e9 / wall, 2),
        "gbps_end_to_end": round(n / 1e9 / min(e2e), 2),
        "ms_walk": round(k_walk, 3), "ms_scan": round(float(np.mean([k[1] for k in kms])), 3),
        "ms_compact": round(float(np.mean([k[2] for k in kms])), 3),
        "roofline": {"bound": "hbm", "kernel": "encode kernels (walk + scan + compact), n + 4T bytes",
                     "achieved": round(alg / 1e9 / (k_all / 1e3), 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(alg / 1e9 / (k_all / 1e3) / HBM_PEAK_GBPS, 4), "algorithmic_bytes": alg,
                     "traffic": None},
    }
    pmc = ENC_PMC_FILE
    if os.path.exists(pmc):
        p = json.load(open(pmc))
        if p.get("workload") == "c3-1g" and p.get("chunk_size", cs) == cs:
            res["roofline"]["traffic"] = round(p["hbm_bytes_per_encode"])
            res["roofline"]["traffic_unit"] = "bytes/encode (all encode kernels)"
            res["roofline"]["traffic_over_algorithmic"] = round(p["hbm_bytes_per_encode"] / alg, 4)
            res["roofline"]["traffic_window"] = f"{os.path.relpath(pmc, ROOT)}: FETCH_SIZE (x2) + WRITE_SIZE passes"
            res["roofline"]["traffic_calibration"] = CAL_NOTE
    fx = os.path.join(GOLD, "encode_c3enc1g.json")
    if os.path.exists(fx) and args.encode_bytes == 1 << 30 and args.vocab_sample_bytes == 104_857_600:
        meta = json.load(open(fx))
        res["fixture_tokens_equal"] = (T == meta["n_tokens"] and
                                       hashlib.sha256(np.ascontiguousarray(tokens, "<u4").tobytes()).hexdigest()
                                       == meta["tokens_sha256"])
    return text, nodes, edges, cs, tokens, res


def cpu_baselines(args, data, enc):
    """The reference algorithm on the host (oracle/bpe_oracle.c, 'port'): first K
    merges of the SAME headline corpus, full pair recount per merge, on the box's
    CPU share (OMP_NUM_THREADS, 16 per GPU on the pool) and on 1 core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_ref
    share = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    nproc = os.cpu_count()
    out = {}
    for cores, k in ((share, args.cpu_merges or 24), (1, max(1, (args.cpu_merges or 24) // 12))):
        t = time.perf_counter()
        r = cpu_ref.train(data, args.vocab, max_merges=k, threads=cores, want_symbols=False)
        dt = time.perf_counter() - t
        out[cores] = (len(r["merges"]) / dt, r["merges"], dt)
    v, merges, dt = out[share]
    base = {"value": round(v, 3), "unit": "merges/s", "cores": share, "kind": "port",
            "sample": f"first {len(merges)} merges of the same 1 GiB corpus, full pair recount per merge (reference "
                      f"algorithm, oracle/bpe_oracle.c, OpenMP), {dt:.1f}s",
            "nproc": nproc, "cpu_share": share,
            "one_core": {"value": round(out[1][0], 4), "merges": len(out[1][1]), "seconds": round(out[1][2], 1)},
            "note": "early merges are the most expensive for a full recount (the stream is longest), so this is a "
                    "lower bound of the whole-run CPU rate; it is a baseline, not a target"}
    enc_base = None
    if enc is not None:
        text, nodes, edges, cs, tokens, er = enc
        t = time.perf_counter()
        ref_tokens = cpu_ref.encode(text, nodes, edges, cs, threads=share)
        dt = time.perf_counter() - t
        enc_base = {"value": round(len(text) / 1e9 / dt, 3), "unit": "GB/s", "cores": share, "kind": "port",
                    "sample": f"full {len(text)} B encode, chunked greedy trie walk (oracle/bpe_oracle.c), {dt:.1f}s",
                    "nproc": nproc, "tokens_equal": bool(np.array_equal(tokens, ref_tokens))}
    return base, merges, enc_base


def single_line(args, lib, ctx, dist, rank):
    data, wall, total, last, det, parity = headline_leg(args, lib, ctx, dist)
    value = total / wall
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "merges/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * wall / max(1, args.steps), 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": f"u{8 * det['bytes_per_symbol']}",
        "data": "synthetic (seeded Zipf English-like corpus, gpubpe.synth)",
        "config": {"workload": "headline: 32K-vocab BPE train on 1,073,741,824 B English-like UTF-8 (seed 2, 0.5% "
                               "3-byte punctuation), heuristic word boundaries, reference compaction; step = one "
                               "complete training run (trainer creation + all 32,512 merges) on the HBM-resident "
                               "corpus",
                   "train_bytes": HEADLINE["n"], "target_vocab": args.vocab,
                   "merges_per_step": det["merges_per_run"], "parallelism": "single"},
        "roofline": train_roofline(det, wall / max(1, args.steps)),
        "reference_rate": det["reference_rate"],
        "train_detail": det,
        "parity": parity,
    }
    if not args.no_c1:
        line["c1"] = c1_leg(args, lib, ctx, dist)
    if not args.no_c2:
        _, line["c2"] = c2_leg(args, lib, ctx, dist)
    enc = None
    if not args.no_encode:
        enc = encode_leg(args, lib, ctx, dist, rank)
        line["tokenize"] = enc[-1]
    if not args.no_c4:
        t = time.time()
        shard = make_corpus({"gen": "multilingual", "n": 1 << 30, "seed": 5})
        log(f"[bench] C4 shard {len(shard)} B generated in {time.time() - t:.1f}s")
        line["c4_shard"] = config_leg(
            args, lib, ctx, dist, "ml1g64k", shard, 65536, 0,
            "C4 rank-0 shard alone: 64K-vocab train on 1,073,741,824 B multilingual UTF-8 (seed 5; C4 = 8 such "
            "shards, seed 5 + rank), u32 symbols, run to the 0xFFFF id stop")
        del shard
    if not args.no_ml1g:   # the metric's "1 GiB UTF-8" on multi-byte text
        t = time.time()
        ml = make_corpus({"gen": "multilingual", "n": 1 << 30, "seed": 3})
        log(f"[bench] ml1g corpus {len(ml)} B generated in {time.time() - t:.1f}s")
        line["ml1g"] = config_leg(
            args, lib, ctx, dist, "ml1g", ml, 32768, 0,
            "ml1g: 32K-vocab train on 1,073,741,824 B multilingual UTF-8 (seed 3: Latin/English, Turkish, Cyrillic, "
            "CJK, Arabic, emoji paragraphs), heuristic word boundaries, u16 symbols", runs=max(2, args.steps // 2))
        del ml
    if not args.no_c5:
        from gpubpe import _lib
        t = time.time()
        code = make_corpus({"gen": "code", "n": 1 << 30, "seed": 6})
        log(f"[bench] C5 corpus {len(code)} B generated in {time.time() - t:.1f}s")
        line["c5"] = config_leg(args, lib, ctx, dist, "code1g", code, 50000, _lib.GBPE_TRAIN_GPT4_BOUNDARIES,
                                "C5: 50K-vocab train on 1,073,741,824 B code (seed 6), GPT-4 rule word starts "
                                "computed on the device, u32 symbols")
        del code
    if not args.no_cpu:
        base, cpu_merges, enc_base = cpu_baselines(args, data, enc)
        line["cpu_baseline"] = base
        line["parity"]["train_cpu_first_merges_equal"] = cpu_merges == last[: len(cpu_merges)].tolist()
        if enc_base is not None:
            line["tokenize"]["cpu_baseline"] = enc_base
    return line


# ── multi-GPU: strong scaling over one corpus ──────────────────────────────────

def shard_of(data: bytes, rank: int, world: int) -> bytes:
    """Rank r's contiguous slice of the corpus, cut right after a newline (a word
    start under the reference heuristic: train.wgsl:166-170), so pair counts add
    up across ranks and the concatenation is the original stream."""
    n = len(data)
    arr = np.frombuffer(data, dtype=np.uint8)
    nl = np.flatnonzero(arr == 0x0A)
    cuts = [0]
    for r in range(1, world):
        k = int(np.searchsorted(nl, n * r // world))
        cuts.append(max(cuts[-1], int(nl[k]) + 1 if k < nl.shape[0] else n))
    cuts.append(n)
    return data[cuts[rank]:cuts[rank + 1]]


def c3_vocab_trie(args, lib, ctx):
    """The C3 vocabulary (32K, trained on the GPU on the 100 MiB multilingual
    sample, seed 4), compiled to the reference trie and uploaded."""
    from gpubpe import _lib, compile_vocab_to_trie, parse_header, parse_trie_buffers
    from gpubpe.vocab import Vocab
    sample = make_corpus({"gen": "multilingual", "n": args.vocab_sample_bytes, "seed": 4})
    d = device_buffer(lib, ctx, sample)
    merges, _ = train_run(lib, ctx, d, len(sample), args.vocab)
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
    return trie, max(512, min(2048, hdr["maxTokenLen"] * 8))   # tokenizer.js:67-68


def split_encode_leg(args, lib, ctx, dist, rank, world):
    """C3 at N ranks: one 1 GiB input, chunk-aligned slice per rank."""
    import torch
    from gpubpe import _lib
    from gpubpe.split_encode import slice_bounds
    trie, cs = c3_vocab_trie(args, lib, ctx)
    text = make_corpus({"gen": "multilingual", "n": args.encode_bytes, "seed": 3})
    n = len(text)
    s0, e0 = slice_bounds(n, cs, world)[rank]
    part = text[s0:e0]
    d_in = device_buffer(lib, ctx, part)
    d_out = C.c_void_p()
    _lib.check(lib.gbpe_device_alloc(ctx, 4 * len(part) + 64, C.byref(d_out)), ctx, "alloc out")
    n_out = C.c_uint64()
    _lib.check(lib.gbpe_encode_device(ctx, trie, d_in, len(part), cs, d_out, len(part), C.byref(n_out)), ctx, "warm")
    reps = 5
    lib.gbpe_synchronize(ctx)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        _lib.check(lib.gbpe_encode_device(ctx, trie, d_in, len(part), cs, d_out, len(part), C.byref(n_out)), ctx, "enc")
    lib.gbpe_synchronize(ctx)
    wall = dist.max((time.perf_counter() - t0) / reps)
    dist.barrier()
    local = np.empty(int(n_out.value), dtype=np.uint32)
    if local.shape[0]:
        _lib.check(lib.gbpe_memcpy_d2h(ctx, local.ctypes.data_as(C.c_void_p), d_out, 4 * local.shape[0]), ctx, "d2h")
    lib.gbpe_device_free(ctx, d_in)
    lib.gbpe_device_free(ctx, d_out)
    lib.gbpe_trie_free(trie)
    # gather: slice totals (exclusive scan -> offsets), then the tokens to rank 0
    dev = "cuda" if dist.transport == "nccl" else "cpu"
    cnt = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.dist.all_gather(cnt, torch.tensor([local.shape[0]], dtype=torch.int64, device=dev))
    counts = [int(c.item()) for c in cnt]
    cap = max(counts)
    buf = torch.zeros(cap, dtype=torch.int32, device=dev)
    buf[: local.shape[0]] = torch.from_numpy(local.view(np.int32)).to(dev)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.dist.all_gather(parts, buf)
    res = {"workload": f"C3 split over {world} ranks: chunked greedy trie encode of one 1,073,741,824 B multilingual "
                       f"UTF-8 input (seed 3), chunk-aligned slices (chunk {cs}), 32K vocab",
           "bytes": n, "tokens": int(sum(counts)), "chunk_size": cs, "gbps_kernels_split": round(n / 1e9 / wall, 2),
           "slice_tokens": counts}
    if rank == 0:
        toks = np.concatenate([p[:c].cpu().numpy().view(np.uint32) for p, c in zip(parts, counts)])
        fx = os.path.join(GOLD, "encode_c3enc1g.json")
        if os.path.exists(fx) and args.encode_bytes == 1 << 30 and args.vocab_sample_bytes == 104_857_600:
            meta = json.load(open(fx))
            res["fixture_tokens_equal"] = (toks.shape[0] == meta["n_tokens"] and
                                           hashlib.sha256(np.ascontiguousarray(toks, "<u4").tobytes()).hexdigest()
                                           == meta["tokens_sha256"])
    return res


def recount_pairs(fin_host: np.ndarray):
    """Live pair counts of a u32 reference-layout stream, recounted on the device
    with torch (a pair (i-1, i) counts iff i is not a word start and neither token
    is 0: train.wgsl:393-399).  Returns (sorted pair ids, counts)."""
    import torch
    n = fin_host.shape[0]
    step = 1 << 28
    keys, cnts = [], []
    for s0 in range(0, max(1, n - 1), step):
        s1 = min(n, s0 + step + 1)
        x = torch.from_numpy(fin_host[s0:s1].view(np.int32)).cuda().to(torch.int64) & 0xFFFFFFFF
        prev, cur = x[:-1], x[1:]
        ok = ((cur & 0x10000) == 0) & ((prev & 0xFFFF) != 0) & ((cur & 0xFFFF) != 0)
        pid = ((prev & 0xFFFF) << 16) | (cur & 0xFFFF)
        u, c = torch.unique(pid[ok], return_counts=True)
        keys.append(u)
        cnts.append(c)
        del x, prev, cur, ok, pid
    k = torch.cat(keys)
    c = torch.cat(cnts)
    u, inv = torch.unique(k, return_inverse=True)
    tot = torch.zeros(u.shape[0], dtype=torch.int64, device=u.device).index_add_(0, inv, c)
    return u.cpu().numpy().astype(np.uint32), tot.cpu().numpy()


def root_recount_check(lib, ctx, be, fin):
    """The hand-over root's live pair counts (gbpe_trainer_pair_counts) against a
    device recount of the final stream it rebuilt from every rank's occurrence list
    (counts are additive over word-start pieces: train.wgsl:395, 483, 493)."""
    from gpubpe import _lib
    st = be.root_stats()
    cnt = C.c_uint64()
    lib.gbpe_trainer_pair_counts(be.t, None, None, 0, C.byref(cnt))
    pids = np.zeros(max(1, cnt.value), np.uint32)
    cts = np.zeros(max(1, cnt.value), np.uint32)
    _lib.check(lib.gbpe_trainer_pair_counts(be.t, pids.ctypes.data_as(_lib.u32p), cts.ctypes.data_as(_lib.u32p),
                                            cnt.value, C.byref(cnt)), ctx, "pair_counts")
    o = np.argsort(pids[: cnt.value])
    tp, tc = pids[: cnt.value][o], cts[: cnt.value][o].astype(np.int64)
    t0 = time.perf_counter()
    lib.gbpe_ctx_trim(ctx)   # the context's idle pooled blocks back before torch allocates beside it
    rp, rc = recount_pairs(fin)
    res = {"final_symbols": int(fin.shape[0]), "final_symbols_equal_trainer": int(fin.shape[0]) == int(st.symbol_count),
           "pairs_live_table": int(tp.shape[0]), "pairs_live_recount": int(rp.shape[0]),
           "counts_equal_recount": bool(tp.shape == rp.shape and np.array_equal(tp, rp) and np.array_equal(tc, rc)),
           "seconds_recount": round(time.perf_counter() - t0, 2)}
    if not res["counts_equal_recount"] and tp.shape == rp.shape:
        bad = np.flatnonzero((tp != rp) | (tc != rc))
        res["first_diff"] = [int(tp[bad[0]]), int(tc[bad[0]]), int(rp[bad[0]]), int(rc[bad[0]])]
    return res


def lexshard_run(lib, ctx, dist, d, n, vocab, flags=0, want_final=False, check=False):
    """One complete run of the sharded first pass + lexicon hand-over (DESIGN §5,
    gpubpe/lexshard.py) on this rank's HBM-resident piece; every rank returns the
    global merge list.  RCCL moves the stores point to point (device tensors);
    GBPE_SHARD_TRANSPORT=gloo (ranks sharing one GPU) moves host copies.  `check`:
    after the run the root recounts the final stream (root_recount_check; returned
    on the root, None elsewhere)."""
    from gpubpe.lexshard import GpuLexBackend, LexShardTrainer
    be = GpuLexBackend(lib, ctx, vocab, flags=flags)
    staged = dist.transport != "nccl"
    tr = LexShardTrainer(be, dist.dist, staged=staged, host_group=None if staged else dist.host)
    chk = None
    try:
        merges, early = tr.train(d, n, True, vocab)
        fin = tr.final_stream() if (want_final or check) else None
        if check and tr.rank == tr.root:
            chk = root_recount_check(lib, ctx, be, fin)
            if not want_final:
                fin = None
    finally:
        be.close()
    m = np.array(merges, dtype=np.uint32).reshape(-1, 4)
    return (m, tr, fin, chk) if check else (m, tr, fin)


LEX_PHASES = ("create_s", "build_s", "exchange_s", "root_create_s", "loop_s", "total_s")   # LexShardTrainer.timing


def lex_timing(dist, tr):
    """Phase times of the last run (seconds since its start), max over ranks (the
    same keys on every rank: each is one collective)."""
    return {k: round(dist.max(float(tr.timing.get(k, 0.0))), 4) for k in LEX_PHASES}


def lexshard_line(args, lib, ctx, dist, rank, world):
    """N > 1: the headline corpus cut at word starts into one piece per rank; the
    first pass (symbols, counts, word lexicon) runs on every GPU, the merge chain
    on the last rank (the reference's loop is sequential: training-pipeline.js:
    178-222).  value = merges of the K timed runs / max wall over ranks."""
    t = time.time()
    full = make_corpus(HEADLINE)
    piece = shard_of(full, rank, world)
    log(f"[bench] rank {rank}: piece {len(piece)} B of {len(full)} in {time.time() - t:.1f}s")
    d = device_buffer(lib, ctx, piece)
    n = len(piece)
    for _ in range(args.warmup):
        lexshard_run(lib, ctx, dist, d, n, args.vocab)
    lib.gbpe_synchronize(ctx)
    dist.barrier()
    lib.gbpe_synchronize(ctx)
    t0 = time.perf_counter()
    total, last, tr = 0, None, None
    for _ in range(args.steps):
        last, tr, _ = lexshard_run(lib, ctx, dist, d, n, args.vocab)
        total += last.shape[0]
    lib.gbpe_synchronize(ctx)
    t1 = time.perf_counter()
    dist.barrier()
    wall = dist.max(t1 - t0)
    timing = lex_timing(dist, tr)
    lib.gbpe_device_free(ctx, d)
    want, meta = fixture("en1g")
    parity = {}
    if want is not None and args.vocab == 32768:
        ok = 1.0 if (last.shape == want.shape and np.array_equal(last, want)) else 0.0
        parity = {"train_fixture": "tests/golden/train_en1g.npz", "merges_checked": int(want.shape[0]),
                  "all_ranks_merges_equal_fixture": -dist.max(-ok) == 1.0}
    # secondary: every rank trains the whole corpus on its own GPU (replicated)
    dfull = device_buffer(lib, ctx, full)
    rwall, rtotal, rlast, _ = timed_runs(args, lib, ctx, dist, dfull, len(full), args.vocab, 2, 1)
    lib.gbpe_device_free(ctx, dfull)
    rst = tr.root_stats if rank == world - 1 else None
    sh = tr.shapes
    # the roofline and the CPU baseline of the N = 1 line, measured on rank 0 (the
    # merge loop is the single-GPU one: the root runs it on the global lexicon)
    roof, cpu_base = None, None
    if rank == 0:
        droof = device_buffer(lib, ctx, full)
        roof = single_gpu_roofline(args, lib, ctx, droof, len(full))
        lib.gbpe_device_free(ctx, droof)
        if not args.no_cpu:
            cpu_base, _, _ = cpu_baselines(args, full, None)
    dist.barrier()
    line = {
        "metric": METRIC,
        "value": round(total / wall, 1),
        "unit": "merges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * wall / max(1, args.steps), 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u16" if args.vocab <= 32768 else "u32",
        "data": "synthetic (seeded Zipf English-like corpus, gpubpe.synth)",
        "config": {"workload": f"headline: 32K-vocab BPE train on one 1,073,741,824 B English-like UTF-8 corpus "
                               f"(seed 2) cut at word starts into {world} pieces; step = one complete training run: "
                               "per-rank first pass (symbols, word boundaries, pair counts, word lexicon) on every "
                               "GPU, stores to the last rank, one global lexicon, all 32,512 merges there (the merge "
                               "chain is sequential), merge list broadcast",
                   "train_bytes": HEADLINE["n"], "target_vocab": args.vocab,
                   "merges_per_step": int(last.shape[0]), "parallelism": f"lexshard{world} ({dist.transport})"},
        "roofline": roof,
        "train_detail": {"timing_s_max_over_ranks": timing,
                         "pieces": {"symbols": sh[:, 5].tolist(), "store_symbols": sh[:, 0].tolist(),
                                    "entries": sh[:, 1].tolist(), "words": sh[:, 2].tolist(),
                                    "zone": int(sh[-1, 4])},
                         "amdahl": "only the first pass runs on every GPU; the merge loop (~90 % of a single-GPU "
                                   "run at 1 GiB) stays on one: DESIGN §5"},
        "replicated": {"value": round(rtotal / rwall, 1), "unit": "merges/s", "runs": 2,
                       "meaning": "every rank trains the whole corpus on its own GPU (no exchange); max wall",
                       "merges_equal_fixture": bool(want is not None and np.array_equal(rlast, want))},
        "parity": parity,
    }
    if cpu_base is not None:
        line["cpu_baseline"] = cpu_base
    if rst is not None:
        line["train_detail"]["root"] = {"sparse_exits": int(rst.sparse_exits), "max_live_pairs": int(rst.max_live_pairs),
                                        "lexicon_entries": int(rst.lexicon_entries)}
    if not args.no_encode:
        line["tokenize"] = split_encode_leg(args, lib, ctx, dist, rank, world)
    return line


C4_SHARD = 1 << 30   # 8 x 1 GiB multilingual, seed 5 + rank, 64K vocab


def c4_line(args, lib, ctx, dist, rank, world):
    """C4 (BASELINE configs[3]): one 64K vocabulary over the concatenation of
    `world` multilingual shards of --c4-shard bytes (seed 5 + rank), one shard per
    rank, re-cut at the concatenated stream's word starts (gpubpe.lexshard
    .pieces_at_word_starts); the sharded first pass + lexicon hand-over.  No
    oracle holds 8 GiB: the merge-list sha256 is reported, and the same code path
    is pinned at 8 x 128 MiB by tests/test_gpu_lexshard.py's fixture test."""
    from gpubpe.lexshard import device_word_boundary, pieces_at_word_starts
    t = time.time()
    shard = make_corpus({"gen": "multilingual", "n": args.c4_shard, "seed": 5 + rank})
    piece = pieces_at_word_starts(dist.dist, shard, device_word_boundary(lib, ctx), host_group=dist.host)
    del shard
    log(f"[bench] rank {rank}: C4 piece {len(piece)} B in {time.time() - t:.1f}s")
    d = device_buffer(lib, ctx, piece)
    n = len(piece)
    del piece
    runs = max(1, args.c4_runs)
    lib.gbpe_synchronize(ctx)
    dist.barrier()
    t0 = time.perf_counter()
    last, tr = None, None
    for _ in range(runs):
        last, tr, _ = lexshard_run(lib, ctx, dist, d, n, 65536)
    lib.gbpe_synchronize(ctx)
    t1 = time.perf_counter()
    dist.barrier()
    wall = dist.max(t1 - t0) / runs
    timing = lex_timing(dist, tr)
    # the self-check: one more, untimed run whose root recounts
    # the final stream the ranks' occurrence lists rebuild, against its live counts
    check = None
    if not args.no_c4_check:
        try:
            clast, _, _, check = lexshard_run(lib, ctx, dist, d, n, 65536, check=True)
            if check is not None:
                check["merges_equal_timed_run"] = bool(np.array_equal(clast, last))
        except Exception as e:  # noqa: BLE001
            check = {"error": f"{type(e).__name__}: {e}"}
        objs = [None] * world
        dist.dist.all_gather_object(objs, check, group=dist.host)
        check = next((o for o in objs if o is not None), None)
    lib.gbpe_device_free(ctx, d)
    sh = tr.shapes
    rst = tr.root_stats if rank == world - 1 else None
    res = {"workload": f"C4: 64K-vocab train on {world} x {args.c4_shard} B multilingual UTF-8 shards "
                       f"(seeds 5..{4 + world}) concatenated ({int(sh[:, 5].sum())} symbols), sharded first pass + "
                       "lexicon hand-over to the last rank",
           "value": round(last.shape[0] / wall, 1), "unit": "merges/s", "runs": runs, "s_per_run": round(wall, 3),
           "merges": int(last.shape[0]), "last_merge": last[-1].tolist() if last.shape[0] else [],
           "merges_sha256": hashlib.sha256(np.ascontiguousarray(last, "<u4").tobytes()).hexdigest(),
           "timing_s_max_over_ranks": timing, "transport": dist.transport,
           "stream_symbols": int(sh[:, 5].sum()), "store_symbols": int(sh[:, 0].sum()), "zone": int(sh[-1, 4])}
    if check is not None:
        res["check"] = check
        res["counts_equal_recount"] = bool(check.get("counts_equal_recount", False))
    if rst is not None:
        from gpubpe import reftable
        res["root"] = {"sparse_exits": int(rst.sparse_exits), "lexicon_entries": int(rst.lexicon_entries),
                       "tail_dropped": int(rst.tail_dropped), "final_symbols": int(rst.symbol_count),
                       "reference_table": reftable.report(int(rst.max_live_pairs))}
    return res


def replicated_line(args, lib, ctx, dist, rank, world):
    data, wall, total, last, det, parity = headline_leg(args, lib, ctx, dist)
    line = {
        "metric": METRIC,
        "value": round(total / wall, 1),
        "unit": "merges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * wall / max(1, args.steps), 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": f"u{8 * det['bytes_per_symbol']}",
        "data": "synthetic (seeded Zipf English-like corpus, gpubpe.synth)",
        "config": {"workload": "headline: 32K-vocab BPE train on one 1,073,741,824 B English-like UTF-8 corpus (seed 2); "
                               f"{world} ranks each run the complete training (the merge chain is sequential: "
                               "replicated, no per-merge exchange); step = one complete training run; value = global "
                               "merges / max wall over ranks",
                   "train_bytes": HEADLINE["n"], "target_vocab": args.vocab,
                   "merges_per_step": det["merges_per_run"], "parallelism": f"replicated{world}"},
        "roofline": train_roofline(det, wall / max(1, args.steps)),
        "train_detail": det,
        "parity": parity,
    }
    ok = 1.0 if parity.get("train_merges_equal_fixture", True) else 0.0
    line["parity"]["all_ranks_merges_equal_fixture"] = -dist.max(-ok) == 1.0
    if not args.no_encode:
        line["tokenize"] = split_encode_leg(args, lib, ctx, dist, rank, world)
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5, help="timed steps: complete training runs of the headline corpus")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--vocab", type=int, default=32768)
    ap.add_argument("--encode-bytes", type=int, default=1 << 30)
    ap.add_argument("--vocab-sample-bytes", type=int, default=104_857_600)
    ap.add_argument("--no-encode", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-c1", action="store_true", help="skip the C1 leg (1K vocab on 256 KiB ASCII)")
    ap.add_argument("--no-c2", action="store_true")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 per-rank shard leg (64K vocab)")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 leg (1 GiB code, 50K vocab, GPT-4 rules)")
    ap.add_argument("--no-ml1g", action="store_true", help="skip the 1 GiB multilingual @ 32K training leg")
    ap.add_argument("--no-kernel-timing", action="store_true", help="skip the HIP-event roofline run")
    ap.add_argument("--cpu-merges", type=int, default=0, help="CPU baseline merges on the CPU share (0 = 24)")
    ap.add_argument("--replicated", action="store_true",
                    help="N > 1: every rank trains the whole corpus (round-2 line) instead of the lexicon hand-over")
    ap.add_argument("--c4-only", action="store_true",
                    help="only the C4 leg: one multilingual shard per rank (seed 5 + rank), one 64K vocab")
    ap.add_argument("--c4-shard", type=int, default=C4_SHARD, help="C4 shard bytes per rank")
    ap.add_argument("--c4-runs", type=int, default=1)
    ap.add_argument("--no-c4-check", action="store_true",
                    help="skip the C4 leg's untimed self-check run (root live counts vs a recount of the final stream)")
    args = ap.parse_args()

    rank, world, local = dist_env()
    dist = Dist(world, local, force=args.c4_only)
    from gpubpe import _lib
    lib = _lib.load()
    ctx = C.c_void_p()
    rc = lib.gbpe_ctx_create(int(os.environ.get("GBPE_BENCH_DEVICE", local)) if world > 1 else 0, C.byref(ctx))
    if rc != 0:
        raise SystemExit(f"gbpe_ctx_create failed ({rc}): no MI355X visible")
    if args.c4_only:
        line = {"metric": METRIC, "c4": c4_line(args, lib, ctx, dist, rank, world)}
    elif world > 1 and args.replicated:
        line = replicated_line(args, lib, ctx, dist, rank, world)
    elif world > 1:
        line = lexshard_line(args, lib, ctx, dist, rank, world)
        if world == 8 and not args.no_c4:   # C4's configuration: one 1 GiB shard per GPU
            try:
                line["c4"] = c4_line(args, lib, ctx, dist, rank, world)
            except Exception as e:  # noqa: BLE001
                line["c4"] = {"error": f"{type(e).__name__}: {e}"}
    else:
        line = single_line(args, lib, ctx, dist, rank)
    if rank == 0:
        print(json.dumps(line), flush=True)
    lib.gbpe_ctx_destroy(ctx)


if __name__ == "__main__":
    main()
