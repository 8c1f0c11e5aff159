#!/usr/bin/env python3
"""C4 above 2^32 symbols (Missing 4): the lexicon hand-over at full
size, 8 x 1 GiB multilingual shards (seeds 5..12, 8,589,934,592 symbols), 64K
vocab, checked two ways:

  (a) the first K merges against the reference algorithm restated on the CPU
      with 64-bit positions (oracle/bpe_oracle.c, full pair recount per merge)
      on the concatenated corpus;
  (b) after the whole run, the root's live pair counts (gbpe_trainer_pair_counts)
      against a recount of the final stream the root rebuilds from every rank's
      occurrence list (gbpe_trainer_expand), counted on the device with torch
      (pairs never span a word start or hold token 0: train.wgsl:393-399).

Ranks share one GPU over gloo (the one-GPU rehearsal of DESIGN §5):
  GBPE_BENCH_DEVICE=0 GBPE_SHARD_TRANSPORT=gloo python -m torch.distributed.run \\
      --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29571 tools/c4_check.py
Rank 0 prints one JSON line.  Diagnostic; not part of the product.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gpu-bpe_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import bench as B  # noqa: E402

SHARD = int(os.environ.get("C4_SHARD", str(1 << 30)))
K = int(os.environ.get("C4_K", "6"))
WS = 0x10000


def log(*a):
    print(*a, file=sys.stderr, flush=True)


recount = B.recount_pairs   # (bench.py: the C4 leg runs the same check)


def heartbeat(rank):
    # gpurun takes 3 minutes without output for a hang: one line per 30 s
    import threading

    def beat():
        t0 = time.time()
        while True:
            time.sleep(30)
            log(f"[c4check] rank {rank} alive {time.time() - t0:.0f}s")
    threading.Thread(target=beat, daemon=True).start()


def main():
    from gpubpe import _lib, synth
    from gpubpe.lexshard import GpuLexBackend, LexShardTrainer, device_word_boundary, pieces_at_word_starts
    rank, world, local = B.dist_env()
    if rank == 0:
        heartbeat(rank)
    dist = B.Dist(world, local, force=True)
    lib = _lib.load()
    ctx = C.c_void_p()
    _lib.check(lib.gbpe_ctx_create(int(os.environ.get("GBPE_BENCH_DEVICE", local)), C.byref(ctx)), None, "ctx")
    t0 = time.time()
    shard = synth.multilingual(SHARD, seed=5 + rank)
    shm = f"/dev/shm/c4check_{os.getpid()}_{rank}"
    with open(shm, "wb") as f:   # rank 0 builds the concatenated corpus for the CPU oracle from these
        f.write(shard)
    all_names = [None] * world
    dist.dist.all_gather_object(all_names, shm, group=dist.host)
    piece = pieces_at_word_starts(dist.dist, shard, device_word_boundary(lib, ctx), host_group=dist.host)
    del shard
    log(f"[c4check] rank {rank}: piece {len(piece)} B in {time.time() - t0:.1f}s")
    d = B.device_buffer(lib, ctx, piece)
    n = len(piece)
    del piece
    be = GpuLexBackend(lib, ctx, 65536)
    tr = LexShardTrainer(be, dist.dist, staged=True, host_group=dist.host)
    t1 = time.time()
    merges, early = tr.train(d, n, True, 65536)
    t2 = time.time()
    res = {"shards": world, "shard_bytes": SHARD, "merges": len(merges), "seconds_train": round(t2 - t1, 2),
           "stream_symbols": int(tr.shapes[:, 5].sum()), "zones": tr.shapes[:, 4].tolist(),
           "merges_sha256": hashlib.sha256(np.ascontiguousarray(np.array(merges, np.uint32), "<u4").tobytes()).hexdigest(),
           "store_symbols": int(tr.shapes[:, 0].sum()), "store_entries": int(tr.shapes[:, 1].sum()),
           "timing_rank%d" % rank: {k: round(float(v), 3) for k, v in tr.timing.items()}}
    fin = tr.final_stream()   # root: the final stream (host u32), rebuilt from every rank's occurrence list
    lib.gbpe_device_free(ctx, d)
    if rank == tr.root:
        st = be.root_stats()
        res["final_symbols"] = int(fin.shape[0])
        res["final_symbols_equal_trainer"] = int(fin.shape[0]) == int(st.symbol_count)
        # (b) live pair counts of the root's table against a recount of the expanded stream
        cnt = C.c_uint64()
        lib.gbpe_trainer_pair_counts(be.t, None, None, 0, C.byref(cnt))
        pids = np.zeros(max(1, cnt.value), np.uint32)
        cts = np.zeros(max(1, cnt.value), np.uint32)
        _lib.check(lib.gbpe_trainer_pair_counts(be.t, pids.ctypes.data_as(_lib.u32p), cts.ctypes.data_as(_lib.u32p),
                                                cnt.value, C.byref(cnt)), ctx, "pair_counts")
        o = np.argsort(pids[: cnt.value])
        tp, tc = pids[: cnt.value][o], cts[: cnt.value][o].astype(np.int64)
        t3 = time.time()
        rp, rc = recount(fin)
        res["pairs_live_table"] = int(tp.shape[0])
        res["pairs_live_recount"] = int(rp.shape[0])
        res["pair_counts_equal"] = bool(tp.shape == rp.shape and np.array_equal(tp, rp) and np.array_equal(tc, rc))
        res["seconds_recount"] = round(time.time() - t3, 1)
        if not res["pair_counts_equal"] and tp.shape == rp.shape:
            bad = np.flatnonzero((tp != rp) | (tc != rc))
            res["first_diff"] = [int(tp[bad[0]]), int(tc[bad[0]]), int(rp[bad[0]]), int(rc[bad[0]])]
        del fin
    # (a) the first K merges against the CPU restatement on the concatenation (rank 0)
    dist.barrier()
    be.close()
    if rank == 0:
        import cpu_ref
        t4 = time.time()
        data = b"".join(open(p, "rb").read() for p in all_names)
        share = int(os.environ.get("OMP_NUM_THREADS", "0")) or 16
        r = cpu_ref.train(data, 65536, max_merges=K, threads=share, want_symbols=False)
        res["cpu_first_merges"] = r["merges"]
        res["cpu_first_merges_equal"] = r["merges"] == merges[: len(r["merges"])]
        res["cpu_seconds"] = round(time.time() - t4, 1)
        res["cpu_threads"] = share
        del data
    dist.barrier()
    os.remove(shm)
    # the root's results to rank 0
    out = [None] * world
    dist.dist.all_gather_object(out, res, group=dist.host)
    if rank == 0:
        merged = dict(out[0])
        merged.update({k: v for k, v in out[world - 1].items() if k not in merged})
        merged["timing_max_over_ranks"] = {k: max(o["timing_rank%d" % q].get(k, 0.0) for q, o in enumerate(out))
                                           for k in out[world - 1]["timing_rank%d" % (world - 1)]}
        print(json.dumps(merged), flush=True)
    lib.gbpe_ctx_destroy(ctx)


if __name__ == "__main__":
    main()
