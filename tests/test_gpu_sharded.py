"""Sharded training through the C-ABI on the GPU (world size 2 and 3 sharing
one MI355X, gloo with host-staged records): merge lists and the concatenated
final stream equal the single-stream oracle (reference semantics).  Also the
consolidation path: a sharded run handed over to one device mid-run, and a
single trainer's state exported and resumed (gbpe_trainer_export_state /
gbpe_trainer_create_from_state)."""
from __future__ import annotations

import json
import os
import sys
import tempfile

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "gpu-bpe_amd"))

import bpe_oracle as O  # noqa: E402
from gpubpe import synth  # noqa: E402
from test_sharded import _free_port, cut_at_word_starts  # noqa: E402

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, case, outdir):
    import ctypes as C
    import torch
    import torch.distributed as dist
    from gpubpe import _lib
    from gpubpe.sharded import GpuShardBackend, GpuSingleBackend, ShardedTrainer
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    nccl = case.get("nccl", False)   # RCCL over device buffers: the HBM-resident hand-over
    if nccl:
        torch.cuda.set_device(0)
    dist.init_process_group("nccl" if nccl else "gloo", rank=rank, world_size=world)
    lib = _lib.load()
    ctx = C.c_void_p()
    _lib.check(lib.gbpe_ctx_create(0, C.byref(ctx)), ctx, "ctx")
    try:
        torch.cuda.set_device(0)
        data = synth.english(case["bytes"], seed=case["seed"])
        shards, _ = cut_at_word_starts(data, case["fracs"])
        d, ws = shards[rank]
        flags = {None: 0, "dense": _lib.GBPE_TRAIN_DENSE_ONLY, "early": _lib.GBPE_TRAIN_SPARSE_EARLY}[case.get("sparse")]
        be = GpuShardBackend(lib, ctx, d, ws, rank, world, case["vocab"], exact=case["exact"],
                             table_log2=16, cap_extra=len(data), stream=torch.cuda.current_stream().cuda_stream,
                             flags=flags)
        assert lib.gbpe_ctx_get_stream(ctx) == (torch.cuda.current_stream().cuda_stream or None)
        tr = ShardedTrainer(be, dist, device="cuda", staged=not nccl, cap_list=case["cap"], cap_win=case["cap"])
        tr.setup()
        cb = case.get("consolidate")
        below = None if cb is None else int(cb * len(data))
        merges, early = tr.train(case["vocab"], batch=case.get("batch", 128), consolidate_below=below,
                                 make_single=lambda c, p, nid: GpuSingleBackend(lib, ctx, c, p, case["vocab"], nid,
                                                                                exact=case["exact"]),
                                 root=case.get("root", 0))
        st = _lib.TrainerStats()
        lib.gbpe_trainer_stats_get(be.t, C.byref(st))
        single_sparse = 0
        if tr.single is not None:   # the root holds the whole stream; the others none
            sym = tr.single.symbols()
            single_sparse = int(tr.single.stats().sparse_merges)
            tr.single.close()
        elif tr.consolidated_at is not None:
            sym = np.zeros(0, np.uint32)
        else:
            sym = be.symbols()
        np.save(os.path.join(outdir, f"sym{rank}.npy"), sym)
        with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
            json.dump({"merges": merges, "early": early, "stalls": tr.stalls, "sparse_merges": int(st.sparse_merges),
                       "consolidated_at": tr.consolidated_at, "single_sparse": single_sparse}, f)
        be.close()
    finally:
        lib.gbpe_ctx_destroy(ctx)
        dist.destroy_process_group()


def run_case(world, case):
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as td:
        mp.start_processes(_worker, args=(world, _free_port(), case, td), nprocs=world, start_method="spawn",
                           join=True)
        res = [json.load(open(os.path.join(td, f"r{r}.json"))) for r in range(world)]
        syms = [np.load(os.path.join(td, f"sym{r}.npy")) for r in range(world)]
    return res, syms


# sparse: None = the library's policy (dense, then the sector-sparse loop once the
# counts allow), "dense" = the dense loop only, "early" = sparse from the first
# step boundary where the last rank's zone fits
CASES = [
    ("ref_w2", 2, dict(bytes=60_000, seed=21, fracs=[0.5], vocab=700, exact=False, cap=1 << 14)),
    ("exact_w2", 2, dict(bytes=60_000, seed=22, fracs=[0.5], vocab=700, exact=True, cap=1 << 14)),
    ("ref_w3_tiny_middle", 3, dict(bytes=20_000, seed=13, fracs=[0.945, 0.965], vocab=480, exact=False,
                                   cap=1 << 14)),
    ("ref_w2_stalls", 2, dict(bytes=16_000, seed=14, fracs=[0.6], vocab=420, exact=False, cap=8, batch=32)),
    ("dense_ref_w2", 2, dict(bytes=60_000, seed=21, fracs=[0.5], vocab=700, exact=False, cap=1 << 14,
                             sparse="dense")),
    ("dense_ref_w3_tiny_middle", 3, dict(bytes=20_000, seed=13, fracs=[0.945, 0.965], vocab=480, exact=False,
                                         cap=1 << 14, sparse="dense")),
    ("sparse_ref_w2", 2, dict(bytes=80_000, seed=23, fracs=[0.5], vocab=1200, exact=False, cap=1 << 14,
                              sparse="early", batch=16)),
    ("sparse_exact_w3", 3, dict(bytes=80_000, seed=24, fracs=[0.3, 0.7], vocab=1000, exact=True, cap=1 << 14,
                                sparse="early", batch=32)),
    ("sparse_ref_w3_stalls", 3, dict(bytes=40_000, seed=25, fracs=[0.4, 0.75], vocab=800, exact=False, cap=8,
                                     sparse="early", batch=16)),
    # consolidation: hand-over to one device once the global stream is <= a
    # fraction of the corpus (from the dense and from the sector-sparse shard loop)
    ("consolidate_ref_w2", 2, dict(bytes=60_000, seed=21, fracs=[0.5], vocab=700, exact=False, cap=1 << 14,
                                   batch=32, consolidate=0.7)),
    ("consolidate_exact_w2", 2, dict(bytes=60_000, seed=22, fracs=[0.5], vocab=700, exact=True, cap=1 << 14,
                                     batch=32, consolidate=0.7)),
    ("consolidate_nccl_w1", 1, dict(bytes=60_000, seed=21, fracs=[], vocab=700, exact=False, cap=1 << 14,
                                    batch=32, consolidate=0.7, nccl=True)),
    ("consolidate_sparse_ref_w3", 3, dict(bytes=80_000, seed=24, fracs=[0.3, 0.7], vocab=1000, exact=False,
                                          cap=1 << 14, sparse="early", batch=16, consolidate=0.6, root=1)),
]


@pytest.mark.parametrize("name,world,case", CASES, ids=[c[0] for c in CASES])
def test_gpu_sharded_matches_single_stream(name, world, case):
    res, syms = run_case(world, case)
    data = synth.english(case["bytes"], seed=case["seed"])
    exp = O.train(data, case["vocab"], compaction="exact" if case["exact"] else "reference")
    for r in range(world):
        assert res[r]["merges"] == exp["merges"], f"rank {r} merge list differs"
        assert res[r]["early"] == exp["early_stop"]
    np.testing.assert_array_equal(np.concatenate(syms), exp["symbols"])
    if name.endswith("stalls"):
        assert res[0]["stalls"] > 0
    if case.get("consolidate"):
        at = res[0]["consolidated_at"]
        assert at is not None and 0 < at < len(exp["merges"]), at
        assert all(r["consolidated_at"] == at for r in res)
    if case.get("sparse") == "early":
        assert all(r["sparse_merges"] > 0 for r in res), "the sector-sparse loop never ran"
    if case.get("sparse") == "dense":
        assert all(r["sparse_merges"] == 0 for r in res)


RESUME = [("ref", False, 300), ("exact", True, 300), ("ref_first", False, 0), ("ref_late", False, 1100)]


@pytest.mark.parametrize("name,exact,split", RESUME, ids=[r[0] for r in RESUME])
def test_gpu_export_state_resume(name, exact, split):
    """One trainer runs `split` merges, exports (current, previous) streams; a
    second trainer created from that state finishes the run: merges and the
    final stream equal the oracle's uninterrupted run."""
    import ctypes as C
    from gpubpe import _lib
    from gpubpe.sharded import GpuSingleBackend, export_state
    lib = _lib.load()
    ctx = C.c_void_p()
    _lib.check(lib.gbpe_ctx_create(0, C.byref(ctx)), ctx, "ctx")
    data = synth.english(400_000, seed=31)
    vocab = 1800
    exp = O.train(data, vocab, compaction="exact" if exact else "reference")
    try:
        opts = _lib.TrainOpts(target_vocab_size=vocab, vocab_size=256, next_token_id=256, batch_size=128,
                              flags=_lib.GBPE_TRAIN_EXACT_COMPACTION if exact else 0, table_log2=0)
        t = C.c_void_p()
        buf = C.create_string_buffer(data, len(data))
        _lib.check(lib.gbpe_trainer_create(ctx, buf, len(data), None, 0, C.byref(opts), C.byref(t)), ctx, "create")
        got = []
        out = (C.c_uint32 * 512)()
        while len(got) < split:
            nd, es = C.c_uint32(), C.c_uint32()
            _lib.check(lib.gbpe_trainer_step(t, min(128, split - len(got)), out, C.byref(nd), C.byref(es)), ctx, "step")
            got += [list(out[4 * i: 4 * i + 4]) for i in range(nd.value)]
        cur, prev = export_state(lib, ctx, t)
        lib.gbpe_trainer_destroy(t)
        assert cur.shape[0] == exp["n_history"][split]
        assert prev.shape[0] == (exp["n_history"][split - 1] if split else cur.shape[0])
        single = GpuSingleBackend(lib, ctx, cur, prev, vocab, 256 + split, exact=exact)
        while len(got) < len(exp["merges"]):
            m, early = single.step(128)
            got += m
            if early or not m:
                break
        assert got == exp["merges"]
        np.testing.assert_array_equal(single.symbols(), exp["symbols"])
        single.close()
    finally:
        lib.gbpe_ctx_destroy(ctx)
