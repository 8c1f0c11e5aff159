"""Sharded training protocol over gloo (world size 2 and 3, CPU).

The real orchestration (gpubpe.sharded.ShardedTrainer) drives numpy models of
each rank (tests/shard_model.py) through torch.distributed all-gathers; the
merge list and the final global stream must equal the single-stream oracle
(reference semantics, both compaction modes) on the concatenated corpus.
Shards are cut at word starts of the global heuristic mask, which is passed to
each rank as its external word-start mask (trainer.js:115-121).
"""
from __future__ import annotations

import json
import os
import socket
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


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def cut_at_word_starts(data: bytes, fracs):
    """Cut points at word starts of the global heuristic mask, near the given
    cumulative fractions. Returns [(bytes, ws_slice)]."""
    arr = np.frombuffer(data, np.uint8)
    ws = O.heuristic_word_starts(arr)
    starts = np.flatnonzero(ws)
    cuts = [0]
    for f in fracs:
        target = int(f * len(data))
        i = int(np.searchsorted(starts, target))
        c = int(starts[min(i, len(starts) - 1)])
        cuts.append(max(c, cuts[-1]))
    cuts.append(len(data))
    return [(data[a:b], ws[a:b].astype(np.uint8)) for a, b in zip(cuts[:-1], cuts[1:])], ws


def _worker(rank, world, port, case, outdir):
    import torch.distributed as dist
    from gpubpe.sharded import ShardedTrainer
    from shard_model import ModelShardBackend, OracleSingle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = synth.english(case["bytes"], seed=case["seed"])
        shards, _ = cut_at_word_starts(data, case["fracs"])
        d, ws = shards[rank]
        be = ModelShardBackend(d, ws, rank, world, case["vocab"], exact=case["exact"])
        tr = ShardedTrainer(be, dist, cap_list=case["cap"], cap_win=case["cap"])
        tr.setup()
        cb = case.get("consolidate")
        below = None if cb is None else int(cb * len(data))

        def make_single(c, p, nid):
            if case.get("fail_single"):
                raise MemoryError("simulated failure building the consolidated trainer")
            return OracleSingle(c, p, nid, case["exact"])
        if case.get("fail_single"):   # every rank must raise (root: the error; others: the -1 status)
            try:
                tr.train(case["vocab"], batch=case.get("batch", 128), consolidate_below=below,
                         make_single=make_single, root=case.get("root", 0))
                raised = ""
            except Exception as e:  # noqa: BLE001
                raised = type(e).__name__
            with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
                json.dump({"raised": raised}, f)
            np.save(os.path.join(outdir, f"sym{rank}.npy"), np.zeros(0, np.uint32))
            return
        merges, early = tr.train(case["vocab"], batch=case.get("batch", 128), consolidate_below=below,
                                 make_single=make_single, root=case.get("root", 0))
        if tr.single is not None:   # the root holds the whole stream; the others none
            sym = tr.single.symbols()
        elif tr.consolidated_at is not None:
            sym = np.zeros(0, np.uint32)
        else:
            sym = be.symbols()
        np.save(os.path.join(outdir, f"sym{rank}.npy"), sym)
        with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
            json.dump({"merges": merges, "early": early, "stalls": tr.stalls, "events": be.events,
                       "consolidated_at": tr.consolidated_at}, f)
    finally:
        dist.destroy_process_group()


def run_case(world, case):
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as td:
        mp.start_processes(_worker, args=(world, _free_port(), case, td), nprocs=world, start_method="spawn",
                           join=True)
        res = [json.load(open(os.path.join(td, f"r{r}.json"))) for r in range(world)]
        syms = [np.load(os.path.join(td, f"sym{r}.npy")) for r in range(world)]
    return res, syms


def _expected(case):
    data = synth.english(case["bytes"], seed=case["seed"])
    return O.train(data, case["vocab"], compaction="exact" if case["exact"] else "reference")


CASES = [
    ("ref_w2", 2, dict(bytes=24_000, seed=11, fracs=[0.5], vocab=520, exact=False, cap=1 << 14)),
    ("exact_w2", 2, dict(bytes=24_000, seed=12, fracs=[0.5], vocab=520, exact=True, cap=1 << 14)),
    # tiny last shard: the stale window spans ranks, trailing ranks empty out, owner moves
    ("ref_w3_tiny_tail", 3, dict(bytes=20_000, seed=13, fracs=[0.945, 0.965], vocab=480, exact=False, cap=1 << 14)),
    # tiny capacities: every early merge stalls and the host grows C/Cw
    ("ref_w2_stalls", 2, dict(bytes=16_000, seed=14, fracs=[0.6], vocab=420, exact=False, cap=8, batch=32)),
    # consolidation onto one rank once the global stream is <= a fraction of the
    # corpus: the merge list and the final stream are unchanged
    ("ref_w2_consolidate", 2, dict(bytes=24_000, seed=11, fracs=[0.5], vocab=520, exact=False, cap=1 << 14,
                                   batch=32, consolidate=0.8)),
    ("exact_w2_consolidate", 2, dict(bytes=24_000, seed=12, fracs=[0.5], vocab=520, exact=True, cap=1 << 14,
                                     batch=32, consolidate=0.8)),
    # windows spanning ranks right before the hand-over; root is the last rank
    ("ref_w3_tiny_tail_consolidate", 3, dict(bytes=20_000, seed=13, fracs=[0.945, 0.965], vocab=480, exact=False,
                                             cap=1 << 14, batch=16, consolidate=0.75, root=2)),
]


@pytest.mark.parametrize("name,world,case", CASES, ids=[c[0] for c in CASES])
def test_sharded_matches_single_stream(name, world, case):
    res, syms = run_case(world, case)
    exp = _expected(case)
    for r in range(world):
        assert res[r]["merges"] == exp["merges"], f"rank {r} merge list differs"
        assert res[r]["early"] == exp["early_stop"]
    np.testing.assert_array_equal(np.concatenate(syms), exp["symbols"])
    if case.get("consolidate"):
        at = res[0]["consolidated_at"]
        assert at is not None and 0 < at < len(exp["merges"]), at
    if name.endswith("stalls"):
        assert res[0]["stalls"] > 0
    if name.endswith("tiny_tail"):
        ev = res[0]["events"]
        assert ev["window_multi_rank"] > 0 and ev["owner_not_last"] > 0, ev


def test_consolidation_failure_on_root_reaches_every_rank():
    """a failure on root during consolidation must not leave the other
    ranks blocked in the merge-list broadcast."""
    case = dict(bytes=24_000, seed=11, fracs=[0.5], vocab=520, exact=False, cap=1 << 14, batch=32, consolidate=0.8,
                fail_single=True)
    res, _ = run_case(2, case)
    assert res[0]["raised"] == "MemoryError"
    assert res[1]["raised"] == "RuntimeError"
