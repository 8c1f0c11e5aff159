"""Lexicon hand-over protocol over gloo (world size 1, 2 and 3, CPU).

The real host loop (gpubpe.lexshard.LexShardTrainer, pieces_at_word_starts)
drives numpy models of a rank and of the root (tests/lexshard_model.py) through
torch.distributed point-to-point transfers and all-gathers: the corpus is given
as R consecutive shards cut anywhere (not at word starts), each rank's piece is
re-cut at the concatenated stream's word starts (the halo of the previous
shard's last byte), the stores meet on the last rank, and the merge list and
the final stream rebuilt from every rank's occurrence list must equal the
single-stream oracle on the concatenated corpus (both compaction modes).
"""
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


from dist_util import free_port as _free_port  # noqa: E402


def _corpus(case):
    if case.get("gen") == "multilingual":
        return b"".join(synth.multilingual(case["shard"], seed=sd) for sd in case["seeds"])
    return synth.english(case["bytes"], seed=case["seed"])


def _shards(data: bytes, fracs):
    cuts = [0] + [int(f * len(data)) for f in fracs] + [len(data)]
    return [data[a:b] for a, b in zip(cuts[:-1], cuts[1:])]


def _worker(rank, world, port, case, outdir):
    import torch.distributed as dist
    from gpubpe.lexshard import LexShardTrainer, pieces_at_word_starts
    from lexshard_model import ModelLexBackend
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = _corpus(case)
        shard = _shards(data, case["fracs"])[rank]
        piece = pieces_at_word_starts(dist, shard, lambda b: O.heuristic_word_starts(np.frombuffer(b, np.uint8)),
                                      halo=case.get("halo", 1 << 16))
        be = ModelLexBackend(exact=case["exact"])
        if case.get("fail_build") == rank:   # a rank whose build fails: every rank must raise, none may hang
            def boom(zt):
                raise RuntimeError("injected build failure")
            be.build = boom
        tr = LexShardTrainer(be, dist, staged=True)
        try:
            merges, early = tr.train(piece, len(piece), False, case["vocab"], batch=case.get("batch", 128))
        except RuntimeError as e:
            with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
                json.dump({"error": str(e)}, f)
            return
        fin = tr.final_stream()
        if fin is not None:
            np.save(os.path.join(outdir, "final.npy"), fin)
        with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
            json.dump({"merges": merges, "early": early, "piece": len(piece), "zones": tr.shapes[:, 4].tolist()}, f)
    finally:
        dist.destroy_process_group()


def run_case(world, case):
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as td:
        mp.start_processes(_worker, args=(world, _free_port(), case, td), nprocs=world, start_method="spawn",
                           join=True)
        res = [json.load(open(os.path.join(td, f"r{r}.json"))) for r in range(world)]
        fin = np.load(os.path.join(td, "final.npy")) if os.path.exists(os.path.join(td, "final.npy")) else None
    return res, fin


CASES = [
    ("ref_w1", 1, dict(bytes=20_000, seed=21, fracs=[], vocab=480, exact=False)),
    ("ref_w2", 2, dict(bytes=24_000, seed=22, fracs=[0.4], vocab=520, exact=False)),
    ("exact_w2", 2, dict(bytes=24_000, seed=23, fracs=[0.5], vocab=520, exact=True, batch=32)),
    ("ref_w3", 3, dict(bytes=30_000, seed=24, fracs=[0.2, 0.45], vocab=560, exact=False, batch=16)),
    # C4-shaped: the concatenation of independently generated multilingual shards
    # (UTF-8 sequences and words cut at the shard seams), 3 shards at 64K-style ids
    ("c4_shaped_w3", 3, dict(gen="multilingual", shard=12_000, seeds=[5, 6, 7], fracs=[1 / 3, 2 / 3], vocab=600,
                             exact=False)),
    # the zone (5 x the first count) is longer than the last piece: it spans the
    # tail of one piece and the whole of the next ones (the N=8 headline shape)
    ("zone_spans_w3", 3, dict(bytes=30_000, seed=25, fracs=[0.6, 0.93], vocab=560, exact=False, spans=2)),
    ("zone_spans_w4_exact", 4, dict(bytes=30_000, seed=26, fracs=[0.5, 0.9, 0.95], vocab=560, exact=True, batch=32,
                                    spans=3)),
]


@pytest.mark.parametrize("name,world,case", CASES, ids=[c[0] for c in CASES])
def test_lexshard_matches_single_stream(name, world, case):
    res, fin = run_case(world, case)
    data = _corpus(case)
    exp = O.train(data, case["vocab"], compaction="exact" if case["exact"] else "reference")
    for r in range(world):
        assert res[r]["merges"] == exp["merges"], f"rank {r} merge list differs"
        assert res[r]["early"] == exp["early_stop"]
    assert sum(r["piece"] for r in res) == len(data)       # the pieces tile the corpus
    np.testing.assert_array_equal(fin, exp["symbols"])
    if "spans" in case:
        assert sum(1 for z in res[0]["zones"] if z) >= case["spans"], res[0]["zones"]


def test_lexshard_failure_reaches_every_rank():
    # a rank failing in its build must not leave the others blocked in
    # the next collective — every rank raises
    res, _ = run_case(3, dict(bytes=24_000, seed=22, fracs=[0.4, 0.7], vocab=520, exact=False, fail_build=1))
    assert all("error" in r for r in res), res
    assert "injected" in res[1]["error"] and "rank(s) [1]" in res[0]["error"]
