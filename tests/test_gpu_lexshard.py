"""Sharded first pass + lexicon hand-over through the C-ABI on the GPU
(gbpe_lexshard_* / gbpe_trainer_create_from_lexicon / gbpe_trainer_expand):
2, 3 and 8 ranks sharing one MI355X over gloo (host-staged transfers).  Every
rank's merge list and the final stream rebuilt from every rank's occurrence
list equal the single-stream oracle on the concatenated corpus — the C
incremental restatement (oracle/bpe_oracle_inc.c via cpu_ref) for the small
cases, and the committed C4-shaped fixture tests/golden/train_c4s8x128m.npz
(8 x 128 MiB multilingual shards, seeds 5..12, 64K vocab) at world 8."""
from __future__ import annotations

import hashlib
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

from gpubpe import synth  # noqa: E402
from dist_util import free_port as _free_port  # noqa: E402

pytestmark = pytest.mark.gpu
GOLD = os.path.join(HERE, "golden")


def _corpus(case):
    if case["gen"] == "ml_shards":
        return [synth.multilingual(case["shard"], seed=sd) for sd in case["seeds"]]
    data = synth.english(case["bytes"], seed=case["seed"])
    cuts = [0] + [int(f * len(data)) for f in case["fracs"]] + [len(data)]
    return [data[a:b] for a, b in zip(cuts[:-1], cuts[1:])]


def _worker(rank, world, port, case, outdir):
    import ctypes as C
    import torch.distributed as dist
    from gpubpe import _lib
    from gpubpe.lexshard import GpuLexBackend, LexShardTrainer, device_word_boundary, pieces_at_word_starts
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = _lib.load()
    ctx = C.c_void_p()
    _lib.check(lib.gbpe_ctx_create(0, C.byref(ctx)), ctx, "ctx")
    be = None
    try:
        if case["gen"] == "ml_shards":
            shard = synth.multilingual(case["shard"], seed=case["seeds"][rank])
        else:
            shard = _corpus(case)[rank]
        piece = pieces_at_word_starts(dist, shard, device_word_boundary(lib, ctx))
        del shard
        flags = _lib.GBPE_TRAIN_EXACT_COMPACTION if case.get("exact") else 0
        be = GpuLexBackend(lib, ctx, case["vocab"], flags=flags)
        tr = LexShardTrainer(be, dist, staged=True)
        merges, early = tr.train(piece, len(piece), False, case["vocab"])
        fin = tr.final_stream()
        res = {"merges": merges, "early": early, "piece": len(piece), "timing": tr.timing,
               "shapes": tr.shapes.tolist()}
        if fin is not None:
            res["final_n"] = int(fin.shape[0])
            res["final_sha256"] = hashlib.sha256(np.ascontiguousarray(fin, "<u4").tobytes()).hexdigest()
            st = tr.root_stats
            res["root"] = {"sparse_exits": int(st.sparse_exits), "sparse_merges": int(st.sparse_merges),
                           "lexicon_entries": int(st.lexicon_entries), "tail_dropped": int(st.tail_dropped),
                           "symbol_count": int(st.symbol_count)}
        with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
            json.dump(res, f)
    finally:
        if be is not None:
            be.close()
        lib.gbpe_ctx_destroy(ctx)
        dist.destroy_process_group()


def run_case(world, case):
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as td:
        mp.start_processes(_worker, args=(world, _free_port(), case, td), nprocs=world, start_method="spawn",
                           join=True)
        return [json.load(open(os.path.join(td, f"r{r}.json"))) for r in range(world)]


def _expected(case):
    import cpu_ref
    data = b"".join(_corpus(case))
    r = cpu_ref.train_inc(data, case["vocab"], want_symbols=True, exact=case.get("exact", False))
    syms = np.ascontiguousarray(r["symbols"], dtype="<u4")
    return data, r["merges"], r["early_stop"], hashlib.sha256(syms.tobytes()).hexdigest(), int(syms.shape[0])


CASES = [
    ("en8m_w2", 2, dict(gen="english", bytes=8 << 20, seed=31, fracs=[0.45], vocab=8192)),
    ("en8m_exact_w3", 3, dict(gen="english", bytes=8 << 20, seed=32, fracs=[0.3, 0.55], vocab=6000, exact=True)),
    # C4-shaped at 64K ids (u32 symbols): independent multilingual shards, seams inside words
    ("ml3x4m_64k_w3", 3, dict(gen="ml_shards", shard=4 << 20, seeds=[5, 6, 7], vocab=65536)),
    # the headline's shape at N = 8: English's top count makes the zone
    # (5 x the summed top counts) longer than one eighth of the stream, so it spans
    # the tails of several pieces
    ("en8m_w8_zone_spans", 8, dict(gen="english", bytes=8 << 20, seed=33, fracs=[k / 8 for k in range(1, 8)],
                                   vocab=4096, spans=True)),
]


@pytest.mark.parametrize("name,world,case", CASES, ids=[c[0] for c in CASES])
def test_lexshard_matches_oracle(name, world, case):
    data, merges, early, sha, n = _expected(case)
    res = run_case(world, case)
    for r in range(world):
        assert res[r]["merges"] == [list(m) for m in merges], f"rank {r} merge list differs"
        assert res[r]["early"] == early
    assert sum(r["piece"] for r in res) == len(data)
    root = res[-1]
    assert root["final_n"] == n and root["final_sha256"] == sha
    assert root["root"]["sparse_exits"] == 0
    if case.get("spans"):
        zones = [row[4] for row in root["shapes"]]
        assert sum(1 for z in zones if z) >= 2, f"zone parts {zones}: the case no longer spans pieces"


def test_c4_shaped_fixture_world8():
    """C4 at a size the oracle holds: 8 ranks, one 128 MiB
    multilingual shard each (seeds 5..12), one 64K vocabulary over their
    concatenation — every merge and the final stream equal the fixture."""
    z = np.load(os.path.join(GOLD, "train_c4s8x128m.npz"), allow_pickle=False)
    want, meta = z["merges"], json.loads(str(z["meta"]))
    spec = meta["corpus"]
    case = dict(gen="ml_shards", shard=spec["shard"], seeds=spec["seeds"], vocab=meta["target_vocab"])
    res = run_case(8, case)
    for r in range(8):
        got = np.array(res[r]["merges"], dtype=np.uint32)
        assert got.shape == want.shape and np.array_equal(got, want), f"rank {r} merge list differs"
    assert sum(r["piece"] for r in res) == spec["shard"] * 8
    root = res[-1]
    assert root["final_n"] == meta["final_n"]
    assert root["final_sha256"] == meta["final_stream_sha256"]
    assert root["root"]["tail_dropped"] == meta["tail_total"]
