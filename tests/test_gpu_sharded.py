"""Sharded training through the C-ABI on the GPU (world size 2 and 3 sharing
one MI355X, gloo with host-staged records): merge lists and the concatenated
final stream equal the single-stream oracle (reference semantics)."""
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
    from gpubpe.sharded import GpuShardBackend, ShardedTrainer
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = _lib.load()
    ctx = C.c_void_p()
    _lib.check(lib.gbpe_ctx_create(0, C.byref(ctx)), ctx, "ctx")
    try:
        torch.cuda.set_device(0)
        data = synth.english(case["bytes"], seed=case["seed"])
        shards, _ = cut_at_word_starts(data, case["fracs"])
        d, ws = shards[rank]
        be = GpuShardBackend(lib, ctx, d, ws, rank, world, case["vocab"], exact=case["exact"],
                             table_log2=16, cap_extra=len(data), stream=torch.cuda.current_stream().cuda_stream)
        assert lib.gbpe_ctx_get_stream(ctx) == (torch.cuda.current_stream().cuda_stream or None)
        tr = ShardedTrainer(be, dist, device="cuda", staged=True, cap_list=case["cap"], cap_win=case["cap"])
        tr.setup()
        merges, early = tr.train(case["vocab"], batch=case.get("batch", 128))
        np.save(os.path.join(outdir, f"sym{rank}.npy"), be.symbols())
        with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
            json.dump({"merges": merges, "early": early, "stalls": tr.stalls}, f)
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


CASES = [
    ("ref_w2", 2, dict(bytes=60_000, seed=21, fracs=[0.5], vocab=700, exact=False, cap=1 << 14)),
    ("exact_w2", 2, dict(bytes=60_000, seed=22, fracs=[0.5], vocab=700, exact=True, cap=1 << 14)),
    ("ref_w3_tiny_middle", 3, dict(bytes=20_000, seed=13, fracs=[0.945, 0.965], vocab=480, exact=False,
                                   cap=1 << 14)),
    ("ref_w2_stalls", 2, dict(bytes=16_000, seed=14, fracs=[0.6], vocab=420, exact=False, cap=8, batch=32)),
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
