"""One input encoded across ranks (gpubpe.split_encode) over gloo,
world size 2 and 3 on the CPU: chunk-aligned slices, the exclusive scan of the
slice totals and the gather must give exactly the single-pass tokens of the
reference's chunked walk (the CPU restatement stands in for each rank's GPU)."""
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
from gpubpe.split_encode import slice_bounds  # noqa: E402
from dist_util import free_port as _free_port  # noqa: E402


def _setup():
    vocab = O.vocab_from_merges(O.train(synth.multilingual(30000, seed=51), 700, compaction="exact")["merges"]).entries
    blob = O.compile_vocab_to_trie(vocab)
    nodes, edges = O.parse_trie_buffers(blob, O.parse_header(blob))
    return nodes, edges


def _worker(rank, world, port, case, outdir):
    import torch.distributed as dist
    from gpubpe.split_encode import encode_split
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        nodes, edges = _setup()
        text = synth.multilingual(case["bytes"], seed=52)
        cs = case["cs"]
        toks, offs, cnts = encode_split(lambda b: O.encode_chunked(b, nodes, edges, cs), text, cs, dist,
                                        gather_to=case["gather_to"])
        res = {"offsets": offs, "counts": cnts, "tokens": None if toks is None else toks.tolist()}
        with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
            json.dump(res, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nbytes,cs,gather_to", [(2, 20000, 512, 0), (3, 20000, 64, None), (3, 700, 512, 2),
                                                      (2, 9999, 7, 1)])
def test_split_encode_matches_single_pass(world, nbytes, cs, gather_to):
    import torch.multiprocessing as mp
    nodes, edges = _setup()
    text = synth.multilingual(nbytes, seed=52)
    want = O.encode_chunked(text, nodes, edges, cs).tolist()
    case = {"bytes": nbytes, "cs": cs, "gather_to": gather_to}
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), case, d), nprocs=world, join=True)
        res = [json.load(open(os.path.join(d, f"r{r}.json"))) for r in range(world)]
    for r in range(world):
        if gather_to is None or r == gather_to:
            assert res[r]["tokens"] == want, r
        else:
            assert res[r]["tokens"] is None
        assert sum(res[r]["counts"]) == len(want)
    # each slice's tokens sit at its scanned offset
    b = slice_bounds(nbytes, cs, world)
    for q, (s, e) in enumerate(b):
        assert O.encode_chunked(text[s:e], nodes, edges, cs).tolist() == want[res[0]["offsets"][q]:
                                                                             res[0]["offsets"][q] + res[0]["counts"][q]]


def test_slice_bounds_chunk_aligned():
    for n, cs, w in ((0, 512, 3), (1, 512, 2), (5000, 7, 4), (1 << 20, 512, 8), (513, 512, 8)):
        b = slice_bounds(n, cs, w)
        assert len(b) == w and b[0][0] == 0 and b[-1][1] == n
        for (s0, e0), (s1, _) in zip(b, b[1:]):
            assert e0 == s1 and s1 % cs == 0 or s1 == n
