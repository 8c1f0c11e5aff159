"""One input encoded by two ranks sharing one MI355X (gloo, host-staged), each
rank's slice through the C-ABI trie walk: the gathered tokens equal one device
pass and the CPU oracle (gpubpe.split_encode)."""
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

pytestmark = pytest.mark.gpu


def _vocab():
    return O.vocab_from_merges(O.train(synth.multilingual(60000, seed=61), 1000, compaction="exact")["merges"]).entries


def _worker(rank, world, port, nbytes, outdir):
    import torch.distributed as dist
    from gpubpe import BPEEngine, TrieTokenizer
    from gpubpe.split_encode import encode_split
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = BPEEngine(0).init()
        tok = TrieTokenizer.from_vocab(eng, _vocab())
        text = synth.multilingual(nbytes, seed=62)
        toks, offs, cnts = encode_split(tok.encode_bytes, text, tok.chunk_size, dist, gather_to=0)
        with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
            json.dump({"tokens": None if toks is None else toks.tolist(), "cs": tok.chunk_size}, f)
        tok.destroy()
    finally:
        dist.destroy_process_group()


def test_split_encode_two_ranks_one_gpu():
    import torch.multiprocessing as mp
    nbytes = 300_000
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), nbytes, d), nprocs=2, join=True)
        res = [json.load(open(os.path.join(d, f"r{r}.json"))) for r in range(2)]
    vocab = _vocab()
    blob = O.compile_vocab_to_trie(vocab)
    nodes, edges = O.parse_trie_buffers(blob, O.parse_header(blob))
    text = synth.multilingual(nbytes, seed=62)
    want = O.encode_chunked(text, nodes, edges, res[0]["cs"]).tolist()
    assert res[0]["tokens"] == want
    assert res[1]["tokens"] is None
