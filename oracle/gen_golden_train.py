#!/usr/bin/env python3
"""Full-length training and encode fixtures for the GPU parity tests — TEST
INFRASTRUCTURE ONLY (run here, on the CPU; the outputs are committed under
tests/golden/ and read by tests/test_gpu_full.py on the GPU box).

Each training fixture holds the complete merge list ([a, b, id, count] per
merge), the final stream length, the stale-tail total, and the sha256 of the
final symbol stream (u32 little-endian, reference layout: bit 16 = word
start), produced by the incremental restatement oracle/bpe_oracle_inc.c
(itself checked merge-for-merge against the full-recount restatement
oracle/bpe_oracle.c by tests/test_oracle_inc.py).  The corpus sha256 is
stored too, so a drift of numpy's generators on the GPU box fails loudly
instead of comparing different inputs.

    python oracle/gen_golden_train.py [name ...]     (default: all)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [HERE, os.path.join(ROOT, "gpu-bpe_amd")]

import numpy as np  # noqa: E402

import bpe_oracle as O  # noqa: E402
import cpu_ref  # noqa: E402
from gpubpe import synth  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")

# name -> (corpus spec, target vocab, boundary source[, compaction]); compaction "reference"
# (default: the quirk of train.wgsl:605-607 + 698/727) or "exact"
TRAIN = {
    # C1 (BASELINE configs[0]): 256 KiB ASCII English, seed 1, 1K vocab (768 merges)
    "c1": ({"gen": "english", "n": 262_144, "seed": 1}, 1024, "heuristic"),
    "c1x": ({"gen": "english", "n": 262_144, "seed": 1}, 1024, "heuristic", "exact"),
    # C2, exactly the bench's secondary leg (bench.py train_leg)
    "c2": ({"gen": "english", "n": 104_857_600, "seed": 2, "fancy_punct": 0.005}, 32768, "heuristic"),
    # headline: 1 GiB English-like UTF-8 @ 32K (BASELINE.json metric)
    "en1g": ({"gen": "english", "n": 1 << 30, "seed": 2, "fancy_punct": 0.005}, 32768, "heuristic"),
    # C5: 1 GiB code, 50K vocab, GPT-4 rule word starts (pre_tokenizer.mjs:226-292), u32 symbols
    "code1g": ({"gen": "code", "n": 1 << 30, "seed": 6}, 50000, "gpt4"),
    # C3's vocab: 32K trained on a 100 MiB multilingual sample (seed 4)
    "c3vocab": ({"gen": "multilingual", "n": 104_857_600, "seed": 4}, 32768, "heuristic"),
    # 1 GiB multilingual @ 32K (the C3/C4 text model)
    "ml1g": ({"gen": "multilingual", "n": 1 << 30, "seed": 3}, 32768, "heuristic"),
    # C4's rank-0 shard (8 x 1 GiB multilingual, seed 5 + rank) trained
    # alone at C4's 64K vocab (u32 symbols: ids reach 0xFFFF, the stop of train.wgsl:345)
    "ml1g64k": ({"gen": "multilingual", "n": 1 << 30, "seed": 5}, 65536, "heuristic"),
    # C4-shaped at a size the oracle holds: 8 shards x 128 MiB multilingual, seeds 5..12,
    # concatenated in rank order, 64K vocab, heuristic word starts of the concatenated stream
    "c4s8x128m": ({"gen": "ml_shards", "shard": 128 << 20, "seeds": list(range(5, 13))}, 65536, "heuristic"),
}
# name -> (text spec, vocab fixture)
ENCODE = {
    "c3enc64m": ({"gen": "multilingual", "n": 64 << 20, "seed": 3}, "c3vocab"),
    "c3enc1g": ({"gen": "multilingual", "n": 1 << 30, "seed": 3}, "c3vocab"),
}


def corpus(spec: dict) -> bytes:
    g = spec["gen"]
    if g == "english":
        return synth.english(spec["n"], seed=spec["seed"], fancy_punct=spec.get("fancy_punct", 0.0))
    if g == "multilingual":
        return synth.multilingual(spec["n"], seed=spec["seed"])
    if g == "code":
        return synth.code(spec["n"], seed=spec["seed"])
    if g == "ml_shards":
        return b"".join(synth.multilingual(spec["shard"], seed=sd) for sd in spec["seeds"])
    raise ValueError(g)


def sha(b) -> str:
    return hashlib.sha256(b).hexdigest()


def gen_train(name: str):
    spec, vocab, bnd = TRAIN[name][:3]
    compaction = TRAIN[name][3] if len(TRAIN[name]) > 3 else "reference"
    t = time.time()
    data = corpus(spec)
    ws = cpu_ref.gpt4_word_starts_ascii(data) if bnd == "gpt4" else None
    r = cpu_ref.train_inc(data, vocab, word_starts=ws, want_symbols=True, exact=compaction == "exact")
    syms = np.ascontiguousarray(r["symbols"], dtype="<u4")
    meta = {"name": name, "corpus": spec, "corpus_sha256": sha(data), "target_vocab": vocab, "boundaries": bnd,
            "compaction": compaction,
            "final_n": r["final_n"], "tail_total": r["tail_total"], "early_stop": r["early_stop"],
            "final_stream_sha256": sha(syms.tobytes()), "n_merges": len(r["merges"]),
            "generator": "oracle/bpe_oracle_inc.c (oracle/gen_golden_train.py)"}
    np.savez_compressed(os.path.join(GOLD, f"train_{name}.npz"), merges=np.array(r["merges"], dtype=np.uint32),
                        meta=np.array(json.dumps(meta)))
    print(f"{name}: {len(r['merges'])} merges, final_n {r['final_n']}, {time.time() - t:.0f}s", flush=True)


def load_train(name: str):
    z = np.load(os.path.join(GOLD, f"train_{name}.npz"), allow_pickle=False)
    return z["merges"], json.loads(str(z["meta"]))


def gen_encode(name: str):
    spec, vname = ENCODE[name]
    t = time.time()
    merges, _ = load_train(vname)
    voc = O.vocab_from_merges([m[:3] for m in merges.tolist()])
    blob = O.compile_vocab_to_trie(voc.entries)
    hdr = O.parse_header(blob)
    nodes, edges = O.parse_trie_buffers(blob, hdr)
    cs = O.adaptive_chunk_size(hdr["maxTokenLen"])
    text = corpus(spec)
    tok = np.ascontiguousarray(cpu_ref.encode(text, nodes, edges, cs), dtype="<u4")
    meta = {"name": name, "corpus": spec, "corpus_sha256": sha(text), "vocab": vname, "chunk_size": cs,
            "trie_sha256": sha(blob), "n_tokens": int(tok.shape[0]), "tokens_sha256": sha(tok.tobytes()),
            "first_tokens": tok[:64].tolist(), "generator": "oracle/bpe_oracle.c oracle_encode (gen_golden_train.py)"}
    with open(os.path.join(GOLD, f"encode_{name}.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"{name}: {tok.shape[0]} tokens, cs {cs}, {time.time() - t:.0f}s", flush=True)


def main():
    names = sys.argv[1:] or list(TRAIN) + list(ENCODE)
    for nm in names:
        if nm in TRAIN:
            gen_train(nm)
        else:
            gen_encode(nm)


if __name__ == "__main__":
    main()
