"""Debug: run one sharded case and print where the merge list departs from the oracle."""
import json
import os
import sys
sys.path[:0] = ["tests", "gpu-bpe_amd", "oracle"]
import bpe_oracle as O
from gpubpe import synth
import test_gpu_sharded as T

def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "ref_w2"
    case = dict([(c[0], (c[1], c[2])) for c in T.CASES])[name]
    world, cfg = case
    res, syms = T.run_case(world, cfg)
    data = synth.english(cfg["bytes"], seed=cfg["seed"])
    exp = O.train(data, cfg["vocab"], compaction="exact" if cfg["exact"] else "reference")
    for r in range(world):
        got = res[r]["merges"]
        k = next((i for i, (x, y) in enumerate(zip(got, exp["merges"])) if x != y), None)
        print("rank", r, "merges", len(got), "exp", len(exp["merges"]), "first diff", k, "sparse merges", res[r]["sparse_merges"],
              "stalls", res[r]["stalls"])
        if k is not None:
            print("  got", got[max(0, k - 2):k + 3])
            print("  exp", exp["merges"][max(0, k - 2):k + 3])


if __name__ == "__main__":
    main()
