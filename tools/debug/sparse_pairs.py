"""Debug: which live pair counts differ from a recount after sparse-early runs (repeated)."""
import sys
sys.path[:0] = ["tests", "gpu-bpe_amd", "oracle"]
import numpy as np
import bpe_oracle as O
from gpubpe import BPEEngine, synth
from test_gpu_parity import _train_native

eng = BPEEngine(0).init()
data = synth.english(65536, seed=65536 % 97 + 3)
ref = O.train(data, 1024)
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    m, s, pairs, st = _train_native(eng, data, 1024, batch=16, sparse="early")
    up, uc = O.count_pairs(s.astype(np.uint32))
    got = dict(zip(pairs[0].tolist(), pairs[1].tolist()))
    want = dict(zip(up.tolist(), uc.tolist()))
    diff = [(k, got.get(k, 0), want.get(k, 0)) for k in set(got) | set(want) if got.get(k, 0) != want.get(k, 0)]
    print("iter", it, "merges_ok", m == ref["merges"], "syms_ok", np.array_equal(s, ref["symbols"]), "ndiff", len(diff),
          "tail", st.tail_dropped, sum(ref["tail_drops"]), flush=True)
    mset = {(a << 16) | b: i for i, (a, b, _, _) in enumerate(m)}
    for k, g, w in sorted(diff)[:10]:
        print(f"  pid {k >> 16},{k & 0xFFFF}  table {g}  recount {w}  merged_at {mset.get(k)}")
