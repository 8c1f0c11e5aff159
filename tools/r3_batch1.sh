set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
SEL="lexshard" OUT=r3_gt_lex2 TLIM=400 bash tools/r3_gt.sh
timeout -k 10 300 python tools/explore_1g.py en1g code1g > gpurun_out/r3_explore.log 2>&1
python - <<'PY' >> gpurun_out/r3_explore.log
import numpy as np
for name in ("en1g", "code1g"):
    got = np.load(f"gpurun_out/explore_{name}_merges.npy"); want = np.load(f"tests/golden/train_{name}.npz")["merges"]
    print(name, "merges equal fixture:", got.shape == want.shape and bool(np.array_equal(got, want)))
PY
SKIP_N=1 C4SHARD=1073741824 TC4=500 bash tools/r3_rehearse.sh
