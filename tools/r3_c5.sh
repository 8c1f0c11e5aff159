# Round 3: C5 (1 GiB code, GPT-4 rule word starts, 50K) after the one-merge dense step + early lexicon entry
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/probe_webgpu.sh > gpurun_out/r3_webgpu_probe.txt 2>&1 || true
EXPLORE_REPS=2 timeout -k 10 300 python tools/explore_1g.py code1g en1g > gpurun_out/r3_c5_explore.log 2>&1
python - <<'PY' >> gpurun_out/r3_c5_explore.log
import numpy as np
for name in ("code1g", "en1g"):
    got = np.load(f"gpurun_out/explore_{name}_merges.npy")
    want = np.load(f"tests/golden/train_{name}.npz")["merges"]
    print(name, "merges equal fixture:", got.shape == want.shape and bool(np.array_equal(got, want)))
PY
