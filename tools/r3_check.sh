# quick parity + timing check of the 1 GiB configurations (explore_1g: full runs, merges vs fixtures)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
EXPLORE_REPS=${REPS:-2} timeout -k 10 ${TL:-400} python tools/explore_1g.py ${CFGS:-en1g code1g} > gpurun_out/r3_check.log 2>&1
python - <<'PY' >> gpurun_out/r3_check.log
import numpy as np, os, json
for name in os.environ.get("CFGS", "en1g code1g").split():
    got = np.load(f"gpurun_out/explore_{name}_merges.npy"); want = np.load(f"tests/golden/train_{name}.npz")["merges"]
    print(name, "merges equal fixture:", got.shape == want.shape and bool(np.array_equal(got, want)))
PY
python - <<'PY' >> gpurun_out/r3_check.log
import json
for l in open("gpurun_out/r3_check.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["name"], d["rep"], "create %.3f loop %.3f total/s %.0f first10 %s by32 %s" % (d["create_s"], d["loop_s"], d["merges_per_s_total"], d["step_ms_first10"], d["step_ms_by_32"][:4]))
PY
