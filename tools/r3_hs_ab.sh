# A/B of the hand-off selection (GBPE_HS) on the 1 GiB configs: parity vs fixtures + timing
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for hs in ${HSV:-1 0}; do
  GBPE_HS=$hs GBPE_HS_STATS=1 EXPLORE_REPS=${REPS:-1} timeout -k 10 ${TL:-300} python tools/explore_1g.py ${CFGS:-en1g code1g} > gpurun_out/r3_hs$hs.log 2>&1
  python - $hs <<'PY' >> gpurun_out/r3_hs_ab.txt
import numpy as np, os, json, sys
hs = sys.argv[1]
for l in open(f"gpurun_out/r3_hs{hs}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        got = np.load(f"gpurun_out/explore_{d['name']}_merges.npy"); want = np.load(f"tests/golden/train_{d['name']}.npz")["merges"]
        print("HS", hs, d["name"], d["rep"], "equal", got.shape == want.shape and bool(np.array_equal(got, want)),
              "loop %.3f total/s %.0f first10 %s by32 %s" % (d["loop_s"], d["merges_per_s_total"], d["step_ms_first10"], d["step_ms_by_32"]))
    elif "hand-off" in l:
        print("HS", hs, l.strip())
PY
done
