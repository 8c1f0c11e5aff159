# Round-5 final check of the committed tree (one GPU call): the -m gpu suite,
# smoke() and the default bench line, as the driver runs them at round end.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo TESTFAIL; tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail -30 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/final/bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["reference_rate"], d["parity"], d["train_detail"].get("run_s"))
for k in ("c1", "c2", "c4_shard", "c5"):
    print(k, d[k]["value"], d[k].get("merges_equal_fixture"))
t = d["tokenize"]
print("tok", t["gbps_kernels"], t.get("fixture_tokens_equal"))
PY
