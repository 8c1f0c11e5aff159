# Final checks of the round (one GPU call): the whole -m gpu suite, smoke(), the default bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/closing
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo SUITEFAIL; tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail -20 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/closing/bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["parity"])
for k in ("c1", "c2", "c4_shard", "c5"):
    print(k, d[k]["value"], d[k].get("merges_equal_fixture"))
t = d["tokenize"]
print("tok", t["gbps_kernels"], t["ms_walk"], t["ms_compact"], t.get("fixture_tokens_equal"))
print("cpu_inc", d["c2"].get("cpu_incremental"))
PY
