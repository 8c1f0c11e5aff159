# Round-5 closing measurements (one GPU call): smoke(), the en1g profiles (kernel
# durations + k_body PMC traffic) copied into profiles/r5/close/ where bench.py
# reads them, the default bench line, then the C4 leg's self-check rehearsed with
# 2 ranks sharing this GPU over gloo.  (The -m gpu suite runs in its own call.)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/close
mkdir -p $O profiles/r5/close
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
OUT=close bash tools/profile_r5.sh || { echo PROFFAIL; exit 1; }
cp $O/en1g_kernel_stats.csv $O/pmc_kbody.json profiles/r5/close/
python tools/prof_summary.py /tmp/ks > $O/en1g_summary.txt 2>&1 || true
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail -30 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/close/bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["reference_rate"], d["parity"])
print("floor", json.dumps(d["roofline"].get("latency_floor"))[:600])
for k in ("c1", "c2", "c4_shard", "c5"):
    print(k, d[k]["value"], d[k].get("merges_equal_fixture"))
t = d["tokenize"]
print("tok", t["gbps_kernels"], t["ms_walk"], t["ms_compact"], t.get("fixture_tokens_equal"))
PY
GBPE_BENCH_DEVICE=0 GBPE_SHARD_TRANSPORT=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29573 bench.py --gpus 2 --c4-only --c4-shard 134217728 > $O/c4_rehearsal_2r.json 2> $O/c4_rehearsal_2r.err || { echo C4FAIL; tail -30 $O/c4_rehearsal_2r.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/close/c4_rehearsal_2r.json').read().strip().splitlines()[-1]);c=d['c4'];print('c4', c['value'], c.get('counts_equal_recount'), json.dumps(c.get('check'))[:400])"
