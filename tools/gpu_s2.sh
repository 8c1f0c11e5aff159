# Session-2 check (one GPU call): the default bench line, the C4 leg's self-check
# rehearsed with 2 ranks sharing this GPU over gloo, then the round-5 profiles
# (kernel durations + k_body PMC traffic of one en1g run).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s2
mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail -30 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/s2/bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["reference_rate"], d["parity"])
print("floor", json.dumps(d["roofline"].get("latency_floor"))[:600])
for k in ("c1", "c2", "c4_shard", "c5"):
    print(k, d[k]["value"], d[k].get("merges_equal_fixture"))
t = d["tokenize"]
print("tok", t["gbps_kernels"], t["ms_walk"], t["ms_compact"], t.get("fixture_tokens_equal"))
PY
GBPE_BENCH_DEVICE=0 GBPE_SHARD_TRANSPORT=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29573 bench.py --gpus 2 --c4-only --c4-shard 134217728 > $O/c4_rehearsal_2r.json 2> $O/c4_rehearsal_2r.err || { echo C4FAIL; tail -30 $O/c4_rehearsal_2r.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/s2/c4_rehearsal_2r.json').read().strip().splitlines()[-1]);c=d['c4'];print('c4', c['value'], c.get('counts_equal_recount'), json.dumps(c.get('check'))[:400])"
OUT=s2/prof bash tools/profile_r5.sh
python tools/prof_summary.py /tmp/ks > $O/prof/en1g_summary.txt 2>&1 || true
tail -1 $O/prof/pmc_kbody.json
