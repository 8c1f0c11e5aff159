# Session-29 check (one GPU call): the N>1 bench line rehearsed with 2 ranks
# sharing this GPU over gloo (host-staged hand-over), short run.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s29
mkdir -p $O
GBPE_BENCH_DEVICE=0 GBPE_SHARD_TRANSPORT=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29575 bench.py --gpus 2 --steps 2 --warmup 1 > $O/bench_n2.json 2> $O/bench_n2.err || { echo N2FAIL; tail -30 $O/bench_n2.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/s29/bench_n2.json').read().strip().splitlines()[-1]);print(d['value'], d['n_gpus'], d['ms_per_step'], d.get('scaling'), json.dumps(d.get('parity'))[:300], 'roofline' in d, 'cpu_baseline' in d)"
