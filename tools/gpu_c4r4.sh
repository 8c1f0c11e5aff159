# C4 leg's self-check rehearsed with 4 ranks sharing this one GPU over gloo
# (host-staged hand-over; GBPE_C4R4_SHARD bytes per rank, 128 MiB by default, 1 GiB for a 2^32-symbol stream), after the 2-rank close run.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/c4r4
SH=${GBPE_C4R4_SHARD:-134217728}
mkdir -p $O
GBPE_BENCH_DEVICE=0 GBPE_SHARD_TRANSPORT=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29574 bench.py --gpus 4 --c4-only --c4-shard $SH > $O/c4_rehearsal_4r_$SH.json 2> $O/c4_rehearsal_4r_$SH.err || { echo C4FAIL; tail -30 $O/c4_rehearsal_4r_$SH.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/c4r4/c4_rehearsal_4r_'+__import__('os').environ.get('GBPE_C4R4_SHARD','134217728')+'.json').read().strip().splitlines()[-1]);c=d['c4'];print('c4', c['value'], c.get('counts_equal_recount'), c['timing_s_max_over_ranks'], str(c.get('check'))[:500])"
