# Round 3: multi-GPU bench lines rehearsed on ONE GPU (every rank on device 0, gloo transport)
#   N=${N:-2} headline line (lexicon hand-over), and the C4 leg with ${C4N:-8} ranks x ${C4SHARD} bytes
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${SKIP_N:-0}" = 0 ]; then
GBPE_BENCH_DEVICE=0 GBPE_SHARD_TRANSPORT=gloo timeout -k 10 ${TN:-420} python -m torch.distributed.run --nnodes=1 --nproc-per-node ${N:-2} --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus ${N:-2} --steps ${STEPS:-3} --warmup 1 ${NARGS} > gpurun_out/r3_n${N:-2}.json 2> gpurun_out/r3_n${N:-2}.err
fi
if [ -n "${C4SHARD}" ]; then
GBPE_BENCH_DEVICE=0 GBPE_SHARD_TRANSPORT=gloo timeout -k 10 ${TC4:-420} python -m torch.distributed.run --nnodes=1 --nproc-per-node ${C4N:-8} --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus ${C4N:-8} --c4-only --c4-shard ${C4SHARD} > gpurun_out/r3_c4_${C4N:-8}x${C4SHARD}.json 2> gpurun_out/r3_c4_${C4N:-8}x${C4SHARD}.err
fi
