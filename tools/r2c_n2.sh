# N=2 rehearsal of the driver's multi-GPU bench line on one GPU (both ranks on device 0, gloo process group)
set -e
export TMPDIR=/tmp
GBPE_BENCH_DEVICE=0 GBPE_SHARD_TRANSPORT=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 > gpurun_out/n2.json 2> gpurun_out/n2.err
