# C4 above 2^32 symbols on one GPU (8 ranks over gloo) with the root's phase
# timer, then the kernel timeline of C5's first 32 steps (4,096 merges)
set -e
export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out/r4c
GBPE_DEBUG=rtime=1 GBPE_BENCH_DEVICE=0 GBPE_SHARD_TRANSPORT=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29571 tools/c4_check.py > gpurun_out/r4c/c4_check.json 2> gpurun_out/r4c/c4_check.err
cat gpurun_out/r4c/c4_check.json
cd /tmp
EXPLORE_REPS=1 EXPLORE_MAX_STEPS=32 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/c5t -o run -- python3 $R/tools/explore_1g.py code1g > $R/gpurun_out/r4c/c5_trace.log 2>&1
EDGES=0,1,128,512,1024,2048,4096 python3 $R/tools/trace_timeline.py /tmp/c5t 400 > $R/gpurun_out/r4c/c5_first32_timeline.txt
head -40 $R/gpurun_out/r4c/c5_first32_timeline.txt
tail -8 $R/gpurun_out/r4c/c5_first32_timeline.txt
