# Session-16 diagnostic (one GPU call): host enqueue vs wait per training step
# (GBPE_DEBUG=htime=1), 1 GiB headline and C2, no profiler attached.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s16
mkdir -p $O
GBPE_DEBUG=htime=1 EXPLORE_REPS=1 timeout -k 10 300 python3 tools/explore_1g.py en1g c2 > $O/htime.log 2>&1 || { echo HTFAIL; tail -20 $O/htime.log; exit 1; }
grep -E "htime|loop_s" $O/htime.log | cut -c1-400
