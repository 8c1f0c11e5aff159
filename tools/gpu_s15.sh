# Session-15 diagnostic (one GPU call): the idle gaps between kernels of one full
# 1 GiB headline run under the kernel trace (is the host's enqueue ever behind?).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s15
mkdir -p $O
EXPLORE_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tg -o run -- python3 tools/explore_1g.py en1g > $O/tg.log 2>&1 || { echo TGFAIL; tail -20 $O/tg.log; exit 1; }
python3 tools/trace_gaps.py /tmp/tg > $O/gaps_en1g.txt 2>&1
cat $O/gaps_en1g.txt
