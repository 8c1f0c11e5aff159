# Session-5 measurement (one GPU call): kernel timelines of en1g's early phase —
# the first step (sparse entry + 128 merges) and the first 32 steps (4,096
# merges) — to split the first step's 64 ms.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s5
mkdir -p $O
for ms in 1 32; do
  EXPLORE_MAX_STEPS=$ms timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tl_$ms -o tl -- python3 tools/explore_1g.py en1g > $O/explore_en1g_$ms.log 2>&1 || { echo TLFAIL; tail -20 $O/explore_en1g_$ms.log; exit 1; }
  python3 tools/trace_timeline.py /tmp/tl_$ms 400 > $O/en1g_timeline_steps$ms.txt
  head -45 $O/en1g_timeline_steps$ms.txt
done
