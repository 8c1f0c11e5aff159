# Session-9 diagnostic (one GPU call): k_lx_hash workgroup count (GBPE_DEBUG lxwg:
# 65536 ~ the old 16 words per thread; 16384; 4096 = default; 1024) with the
# batched symbol loads — the first en1g step under the kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s9
mkdir -p $O
for w in 65536 16384 4096 1024; do
  GBPE_DEBUG=lxwg=$w EXPLORE_MAX_STEPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lx_$w -o run -- python3 tools/explore_1g.py en1g > $O/lx_$w.log 2>&1 || { echo FAIL $w; tail -20 $O/lx_$w.log; exit 1; }
  f=$(find /tmp/lx_$w -name "*kernel_stats.csv" | head -1)
  echo "== lxwg $w" >> $O/lx_stats.txt
  grep -E "k_lx" $f >> $O/lx_stats.txt
  grep -h '"merges"' $O/lx_$w.log | cut -c1-200 >> $O/lx_stats.txt
done
