# Session-17 diagnostic (one GPU call): the merge period inside a step against
# the merge's own chain (ktrace build), with the host's enqueue/wait split.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s17
mkdir -p $O
for rep in 1 2; do
  GBPE_DEBUG=htime=1 GBPE_LIB=$PWD/gpu-bpe_amd/lib/kt/libgpubpe.so GBPE_KTRACE_OUT=/tmp/kt_en1g_$rep timeout -k 10 300 python -u tools/explore_1g.py en1g > $O/kt_en1g_$rep.log 2>&1 || { echo KTFAIL; tail -20 $O/kt_en1g_$rep.log; exit 1; }
  f=$(ls -t /tmp/kt_en1g_$rep.* | head -1)
  python tools/ktrace_show.py $f > $O/ktrace_en1g_$rep.txt
  grep -h htime $O/kt_en1g_$rep.log | cut -c1-300
  grep -o '"loop_s": [0-9.]*' $O/kt_en1g_$rep.log
  cat $O/ktrace_en1g_$rep.txt
done
