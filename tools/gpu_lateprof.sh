# Late-merge timeline of one 1 GiB English run (diagnostic, one GPU call):
# phase stamps of the -DGBPE_KTRACE build (lib/kt) and the kernel trace of the
# default library with paired launches on and off.   tools/gpu_lateprof.sh OUT [corpus]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
C=${2:-en1g}
mkdir -p $O
GBPE_LIB=$PWD/gpu-bpe_amd/lib/kt/libgpubpe.so GBPE_KTRACE_OUT=/tmp/kt EXPLORE_REPS=1 timeout -k 10 300 \
  python3 tools/explore_1g.py $C > $O/kt_run.txt 2>&1 || { echo KTFAIL; tail $O/kt_run.txt; exit 1; }
f=$(ls -t /tmp/kt.* | head -1)
EDGES=0,300,2000,8000,12000,16000,20000,24000,28000,33000 python3 tools/ktrace_show.py $f > $O/ktrace.txt && rm -f /tmp/kt.*
[ -n "$KT_ONLY" ] && { cat $O/ktrace.txt; exit 0; }
for v in 1 0; do
  GBPE_DEBUG=pair=$v EXPLORE_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p$v -o run -- \
    python3 tools/explore_1g.py $C > $O/p$v.txt 2>&1 || { echo PROFFAIL; tail $O/p$v.txt; exit 1; }
  python3 tools/ktrace_late.py $(find $O/p$v -name "*kernel_trace.csv" | head -1) 6000 > $O/late_p$v.txt
  find $O/p$v -name "*kernel_trace.csv" -delete
done
cat $O/ktrace.txt $O/late_p1.txt $O/late_p0.txt
