# kernel timelines of the first steps of code1g and en1g (production library)
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for C in ${CFGS:-code1g en1g}; do
  cd /tmp && EXPLORE_MAX_STEPS=${STEPS:-2} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tl_$C -o run -- python3 $R/tools/explore_1g.py $C > /tmp/tl_$C.log 2>&1
  cd $R && EDGES=${EDGES:-0,1,16,32,64,128,256} python tools/trace_timeline.py /tmp/tl_$C ${NFIRST:-400} > gpurun_out/r3_first_${C}.txt 2>> gpurun_out/r3_first_err.txt
done
