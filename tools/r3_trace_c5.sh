# kernel timeline of C5's first steps (one run, EXPLORE_MAX_STEPS steps)
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && EXPLORE_MAX_STEPS=${STEPS:-3} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tl -o run -- python3 $R/tools/explore_1g.py ${CFG:-code1g} > /tmp/tl.log 2>&1
cd $R && mkdir -p gpurun_out && python tools/trace_timeline.py /tmp/tl ${NFIRST:-400} > gpurun_out/r3_timeline_${CFG:-code1g}.txt
tail -2 /tmp/tl.log >> gpurun_out/r3_timeline_${CFG:-code1g}.txt
