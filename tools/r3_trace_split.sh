# kernel timeline of the first EXPLORE steps of $CFG with the split-tail diagnostic library
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && env ${LIBV:+GBPE_LIB=$R/gpu-bpe_amd/lib/$LIBV/libgpubpe.so} EXPLORE_MAX_STEPS=${STEPS:-3} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tls -o run -- python3 $R/tools/explore_1g.py ${CFG:-en1g} > /tmp/tls.log 2>&1
cd $R && mkdir -p gpurun_out && python tools/trace_timeline.py /tmp/tls ${NFIRST:-300} > gpurun_out/r3_split_${CFG:-en1g}.txt 2> gpurun_out/r3_split_err.txt
