# the split-tail trace for several diagnostic libraries in one call: $LIBS = "split diag1 diag2"
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for L in ${LIBS:-split}; do
  cd /tmp && GBPE_LIB=$R/gpu-bpe_amd/lib/$L/libgpubpe.so EXPLORE_MAX_STEPS=${STEPS:-3} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tl_$L -o run -- python3 $R/tools/explore_1g.py ${CFG:-en1g} > /tmp/tl_$L.log 2>&1 || echo "$L: run failed (diagnostic builds may stop early)" >> $R/gpurun_out/r3_diag_notes.txt
  cd $R && python tools/trace_timeline.py /tmp/tl_$L 5 > gpurun_out/r3_diag_${CFG:-en1g}_$L.txt 2>&1 || true
done
