# Phase timeline of the sector-sparse kernels on a 1 GiB config (default en1g):
# tools/explore_1g.py with the -DGBPE_KTRACE library (tools/build_variant.sh work kt -DGBPE_KTRACE).
set -e
export TMPDIR=/tmp
C=${1:-en1g}
GBPE_HS=${GBPE_HS:-0} GBPE_LIB=$PWD/gpu-bpe_amd/lib/kt/libgpubpe.so GBPE_KTRACE_OUT=/tmp/kt timeout -k 10 300 python tools/explore_1g.py $C > gpurun_out/kt_$C.log 2>&1
f=$(ls -t /tmp/kt.* | head -1)
python tools/ktrace_show.py $f > gpurun_out/ktrace_$C.txt
