# Phase timeline of the sector-sparse kernels: bench.py's C2 train leg with the
# -DGBPE_KTRACE library (gpu-bpe_amd/lib/kt, see tools/build_variant.sh's recipe).
set -e
export TMPDIR=/tmp
GBPE_LIB=$PWD/gpu-bpe_amd/lib/kt/libgpubpe.so GBPE_KTRACE_OUT=/tmp/kt timeout -k 10 200 python bench.py --no-encode --no-cpu --no-kernel-timing > gpurun_out/kt_bench.json 2> gpurun_out/kt_bench.err
f=$(ls -t /tmp/kt.* | head -1)
python tools/ktrace_show.py $f > gpurun_out/ktrace.txt
