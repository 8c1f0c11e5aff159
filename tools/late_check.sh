# k_late v2 on the GPU: the whole -m gpu suite with the late loop on, A/B against
# the two-launch form (c2, en1g), then phase stamps of a KTRACE build
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
GBPE_DEBUG=late=1 timeout -k 10 560 python -u -m pytest ${SUITE:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_late3_suite.txt 2>&1 || { tail -30 gpurun_out/r4_late3_suite.txt; exit 1; }
tail -3 gpurun_out/r4_late3_suite.txt
AB_REPS=1 AB_ROUNDS=1 timeout -k 10 360 python -u tools/ab_libs.py gpu-bpe_amd/lib/libgpubpe.so:GBPE_DEBUG=late=1 gpu-bpe_amd/lib/libgpubpe.so -- c2 en1g > gpurun_out/r4_late3_ab.txt 2>&1
tail -12 gpurun_out/r4_late3_ab.txt
GBPE_DEBUG=late=1 GBPE_LIB=$PWD/gpu-bpe_amd/lib/kt/libgpubpe.so GBPE_KTRACE_OUT=/tmp/ktl AB_REPS=1 AB_ROUNDS=1 timeout -k 10 200 python -u tools/ab_libs.py gpu-bpe_amd/lib/kt/libgpubpe.so:GBPE_DEBUG=late=1 -- en1g > gpurun_out/r4_late3_kt.txt 2>&1
f=$(ls -S /tmp/ktl.* | head -1)
python tools/ktrace_late.py $f > gpurun_out/r4_late3_ktrace.txt
cat gpurun_out/r4_late3_ktrace.txt
