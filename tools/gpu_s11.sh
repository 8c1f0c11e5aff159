# Session-11 check (one GPU call): LDS delta tables of up to 16 slots per thread
# compacted before the flush, whose probes then go out in one batch (the late
# 256-thread forms took two round trips): A/B against lib/pre3 (fixtures checked), the phase
# stamps of the new build (lib/kt), then the GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s11
mkdir -p $O
L=gpu-bpe_amd/lib
AB_REPS=2 AB_ROUNDS=2 timeout -k 10 600 python -u tools/ab_libs.py $L/pre3/libgpubpe.so $L/libgpubpe.so -- en1g c2 code1g > $O/ab.txt 2>&1 || { echo ABFAIL; tail -30 $O/ab.txt; exit 1; }
tail -8 $O/ab.txt
GBPE_LIB=$PWD/$L/kt/libgpubpe.so GBPE_KTRACE_OUT=/tmp/kt_en1g timeout -k 10 300 python -u tools/explore_1g.py en1g > $O/kt_en1g.log 2>&1 || { echo KTFAIL; tail -20 $O/kt_en1g.log; exit 1; }
f=$(ls -t /tmp/kt_en1g.* | head -1)
python tools/ktrace_show.py $f > $O/ktrace_en1g.txt
cat $O/ktrace_en1g.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo SUITEFAIL; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
