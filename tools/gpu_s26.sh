# Session-26 check (one GPU call): zone segments load their stale-tail positions
# four at a time, both symbols before use (one round trip, not two per position): A/B against the
# lexicon-build library (lib/pre6, merges checked against the fixtures), the phase
# stamps of the new build (lib/kt), then the GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s26
mkdir -p $O
L=gpu-bpe_amd/lib
AB_REPS=2 AB_ROUNDS=2 timeout -k 10 600 python -u tools/ab_libs.py $L/pre6/libgpubpe.so $L/libgpubpe.so -- en1g c2 code1g ml1g64k > $O/ab.txt 2>&1 || { echo ABFAIL; tail -30 $O/ab.txt; exit 1; }
tail -8 $O/ab.txt
GBPE_LIB=$PWD/$L/kt/libgpubpe.so GBPE_KTRACE_OUT=/tmp/kt_en1g timeout -k 10 300 python -u tools/explore_1g.py en1g > $O/kt_en1g.log 2>&1 || { echo KTFAIL; tail -20 $O/kt_en1g.log; exit 1; }
f=$(ls -t /tmp/kt_en1g.* | head -1)
python tools/ktrace_show.py $f > $O/ktrace_en1g.txt
cat $O/ktrace_en1g.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo SUITEFAIL; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
