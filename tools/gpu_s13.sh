# Session-13 check (one GPU call): k_refresh taking up to 256 table blocks per
# workgroup in late steps (C5's late grid 2048 -> 512 workgroups, so 512 partial
# maxima per selection): A/B against the previous library (lib/pre4, fixtures
# checked), the C5 phase stamps of the new build (lib/kt), then the GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s13
mkdir -p $O
L=gpu-bpe_amd/lib
AB_REPS=2 AB_ROUNDS=2 timeout -k 10 600 python -u tools/ab_libs.py $L/pre4/libgpubpe.so $L/libgpubpe.so -- code1g en1g c2 > $O/ab.txt 2>&1 || { echo ABFAIL; tail -30 $O/ab.txt; exit 1; }
tail -8 $O/ab.txt
GBPE_LIB=$PWD/$L/kt/libgpubpe.so GBPE_KTRACE_OUT=/tmp/kt_code1g timeout -k 10 300 python -u tools/explore_1g.py code1g > $O/kt_code1g.log 2>&1 || { echo KTFAIL; tail -20 $O/kt_code1g.log; exit 1; }
f=$(ls -t /tmp/kt_code1g.* | head -1)
python tools/ktrace_show.py $f > $O/ktrace_code1g.txt
cat $O/ktrace_code1g.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo SUITEFAIL; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
