# Session-1 check (one GPU call): A/B of the round-4 library (base) against this
# tree's (in-launch close + pool + blocked signatures; "spread" = the old signature
# layout; close=0 = k_refresh after every merge), then the whole GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s1
mkdir -p $O
L=gpu-bpe_amd/lib
AB_REPS=2 AB_ROUNDS=2 timeout -k 10 600 python -u tools/ab_libs.py $L/base/libgpubpe.so $L/libgpubpe.so $L/spread/libgpubpe.so "$L/libgpubpe.so:GBPE_DEBUG=close=0" -- en1g c2 code1g > $O/ab.txt 2>&1 || { echo ABFAIL; tail -30 $O/ab.txt; exit 1; }
tail -12 $O/ab.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo SUITEFAIL; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
