# Session-1 check 2 (one GPU call): A/B of the round-4 library (base) against this
# tree (pool + blocked signatures; spread = the old signature layout; gused/glive =
# the pair-table growth rule that keeps C5 in 2^24 slots), then the GPU suite with
# every pooled block poisoned (no buffer may rely on a fresh allocation's contents).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s1c
mkdir -p $O
L=gpu-bpe_amd/lib
AB_REPS=2 AB_ROUNDS=2 timeout -k 10 700 python -u tools/ab_libs.py $L/base/libgpubpe.so $L/libgpubpe.so $L/spread/libgpubpe.so "$L/libgpubpe.so:GBPE_DEBUG=gused=70,glive=55" -- en1g c2 code1g > $O/ab.txt 2>&1 || { echo ABFAIL; tail -30 $O/ab.txt; exit 1; }
tail -12 $O/ab.txt
GBPE_DEBUG=poison=1 timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_poison.txt 2>&1 || { echo SUITEFAIL; tail -30 $O/gpu_tests_poison.txt; exit 1; }
tail -2 $O/gpu_tests_poison.txt
