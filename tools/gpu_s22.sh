# Session-22 check (one GPU call): the GPU suite with the round-5 k_body grid
# (one workgroup per bitmap word, 2-4 per word for rows of few words).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s22
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo SUITEFAIL; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
