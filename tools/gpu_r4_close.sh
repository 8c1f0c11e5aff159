# Closing checks (one GPU call): the whole -m gpu suite, smoke(), then the
# round-4 rocprof kernel stats and k_body PMC traffic of one en1g run
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4z
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo SUITEFAIL; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.txt; exit 1; }
tail -3 $O/smoke.txt
GRAFT_REPO_ROOT=$PWD bash tools/profile_r4.sh && ls gpurun_out/r4prof
