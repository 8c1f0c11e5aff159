# One GPU call: late-loop parity first (stops on failure), then A/B, phase stamps,
# the whole GPU suite and the bench.  Every step has its own time limit.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_gpu_full.py -k "c1 or c2" -x -v --timeout 200 --timeout-method thread > $O/t1.txt 2>&1 || { echo T1FAIL; tail -30 $O/t1.txt; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_parity.py tests/test_gpu_resume.py -x -v --timeout 200 --timeout-method thread > $O/t2.txt 2>&1 || { echo T2FAIL; tail -30 $O/t2.txt; exit 1; }
echo tests-ok
AB_REPS=1 AB_ROUNDS=1 timeout -k 10 240 python -u tools/ab_libs.py gpu-bpe_amd/lib/libgpubpe.so:GBPE_DEBUG=late=0 gpu-bpe_amd/lib/libgpubpe.so -- c2 en1g > $O/ab.txt 2>&1 || { echo ABFAIL; tail -20 $O/ab.txt; exit 1; }
tail -4 $O/ab.txt
GBPE_LIB=$PWD/gpu-bpe_amd/lib/kt/libgpubpe.so GBPE_KTRACE_OUT=/tmp/ktl AB_REPS=1 AB_ROUNDS=1 timeout -k 10 200 python -u tools/ab_libs.py gpu-bpe_amd/lib/kt/libgpubpe.so -- en1g > $O/kt.txt 2>&1 && f=$(ls -t /tmp/ktl.* | head -1) && python tools/ktrace_late.py $f > $O/ktrace_late.txt
cat $O/ktrace_late.txt
[ -n "$SKIP_SUITE" ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/suite.txt 2>&1 || { echo SUITEFAIL; tail -30 $O/suite.txt; exit 1; }
tail -2 $O/suite.txt
