# Session-28 check (one GPU call): zone segments of 8K symbols (1024 threads x 8)
# for zones up to 512K (GBPE_DEBUG seg8 = 1, the default now; 0 = 16K segments):
# A/B with the merges checked against the fixtures, the phase stamps, the suite.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s28
mkdir -p $O
L=gpu-bpe_amd/lib
AB_REPS=2 AB_ROUNDS=2 timeout -k 10 700 python -u tools/ab_libs.py "$L/libgpubpe.so:GBPE_DEBUG=seg8=0" "$L/libgpubpe.so" -- en1g c2 code1g ml1g64k > $O/ab.txt 2>&1 || { echo ABFAIL; tail -30 $O/ab.txt; exit 1; }
grep -E "^(en1g|c2|code1g|ml1g64k) " $O/ab.txt
GBPE_LIB=$PWD/$L/kt/libgpubpe.so GBPE_KTRACE_OUT=/tmp/kt_en1g timeout -k 10 300 python -u tools/explore_1g.py en1g > $O/kt_en1g.log 2>&1 || { echo KTFAIL; tail -20 $O/kt_en1g.log; exit 1; }
f=$(ls -t /tmp/kt_en1g.* | head -1)
python tools/ktrace_show.py $f > $O/ktrace_en1g.txt
cat $O/ktrace_en1g.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo SUITEFAIL; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
