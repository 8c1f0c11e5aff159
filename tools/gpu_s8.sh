# Session-8 check (one GPU call): the lexicon build with plain-load word-table
# probes (flush adds last), the occurrence check against the entries' compact
# copy, and no tile recount — the first en1g step under the kernel trace (lib/pre
# against this tree), an A/B of whole runs (merges checked against the fixtures),
# then the GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s8
mkdir -p $O
L=$PWD/gpu-bpe_amd/lib
for v in pre new; do
  lib=$L/$v/libgpubpe.so; [ $v = new ] && lib=$L/libgpubpe.so
  GBPE_LIB=$lib EXPLORE_MAX_STEPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lx_$v -o run -- python3 tools/explore_1g.py en1g > $O/lx_$v.log 2>&1 || { echo FAIL $v; tail -20 $O/lx_$v.log; exit 1; }
  f=$(find /tmp/lx_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v" >> $O/lx_stats.txt
  grep -E "k_lx|k_symbols|k_count_bytes" $f >> $O/lx_stats.txt
done
AB_REPS=2 AB_ROUNDS=2 timeout -k 10 600 python -u tools/ab_libs.py $L/pre/libgpubpe.so $L/libgpubpe.so -- en1g c2 code1g > $O/ab.txt 2>&1 || { echo ABFAIL; tail -30 $O/ab.txt; exit 1; }
tail -6 $O/ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo SUITEFAIL; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
