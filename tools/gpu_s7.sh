# Session-7 diagnostic (one GPU call): where the lexicon build's time goes — the
# first en1g step under the kernel trace with the current library and three
# diagnostic builds (lxd1: k_lx_hash without its global-table flush; lxd2: hashing
# only; lxd3: k_lx_occ without its symbol check).  Results of lxd1/2 are not
# usable builds (the lexicon is abandoned); only the kernel times count.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s7
mkdir -p $O
L=$PWD/gpu-bpe_amd/lib
for v in pre lxd1 lxd2 lxd3; do
  lib=$L/$v/libgpubpe.so
  GBPE_LIB=$lib EXPLORE_MAX_STEPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lx_$v -o run -- python3 tools/explore_1g.py en1g > $O/lx_$v.log 2>&1 || { echo FAIL $v; tail -20 $O/lx_$v.log; exit 1; }
  f=$(find /tmp/lx_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v" >> $O/lx_stats.txt
  grep -E "k_lx|k_symbols|k_count_bytes" $f >> $O/lx_stats.txt
done
cat $O/lx_stats.txt
